"""Reproduction of k_simx's intermittent FX_ERR_SIM_LATE under register
poisoning (tests/test_poison_all.py; the round-4 build shows it too).

Each probe instance runs as `copies` identical copies in one launch (same spec,
so the same simulation) after a dirtying batch and a register fill; every copy
must end with the same (err, events, trace, end).  With the event-log build
(make fvariant V=evlog F=sim_big D="-DFX_SIMX_EVLOG ..."; FX_LIB=...) each
copy also logs every event (key, info, argument, trace hash after it), and for
every copy that differs from the majority the script prints the first event
at which its log differs and the events around it.  No oracle involved."""
import argparse
import ctypes
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from fantoch_amd import _lib  # noqa: E402
from fantoch_amd import sim as S  # noqa: E402
from test_sim_large import sim_test_specs  # noqa: E402

KIND = {0: "MCollect", 1: "MCollectAck", 2: "MCommit", 3: "MConsensus", 4: "MConsensusAck", 6: "MGC",
        8: "MStore", 9: "MStoreAck", 10: "MCommitB", 12: "Submit", 13: "ToClient", 14: "GCtick", 15: "Notif"}


def fmt(ev):
    hi, info, arg, tr = (int(x) for x in ev)
    return "t=%d cls=%d %s from=%d to=%d arg=%#x trace=%08x" % (
        hi >> 8, (hi >> 6) & 3, KIND.get(info & 15, info & 15), (info >> 4) & 15, (info >> 8) & 15, arg, tr)



def main():
    global args
    ap = argparse.ArgumentParser()
    ap.add_argument("--copies", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--probes", type=str, default="sim_epaxos_5_2,config3_epaxos")
    ap.add_argument("--events", type=int, default=0, help="event-log capacity per copy (0: the probe's estimate)")
    ap.add_argument("--fills", type=str, default="1:90,4:0,1:195")
    args = ap.parse_args()

    pl = S.Planet()
    regs = sorted(pl.ids(S.GCP5))
    probes = {
        "sim_epaxos_5_2": (sim_test_specs(S.EPAXOS, 5, 2, seeds=(3,))[0], 130_000),
        "sim_atlas_5_2": (sim_test_specs(S.ATLAS, 5, 2, seeds=(3,))[0], 130_000),
        "config3_epaxos": (S.spec(S.EPAXOS, 5, 2, regs, regs, clients_per_region=64, commands_per_client=20,
                                  conflict_rate=100, seed=12, instance=0), 160_000),
    }
    dirty = sim_test_specs(S.ATLAS, 5, 2, seeds=tuple(range(40, 104)))
    PLIB = ctypes.CDLL(os.path.join(ROOT, "tests", "poison", "build", "libpoison.so"))
    PLIB.fx_dbg_poison_mode.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    fills = [tuple(int(v) for v in f.split(":")) for f in args.fills.split(",") if f]


    total_odd = 0
    for rnd in range(args.rounds):
        for name in args.probes.split(","):
            spec, est = probes[name]
            C = spec.clients_per_region * spec.num_client_regions
            ev = args.events or est
            lat_cap = (4 * ev + C - 1) // C
            for mode, tag in fills:
                S.run(dirty, pl, large=True)
                before = lambda st, m=mode, t=tag: PLIB.fx_dbg_poison_mode(t, 4096, m, st)
                res = S.run([spec] * args.copies, pl, large=True, tiered=False, lat_cap=lat_cap, before_launch=before)
                rows = [(int(res.err[i]), res.events(i), res.trace(i), res.end_ms(i),
                         int(res.stats[i, _lib.FX_SIM_STAT_ERR_SITE])) for i in range(args.copies)]
                cnt = Counter(rows)
                major, nmaj = cnt.most_common(1)[0]
                odd = [i for i, r in enumerate(rows) if r != major]
                total_odd += len(odd)
                print("round %d %s fill %d:%d: majority %s x%d; %d odd %s" % (
                    rnd, name, mode, tag, major, nmaj, len(odd), [rows[i] for i in odd[:4]]), flush=True)
                if not odd:
                    continue
                good = rows.index(major)
                glog = res.latencies(good).reshape(-1)[:4 * ev].reshape(-1, 4)
                for i in odd[:3]:
                    blog = res.latencies(i).reshape(-1)[:4 * ev].reshape(-1, 4)
                    diff = np.nonzero(np.any(glog != blog, axis=1))[0]
                    if not len(diff):
                        print("  copy %d: logs equal over the logged events" % i, flush=True)
                        continue
                    k = int(diff[0])
                    print("  copy %d first differs at event %d:" % (i, k), flush=True)
                    for j in range(max(0, k - 6), min(len(glog), k + 3)):
                        print("    %6d good %s" % (j, fmt(glog[j])), flush=True)
                        if j >= k - 1:
                            print("    %6d bad  %s" % (j, fmt(blog[j])), flush=True)
    print("odd copies in total: %d" % total_odd, flush=True)


if __name__ == "__main__":
    main()
