"""Reproduction of k_sim's schedule-dependent FX_ERR_SIM_LATE (round 3: the
iterative-ILP build of sim_wave.hip stops test_region_subsets_n7 / test_no_gc
instances, only after other launches ran on the device).

A large configs[1]-shaped batch first leaves k_sim state on every CU; then each
probe instance runs as `copies` identical copies (same spec, so the same
simulation), landing on many CUs with different leftover state.  Every copy
must end with the same (err, events, trace, end); the script prints, per probe,
how many copies failed or disagree with the majority.  With --max-events K the
runs stop after K events, so the first event at which copies diverge can be
bracketed.  Product library or FX_LIB=...; no oracle involved."""
import argparse
import itertools
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fantoch_amd import _lib  # noqa: E402
from fantoch_amd import sim as S  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--copies", type=int, default=1024)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--max-events", type=str, default="0", help="comma list of event bounds (0 = none)")
ap.add_argument("--probes", type=str, default="n7_0,n7_2,n7_3,nogc_2")
ap.add_argument("--bisect", type=int, default=0, help="bisect the first diverging event below this bound")
ap.add_argument("--poison", type=str, default="", help="after the dirtying batch, poison registers: "
                "comma list of mode:tag runs (mode 1 vector, 2 scalar, 3 both; tag 0-255)")
args = ap.parse_args()

pl = S.Planet()
regs5 = pl.ids(S.GCP5[:5])
dirty = [S.spec(S.EPAXOS, 5, 2, regs5, regs5, commands_per_client=100, conflict_rate=c, seed=77, instance=i)
         for i, c in enumerate([0, 2, 10, 50, 100] * 820)]
subsets = list(itertools.combinations(range(pl.R), 7))[::9973][:12]
probes = {}
for i, sub in enumerate(subsets):
    probes["n7_%d" % i] = S.spec(S.ATLAS, 7, 1 + (i % 2), list(sub), list(sub), commands_per_client=60,
                                 conflict_rate=10, seed=5, instance=i)
for i in range(4):
    probes["nogc_%d" % i] = S.spec(S.EPAXOS, 5, 2, regs5, regs5, commands_per_client=80, conflict_rate=50,
                                   gc_interval_ms=0, seed=4, instance=i)
names = args.probes.split(",")
PLIB = None
if args.poison:
    import ctypes
    PLIB = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "tests", "poison", "build", "libpoison.so"))
    PLIB.fx_dbg_poison_mode.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]


def groups(name, me):
    S.run(dirty, pl)
    res = S.run([probes[name]] * args.copies, pl, max_events=me, tiered=False)
    return Counter((int(res.err[i]), res.events(i), res.trace(i), res.end_ms(i),
                    int(res.stats[i, _lib.FX_SIM_STAT_SEQ])) for i in range(args.copies))


if args.bisect:
    for name in names:
        lo, hi = 0, args.bisect  # copies agree after lo events, disagree after hi
        while hi - lo > 1:
            mid = (lo + hi) // 2
            g = groups(name, mid)
            print("%s max_events %d: %d groups %s" % (name, mid, len(g), g.most_common(3)), flush=True)
            if len(g) > 1:
                hi = mid
            else:
                lo = mid
        print("%s: copies agree after %d events, differ after %d" % (name, lo, hi), flush=True)
        print("  at %d: %s" % (hi, groups(name, hi).most_common(3)), flush=True)
    sys.exit(0)
runs = [(None, None)] + [tuple(int(v) for v in x.split(":")) for x in args.poison.split(",") if x]
for me in [int(x) for x in args.max_events.split(",")]:
  for mode, tag in runs:
    for rnd in range(args.rounds):
        for name in names:
            S.run(dirty, pl)
            before = None
            if mode is not None:
                before = lambda st, m=mode, t=tag: PLIB.fx_dbg_poison_mode(t, 4096, m, st)
            res = S.run([probes[name]] * args.copies, pl, max_events=me, tiered=False, before_launch=before)
            rows = [(int(res.err[i]), res.events(i), res.trace(i), res.end_ms(i),
                     int(res.stats[i, _lib.FX_SIM_STAT_ERR_SITE])) for i in range(args.copies)]
            cnt = Counter(rows)
            major, nmaj = cnt.most_common(1)[0]
            odd = sorted(((r, c) for r, c in cnt.items() if r != major), key=lambda x: -x[1])[:4]
            print("poison %s:%s " % (mode, tag) + "max_events %d round %d %s: majority %s x%d; others %d %s" % (
                me, rnd, name, major, nmaj, args.copies - nmaj, odd), flush=True)
