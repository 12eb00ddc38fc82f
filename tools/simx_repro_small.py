"""The intermittent k_simx failure appears in small launches (the parity
tests' one or two instances), not in launches of hundreds of copies
(tools/simx_repro.py).  This runs the tests' own small launches many times
with the event-log build (FX_LIB=fantoch_amd/build_evlog/...) and, for every
instance that differs from its first good run, prints the first event at
which its log differs and the events around it."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from fantoch_amd import _lib  # noqa: E402
from fantoch_amd import sim as S  # noqa: E402
import test_poison_all as T  # noqa: E402
from test_sim_large import planet  # noqa: E402
from simx_repro import fmt  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cases = sys.argv[2].split(",") if len(sys.argv) > 2 else ["sim_epaxos_5_2", "config3_epaxos", "sim_atlas_5_2"]
EV = 170_000
good = {}
bad = 0
for rep in range(reps):
    for case in cases:
        specs = T._SIM_CASES[case]()
        C = specs[0].clients_per_region * specs[0].num_client_regions
        lat_cap = (4 * EV + C - 1) // C
        for fill in list(T.FILLS) + [None]:
            res = S.run(specs, planet(), large=True, lat_cap=lat_cap,
                        before_launch=T.poisoner(*fill) if fill else None)
            for i in range(len(specs)):
                key = (case, i)
                row = (int(res.err[i]), res.events(i), res.trace(i), res.end_ms(i),
                       int(res.stats[i, _lib.FX_SIM_STAT_ERR_SITE]))
                log = res.latencies(i).reshape(-1)[:4 * EV].reshape(-1, 4).copy()
                if row[0] == 0 and key not in good:
                    good[key] = (row, log)
                    continue
                if key in good and row == good[key][0]:
                    continue
                bad += 1
                print("rep %d %s fill %s instance %d: %s" % (rep, case, fill, i, row), flush=True)
                if key not in good:
                    continue
                glog = good[key][1]
                diff = np.nonzero(np.any(glog != log, axis=1))[0]
                if not len(diff):
                    print("  logs equal over the logged events", flush=True)
                    continue
                k = int(diff[0])
                print("  first differs at event %d (good run: %s)" % (k, good[key][0]), flush=True)
                for j in range(max(0, k - 8), min(len(glog), k + 3)):
                    print("    %6d good %s" % (j, fmt(glog[j])), flush=True)
                    if j >= k - 1:
                        print("    %6d bad  %s" % (j, fmt(log[j])), flush=True)
    print("rep %d done, bad %d" % (rep, bad), flush=True)
sys.exit(1 if bad else 0)
