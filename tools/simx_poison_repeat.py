"""Runs the poisoned configs[3] k_simx cases of tests/test_poison_all.py a few
times in one process and prints any failed instance's error and source line
(an intermittent register or state read shows up as a failure site)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np

from fantoch_amd import _lib
from fantoch_amd import sim as S
import test_poison_all as T
from test_sim_large import assert_instance_parity, planet

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
cases = sys.argv[2].split(",") if len(sys.argv) > 2 else ["config3_atlas", "config3_epaxos", "sim_epaxos_5_2"]
fills = list(T.FILLS) + [None]  # None: no fill
fails = 0
for rep in range(reps):
    for case in cases:
        specs, orc = T._oracle_sim(case)
        for fill in fills:
            res = S.run(specs, planet(), large=True, before_launch=T.poisoner(*fill) if fill else None)
            for i, e in enumerate(res.err):
                if e:
                    fails += 1
                    print("rep %d %s fill %s: instance %d err %d site %d events %d end %d" % (
                        rep, case, fill, i, int(e), int(res.stats[i, _lib.FX_SIM_STAT_ERR_SITE]), res.events(i),
                        res.end_ms(i)), flush=True)
                else:
                    try:
                        assert_instance_parity(res, i, specs[i], orc[i])
                    except AssertionError as ex:
                        fails += 1
                        print("rep %d %s fill %s: instance %d differs: %s" % (rep, case, fill, i, ex), flush=True)
    print("rep %d done, failures so far %d" % (rep, fails), flush=True)
sys.exit(1 if fails else 0)
