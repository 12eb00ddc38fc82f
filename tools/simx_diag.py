"""k_simx's intermittent FX_ERR_SIM_LATE: runs the small
poisoned launches of tests/test_poison_all.py::test_poisoned_k_simx many
times against the diagnostics build (FX_LIB=fantoch_amd/build_diag/...,
built with -DFX_SIMX_DIAG) and prints, for every failed instance, the state
the kernel snapshotted at its first failure (stats slots 0..15):

  0 site line | 0xD1A6 << 32     1 now | events << 32     2 seq | nfree << 32
  3 xp | rtop << 8 | nfrm << 16 | event info << 32        4 event arg | key hi << 32
  broken event tree (pop):  8 group minimum (hi | lo << 32)   9 group | lane << 16 | k << 32
                            10 leaves' minimum   11 NONE leaves | matches << 8 ...
                            12 mismatching groups | first << 32   13 its lane minimum
                            14 its leaves' minimum   15 junk lanes | lane << 16 | value << 32
  slot gone (handlers):     8 dot | p << 32   9 slot | source's last seq << 32
                            10 tag | masks << 32   11 cnt | client << 32
                            12 R_PST | R_WAIT << 32   13 copy's tag | copy slot << 32
  SCC member not pending:   8 root | tsp << 32   9 ctp | cv << 32   10 member | status << 32
                            11 its tag | masks << 32   12 R_TL | R_MARK << 32   13 index | count << 32
  a canary changed:         16 canaries a | b << 32   17 canary c | events << 32 (words the
                            simulation never writes, set at the start; checked after every event)
No oracle: a failure is the signal."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from fantoch_amd import _lib  # noqa: E402
from fantoch_amd import sim as S  # noqa: E402
import test_poison_all as T  # noqa: E402
from test_sim_large import planet  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
cases = sys.argv[2].split(",") if len(sys.argv) > 2 else ["config3_epaxos", "sim_epaxos_5_2", "sim_atlas_5_2"]
fills = list(T.FILLS) + [None]
arena_fill = os.environ.get("SIMX_DIAG_FILL") == "1"  # the arena starts as 0xA5 bytes (FX_SIM_FLAG_ARENA_FILL)
fails = 0
launches = 0
for rep in range(reps):
    for case in cases:
        specs = T._SIM_CASES[case]()
        for fill in fills:
            res = S.run(specs, planet(), large=True, before_launch=T.poisoner(*fill) if fill else None,
                        arena_fill=arena_fill)
            launches += 1
            for i, e in enumerate(res.err):
                if not e:
                    continue
                fails += 1
                st = [int(x) for x in res.stats[i, :18]]
                print("rep %d %s fill %s: instance %d err %d site %d events %d" % (
                    rep, case, fill, i, int(e), int(res.stats[i, _lib.FX_SIM_STAT_ERR_SITE]), res.events(i)))
                print("   " + " ".join("%d:%016x" % (k, v) for k, v in enumerate(st) if v), flush=True)
    print("rep %d done, %d launches, failures so far %d" % (rep, launches, fails), flush=True)
sys.exit(1 if fails else 0)
