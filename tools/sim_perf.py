"""Quick GPU simulator timing: EPaxos n=5 (configs[1] shape), seeds x conflict rates."""
import argparse
import sys
import time

sys.path.insert(0, ".")
import numpy as np

from fantoch_amd import sim as S

ap = argparse.ArgumentParser()
ap.add_argument("--seeds", type=int, default=256)
ap.add_argument("--cmds", type=int, default=1000)
ap.add_argument("--protocol", type=int, default=S.EPAXOS)
ap.add_argument("--n", type=int, default=5)
ap.add_argument("--f", type=int, default=2)
ap.add_argument("--gc", type=int, default=10)
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
pl = S.Planet()
regs = pl.ids(S.GCP5[:a.n])
specs = [S.spec(a.protocol, a.n, a.f, regs, regs, commands_per_client=a.cmds, conflict_rate=c,
                gc_interval_ms=a.gc, seed=20250213, instance=i)
         for i, c in enumerate([0, 2, 10, 50, 100] * a.seeds)]
for r in range(a.reps):
    t = time.time()
    res = S.run(specs, pl, lat_cap=0)
    dt = time.time() - t
    ev = res.stats[:, 24].sum()
    ex = res.executed_len.sum()
    print("instances %d  %.3f s  events %.3g (%.3g/s)  executed %.3g (%.3g cmds/s)  errors %d" %
          (len(specs), dt, ev, ev / dt, ex, ex / dt, int((res.err != 0).sum())), flush=True)
