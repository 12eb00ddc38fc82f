"""Cycles per simulator phase from the FX_SIM_PROFILE build (make prof).

usage: FX_LIB=fantoch_amd/build_prof/libfantoch_amd.so python tools/sim_phase.py [--seeds N] [--cmds M]
Prints, summed over instances, the shader-clock cycles (s_memtime ticks) spent
popping the next action, in each handler kind, in the executor, and in the
rest of the event, per event and per handler call."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from fantoch_amd import sim as S

ap = argparse.ArgumentParser()
ap.add_argument("--seeds", type=int, default=256)
ap.add_argument("--cmds", type=int, default=200)
ap.add_argument("--n", type=int, default=5)
ap.add_argument("--f", type=int, default=2)
ap.add_argument("--protocol", type=int, default=S.EPAXOS)
a = ap.parse_args()
assert os.environ.get("FX_LIB"), "set FX_LIB to the profile build"
pl = S.Planet()
regs = pl.ids(S.GCP5[:a.n])
specs = [S.spec(a.protocol, a.n, a.f, regs, regs, commands_per_client=a.cmds, conflict_rate=c,
                seed=20250213, instance=i) for i, c in enumerate([0, 2, 10, 50, 100] * a.seeds)]
res = S.run(specs, pl, lat_cap=0)
st = res.stats.astype(np.float64)
ev = st[:, 24].sum()
names = {0: "pop_min", 1: "run_event (all)", 2: "executor x_add", 3: "send_p", 4: "client R event", 5: "x_add load+check", 6: "note", 7: "run_handlers"}
kinds = ["MCollect", "MCollectAck", "MCommit", "MConsensus", "MConsensusAck", "x_add emit_one(fast)", "x_add x_store", "Submit"]
tot = st[:, 0].sum() + st[:, 1].sum()
print("events %d, cycles/event %.0f" % (ev, tot / ev))
for i in sorted(names):
    print("%-22s %8.0f cycles/event  %5.1f %%" % (names[i], st[:, i].sum() / ev, 100 * st[:, i].sum() / tot))
for k in range(8):
    c, n = st[:, 8 + k].sum(), st[:, 16 + k].sum()
    if n:
        print("  handler %-14s %8.0f cycles/call  %9d calls  %5.1f %%" % (kinds[k], c / n, n, 100 * c / tot))
# per conflict rate: cycles per instance and the executor's share
rates = np.array([0, 2, 10, 50, 100] * a.seeds)
for r in [0, 2, 10, 50, 100]:
    m = rates == r
    tr = st[m, 0].sum() + st[m, 1].sum()
    print("conflict %3d%%: %.3g cycles/instance, events/instance %.0f, executor %.1f %%, handlers %.1f %%, send_p %.1f %%"
          % (r, tr / m.sum(), st[m, 24].sum() / m.sum(), 100 * st[m, 2].sum() / tr,
             100 * st[m, 8:16].sum() / tr, 100 * st[m, 3].sum() / tr))
