"""Cycles per phase of the large-instance simulator (sim_big.hip) from the
FX_SIM_PROFILE build (make prof), on BASELINE configs[3]'s shape.

usage: FX_LIB=fantoch_amd/build_prof/libfantoch_amd.so python tools/simx_phase.py [--seeds N] [--cmds M]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from fantoch_amd import sim as S

ap = argparse.ArgumentParser()
ap.add_argument("--seeds", type=int, default=512)
ap.add_argument("--cmds", type=int, default=30)
ap.add_argument("--clients", type=int, default=64)
ap.add_argument("--out", type=str, default=None)
a = ap.parse_args()
assert os.environ.get("FX_LIB"), "set FX_LIB to the profile build"
pl = S.Planet()
regs = sorted(pl.ids(S.GCP5))
specs = [S.spec(S.ATLAS if i % 2 == 0 else S.EPAXOS, 5, 1 if i % 2 == 0 else 2, regs, regs,
                clients_per_region=a.clients, commands_per_client=a.cmds, conflict_rate=100,
                seed=20250213, instance=i) for i in range(a.seeds)]
res = S.run(specs, pl, lat_cap=0)
st = res.stats.astype(np.float64)
names = ["pop", "event (all)", "x_add", "find_scc", "check_pending", "sort", "emit", "handlers", "send",
         "gc", "client"]  # slot 11 is a count (cached first finds)
counts = {11: "cached first finds", 16: "dfs edges", 17: "dfs recursions", 18: "x_add calls", 19: "find_scc calls", 20: "waiters",
          21: "fast-path adds", 22: "events", 23: "sends"}
ev = st[:, 22].sum()
tot = st[:, 0].sum() + st[:, 1].sum()
out = {"events": ev, "cycles_per_event": tot / ev}
print("events %d, cycles/event %.0f" % (ev, tot / ev))
for i, nm in enumerate(names):
    print("%-16s %9.0f cycles/event  %5.1f %%" % (nm, st[:, i].sum() / ev, 100 * st[:, i].sum() / tot))
    out[nm] = st[:, i].sum() / ev
for i, nm in ((12, "ready results"), (13, "handler row load"), (14, "push_event"), (15, "dep states (LX)")):
    print("%-16s %9.0f cycles/event  %5.1f %%" % (nm, st[:, i].sum() / ev, 100 * st[:, i].sum() / tot))
    out[nm] = st[:, i].sum() / ev
for k, nm in counts.items():
    print("%-16s %12.0f per instance  %.3f per event" % (nm, st[:, k].sum() / len(specs), st[:, k].sum() / ev))
    out[nm] = st[:, k].sum() / len(specs)
if a.out:
    json.dump(out, open(a.out, "w"), indent=1)
