"""Error sites of the configs[2]-shaped n = 7 instances of
tests/test_sim_gpu.py::test_region_subsets_n7 on the in-tree library or
FX_LIB (diagnostics for scheduler variants of k_sim)."""
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fantoch_amd import _lib
from fantoch_amd import sim as S

pl = S.Planet()
subsets = list(itertools.combinations(range(pl.R), 7))[::9973][:12]
specs = [S.spec(S.ATLAS, 7, 1 + (i % 2), list(sub), list(sub), commands_per_client=60,
                conflict_rate=10, seed=5, instance=i) for i, sub in enumerate(subsets)]
# the launches test_sim_gpu.py makes before it (a failure that needs them
# points at state a kernel reads before writing)
regs5 = pl.ids(S.GCP5[:5])
pre = [[S.spec(S.ATLAS, 3, 1, pl.ids(S.GCP5[:3]), pl.ids(S.GCP5[:3]), commands_per_client=1000, conflict_rate=2,
               seed=1)]]
for proto, n, f in ((S.EPAXOS, 5, 2), (S.ATLAS, 5, 1), (S.ATLAS, 5, 2)):
    pre.append([S.spec(proto, n, f, regs5, regs5, commands_per_client=100, conflict_rate=c, seed=77, instance=i)
                for i, c in enumerate([0, 2, 10, 50, 100] * 4)])
if "--pre" in sys.argv:
    for ps in pre:
        r = S.run(ps, pl)
        print("pre", len(ps), "err", sorted(set(int(e) for e in r.err)), flush=True)
for generic in (False, True):
    res = S.run(specs, pl, generic=generic)
    print("generic" if generic else "fixed  ", "err", [int(e) for e in res.err],
          "site", [int(res.stats[i, _lib.FX_SIM_STAT_ERR_SITE]) for i in range(len(specs))], flush=True)
