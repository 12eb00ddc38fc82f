"""Error census of a placements batch (debug): err codes per (n, f) group."""
import collections
import sys

sys.path.insert(0, ".")
import numpy as np

import bench_placements as BP
from fantoch_amd import sim as S

pl = S.Planet()
allp = BP.enumerate_placements(pl.R)
for n, f in BP.GROUPS:
    idx = [i for i, p in enumerate(allp) if p[0] == n and p[1] == f][::97][:400]
    specs = [S.spec(S.ATLAS, n, f, list(allp[g][2]), list(allp[g][2]), commands_per_client=100, conflict_rate=2,
                    seed=20250213, instance=g) for g in idx]
    res = S.run(specs, pl, tiered=False)
    c = collections.Counter(int(e) for e in res.err)
    sites = collections.Counter(int(res.stats[i, 30]) for i, e in enumerate(res.err) if e)
    print(n, f, dict(c), "sites", dict(sites), flush=True)
    bad = [i for i, e in enumerate(res.err) if e]
    for i in bad[:3]:
        print("   ", [pl.regions[r] for r in allp[idx[i]][2]], int(res.err[i]), "end", res.end_ms(i), "events",
              res.events(i), "site", int(res.stats[i, 30]))
