"""configs[3] timing: n = 5, 64 clients per process, 100 % conflicts, through
fx_batch_run_tiered and fx_batch_run_cut, against the oracle."""
import sys
import time

sys.path.insert(0, ".")
import numpy as np

from fantoch_amd import _lib
from fantoch_amd import device as fd
from fantoch_amd import streams as fs
from oracle import oracle_lib as O

cmds = int(sys.argv[1]) if len(sys.argv) > 1 else 64000
p = fs.synth_params(seed=3, instances=1, n=5, cmds=cmds, window=320, cycle_pct=30, conflicts=(100,), clients=64)
planes = fs.synth_host(p)
print("streams", planes.S, "steps", planes.steps, flush=True)
t = time.time()
o_order, o_rel, o_nexec, o_err = O.batch_execute(planes, threads=5)
print("oracle %.3f s" % (time.time() - t), flush=True)
for cut in (True, False):
    fd.run_batch(planes, cut=cut, metrics=False)
    t = time.time()
    res = fd.run_batch(planes, cut=cut, metrics=False)
    dt = time.time() - t
    same = np.array_equal(res.nexec, o_nexec) and np.array_equal(res.order, o_order) or None
    rows = np.concatenate([_lib.index(np.arange(planes.steps), s, planes.steps) for s in range(planes.S)])
    same = bool(np.array_equal(res.nexec, o_nexec) and np.array_equal(res.order[rows], o_order[rows]) and
                np.array_equal(res.release[rows], o_rel[rows]))
    extra = ""
    if cut:
        st = res.cut_stats
        extra = "segments %d longest %d whole %d failed %d tiers %s" % (st.segments, st.max_segment, st.whole_streams,
                                                                       st.failed_streams, list(st.tier_counts)[:9])
    else:
        extra = "tiers %s" % res.tier_counts
    print("%s %.3f s (incl. copies) identical %s %s" % ("cut" if cut else "tiered", dt, same, extra), flush=True)
