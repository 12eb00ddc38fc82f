"""Statistics of the reduced dense histograms (Histogram, fantoch/src/metrics/histogram.rs).

The batched executor folds ChainSize / ExecutionDelay samples into dense bins
(k_metrics, all-reduced across ranks); this turns a dense count array into the
reference's `Histogram` statistics through the C-ABI: mean / stddev / cov / mdtm
(histogram.rs:61-110, 172-235, fx_hist_stats_compute) and percentiles
(histogram.rs:111-170, fx_hist_percentile).  The last bin holds every value
>= nbins - 1, so statistics are exact only when it is empty (`clamped` == 0).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check


def dense_stats(counts, percentiles=(0.5, 0.95, 0.99)):
    counts = np.ascontiguousarray(np.asarray(counts, dtype=np.uint64))
    nz = np.flatnonzero(counts)
    values = np.ascontiguousarray(nz.astype(np.uint64))
    cnts = np.ascontiguousarray(counts[nz])
    out = {"count": int(cnts.sum()), "clamped": int(counts[-1]) if len(counts) else 0}
    if not len(nz):
        return out
    u64p = ctypes.POINTER(ctypes.c_uint64)
    vp, cp = values.ctypes.data_as(u64p), cnts.ctypes.data_as(u64p)
    lib = _lib.load()
    st = _lib.HistStats()
    check(lib.fx_hist_stats_compute(vp, cp, len(nz), ctypes.byref(st)), "fx_hist_stats_compute")
    out.update(mean=st.mean, stddev=st.stddev, cov=st.cov, mdtm=st.mdtm, min=st.min, max=st.max)
    for p in percentiles:
        r = ctypes.c_double()
        check(lib.fx_hist_percentile(vp, cp, len(nz), p, ctypes.byref(r)), "fx_hist_percentile")
        out["p%g" % (p * 100)] = r.value
    return out
