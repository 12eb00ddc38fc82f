"""Device-side batch execution through the C-ABI (fx_dev_* plumbing, no torch needed).

`run_batch(planes)` uploads a host `Planes` batch, runs the GPU executor
(fx_batch_run_tiered: tier 0 for every stream, capacity reruns at tiers 1/2)
and the metrics pass, and returns host copies of the outputs.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check


class DeviceBuffer:
    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(_lib.load().fx_dev_alloc(ctypes.byref(p), max(self.nbytes, 16)), "fx_dev_alloc")
        self.ptr = p.value

    def upload(self, arr, stream=None):
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        check(_lib.load().fx_dev_h2d(self.ptr, arr.ctypes.data, arr.nbytes, stream), "fx_dev_h2d")

    def download(self, dtype, count, stream=None):
        out = np.empty(count, dtype)
        check(_lib.load().fx_dev_d2h(out.ctypes.data, self.ptr, out.nbytes, stream), "fx_dev_d2h")
        check(_lib.load().fx_dev_synchronize(stream), "fx_dev_synchronize")
        return out

    def zero(self, stream=None):
        check(_lib.load().fx_dev_memset(self.ptr, 0, self.nbytes, stream), "fx_dev_memset")

    def fill_bytes(self, value, stream=None):
        check(_lib.load().fx_dev_memset(self.ptr, value, self.nbytes, stream), "fx_dev_memset")

    def free(self):
        if self.ptr:
            _lib.load().fx_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def device_count():
    return _lib.load().fx_device_count()


class BatchResult:
    def __init__(self, order, release, nexec, err, chain, delay, tier_counts, status, cut_stats=None):
        self.order = order
        self.release = release
        self.nexec = nexec
        self.err = err
        self.chain = chain
        self.delay = delay
        self.tier_counts = tier_counts
        self.status = status
        self.cut_stats = cut_stats


def run_batch(planes, execute_at_commit=False, nbins_chain=64, nbins_delay=4096, tiered=True,
              tier=None, init_frontier=None, metrics=True, cut=False, before_launch=None):
    """Runs a host batch on the GPU; returns host outputs (BatchResult).

    cut: fx_batch_run_cut (quiescent-cut decomposition, for huge streams);
    tiered: fx_batch_run_tiered starting at `tier` (None = FX_TIER_DEFAULT);
    otherwise one fx_batch_execute launch at `tier` (None = FX_TIER_DEFAULT).
    before_launch(stream): called with the launch's stream (None = the null
    stream) once the inputs are on the device, right before the first
    executor launch (tests: register poisoning, tests/test_poison_all.py)."""
    lib = _lib.load()
    S, steps, pw = planes.S, planes.steps, planes.plane
    bufs = {}
    for name, arr in (("dot", planes.dot), ("hdr", planes.hdr), ("deps", planes.deps)):
        b = DeviceBuffer(arr.nbytes)
        b.upload(arr)
        bufs[name] = b
    lengths = None
    if planes.lengths is not None:
        lengths = DeviceBuffer(S * 4)
        lengths.upload(np.asarray(planes.lengths, np.uint32))
    order = DeviceBuffer(pw * 4)
    release = DeviceBuffer(pw * 4)
    release.fill_bytes(0xFF)  # rows a stream never reaches (an error) stay FX_RELEASE_NONE
    nexec = DeviceBuffer(S * 4)
    err = DeviceBuffer(S * 4)
    # every driver writes every stream's count and status: a sentinel shows any it skipped
    nexec.fill_bytes(0xAB)
    err.fill_bytes(0xAB)
    inb = _lib.StreamBatch(bufs["dot"].ptr, bufs["hdr"].ptr, bufs["deps"].ptr,
                           lengths.ptr if lengths else None, S, steps, planes.dmax, planes.n)
    outb = _lib.OrderBatch(order.ptr, release.ptr, nexec.ptr, err.ptr)
    flags = _lib.FX_FLAG_EXECUTE_AT_COMMIT if execute_at_commit else 0
    tier_counts = (ctypes.c_uint32 * _lib.FX_NUM_TIERS)()
    cut_stats = None
    if before_launch is not None:
        before_launch(None)
    if cut:
        cut_stats = _lib.CutStats()
        status = lib.fx_batch_run_cut(ctypes.byref(inb), ctypes.byref(outb), flags, None,
                                      ctypes.byref(cut_stats))
    elif tiered and init_frontier is None:
        tflags = flags | (_lib.first_tier_flag(tier) if tier is not None else 0)
        status = lib.fx_batch_run_tiered(ctypes.byref(inb), ctypes.byref(outb), tflags, None, tier_counts)
    else:
        tier = _lib.FX_TIER_DEFAULT if tier is None else tier
        front = None
        if init_frontier is not None:
            front = DeviceBuffer(S * 8 * 4)
            front.upload(np.asarray(init_frontier, np.uint32).reshape(S, 8))
        state = None
        if tier in (2, _lib.FX_TIER_SPLIT, _lib.FX_TIER_WIDE_HBM):  # HBM-resident tier's working memory / split scratch
            state = DeviceBuffer(lib.fx_batch_state_bytes(tier, planes.n, S))
        status = lib.fx_batch_execute(ctypes.byref(inb), ctypes.byref(outb), tier, None, S,
                                      state.ptr if state else None, 0, steps,
                                      flags | _lib.FX_FLAG_INIT, front.ptr if front else None, None)
        check(status, "fx_batch_execute")
        check(lib.fx_dev_synchronize(None), "sync")
        tier_counts[tier] = S
    chain = delay = None
    if metrics and not execute_at_commit:
        hc = DeviceBuffer(nbins_chain * 8)
        hd = DeviceBuffer(nbins_delay * 8)
        hc.zero()
        hd.zero()
        hb = _lib.HistBatch(hc.ptr, nbins_chain, hd.ptr, nbins_delay)
        check(lib.fx_batch_metrics(ctypes.byref(inb), ctypes.byref(outb), ctypes.byref(hb), None),
              "fx_batch_metrics")
        chain = hc.download(np.uint64, nbins_chain)
        delay = hd.download(np.uint64, nbins_delay)
    res = BatchResult(order.download(np.uint32, pw), release.download(np.uint32, pw),
                      nexec.download(np.uint32, S), err.download(np.uint32, S),
                      chain, delay, list(tier_counts), status, cut_stats)
    return res


def run_pred(planes, clock_lo, clock_hi, ndeps=None, execute_at_commit=False, tier=None, nbins_delay=4096,
             before_launch=None):
    """PredecessorsExecutor over a host batch with packed Caesar clock planes:
    fx_pred_run (tier None: the escalation chain) or one fx_pred_execute at
    `tier` (FX_PRED_TIER_*); returns a BatchResult (delay histogram from
    fx_batch_metrics)."""
    lib = _lib.load()
    S, steps, pw = planes.S, planes.steps, planes.plane
    bufs = {}
    for name, arr in (("dot", planes.dot), ("hdr", planes.hdr), ("deps", planes.deps),
                      ("clo", np.asarray(clock_lo, np.uint32)), ("chi", np.asarray(clock_hi, np.uint32)),
                      ("nd", np.asarray(ndeps if ndeps is not None else [0], np.uint32))):
        b = DeviceBuffer(arr.nbytes)
        b.upload(arr)
        bufs[name] = b
    lengths = None
    if planes.lengths is not None:
        lengths = DeviceBuffer(S * 4)
        lengths.upload(np.asarray(planes.lengths, np.uint32))
    order, release = DeviceBuffer(pw * 4), DeviceBuffer(pw * 4)
    release.fill_bytes(0xFF)
    nexec, err = DeviceBuffer(S * 4), DeviceBuffer(S * 4)
    base = _lib.StreamBatch(bufs["dot"].ptr, bufs["hdr"].ptr, bufs["deps"].ptr, lengths.ptr if lengths else None,
                            S, steps, planes.dmax, planes.n)
    inb = _lib.PredBatch(base, bufs["clo"].ptr, bufs["chi"].ptr, bufs["nd"].ptr if ndeps is not None else None)
    outb = _lib.OrderBatch(order.ptr, release.ptr, nexec.ptr, err.ptr)
    flags = _lib.FX_FLAG_EXECUTE_AT_COMMIT if execute_at_commit else 0
    reruns = ctypes.c_uint32()
    if before_launch is not None:
        before_launch(None)
    if tier is not None:
        state = DeviceBuffer(lib.fx_pred_state_bytes(planes.n, planes.dmax, S)) if tier == _lib.FX_PRED_TIER_HBM \
            else None
        status = lib.fx_pred_execute(ctypes.byref(inb), ctypes.byref(outb), None, S, tier,
                                     state.ptr if state else None, flags, None)
        check(lib.fx_dev_synchronize(None), "sync")
    else:
        status = lib.fx_pred_run(ctypes.byref(inb), ctypes.byref(outb), flags, None, ctypes.byref(reruns))
    hc, hd = DeviceBuffer(64 * 8), DeviceBuffer(nbins_delay * 8)
    hc.zero()
    hd.zero()
    hb = _lib.HistBatch(hc.ptr, 64, hd.ptr, nbins_delay)
    check(lib.fx_batch_metrics(ctypes.byref(base), ctypes.byref(outb), ctypes.byref(hb), None), "fx_batch_metrics")
    res = BatchResult(order.download(np.uint32, pw), release.download(np.uint32, pw), nexec.download(np.uint32, S),
                      err.download(np.uint32, S), hc.download(np.uint64, 64), hd.download(np.uint64, nbins_delay),
                      [], status)
    res.reruns = int(reruns.value)
    return res
