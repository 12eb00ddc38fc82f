"""oracle/oracle_lib.py — TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/build/liboracle.so, the C++ restatement of the
reference's DependencyGraph (graph_oracle.cpp).  Only tests/, smoke() and
bench.py's cpu_baseline leg may use it, and only as the checker.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")
SRC = os.path.join(HERE, "graph_oracle.cpp")

_lib = None


def build():
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", LIB, SRC,
                           "-lpthread"])


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
            build()
        lib = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        u32 = ctypes.c_uint32
        u64 = ctypes.c_uint64
        P32 = ctypes.POINTER(ctypes.c_uint32)
        P64 = ctypes.POINTER(ctypes.c_uint64)
        lib.oracle_batch_execute.restype = ctypes.c_int
        lib.oracle_batch_execute.argtypes = [vp, vp, vp, u32, u32, u32, vp, u32, u32, vp, vp, vp,
                                             vp, vp, ctypes.c_int, vp, vp]
        lib.oracle_graph_new.restype = vp
        lib.oracle_graph_new.argtypes = [u32, u32]
        lib.oracle_graph_free.argtypes = [vp]
        lib.oracle_graph_handle_add.restype = ctypes.c_int
        lib.oracle_graph_handle_add.argtypes = [vp, u32, u64, P32, P64, u32, u64, u32]
        lib.oracle_graph_index_only.restype = ctypes.c_int
        lib.oracle_graph_index_only.argtypes = [vp, u32, u64, P32, P64, u32, u64, u32]
        lib.oracle_graph_set_executed.argtypes = [vp, u32, u64]
        lib.oracle_graph_find_scc.restype = ctypes.c_int
        lib.oracle_graph_find_scc.argtypes = [vp, u32, u64, ctypes.c_int, P32, P64, u32, P32, P64, P32]
        lib.oracle_graph_drain.restype = u32
        lib.oracle_graph_drain.argtypes = [vp, P32, P64, P32, ctypes.POINTER(ctypes.c_uint8), u32]
        lib.oracle_graph_pending.restype = u32
        lib.oracle_graph_pending.argtypes = [vp, P32, P64, P32, P64, u32]
        lib.oracle_graph_metrics.restype = u32
        lib.oracle_graph_metrics.argtypes = [vp, u32, P64, P64, u32]
        _lib = lib
    return _lib


def batch_execute(planes, execute_at_commit=False, init_frontier=None, threads=1, stats=False):
    """Runs every stream of a host `Planes` batch through the oracle.
    Returns (order, release, nexec, err) in the same plane layout as the GPU
    (+ (max_pending, max_window) per stream with stats=True)."""
    lib = load()
    pw = planes.plane
    order = np.zeros(pw, np.uint32)
    release = np.zeros(pw, np.uint32)
    nexec = np.zeros(planes.S, np.uint32)
    err = np.zeros(planes.S, np.uint32)
    lengths = None
    if planes.lengths is not None:
        lengths = np.ascontiguousarray(planes.lengths, np.uint32)
    front = None
    if init_frontier is not None:
        front = np.ascontiguousarray(init_frontier, np.uint32).reshape(planes.S, 8)
    mp = np.zeros(planes.S, np.uint32)
    mw = np.zeros(planes.S, np.uint32)
    lib.oracle_batch_execute(
        planes.dot.ctypes.data, planes.hdr.ctypes.data, planes.deps.ctypes.data, planes.S,
        planes.steps, planes.dmax, lengths.ctypes.data if lengths is not None else None,
        planes.n, 2 if execute_at_commit else 0,
        front.ctypes.data if front is not None else None, order.ctypes.data,
        release.ctypes.data, nexec.ctypes.data, err.ctypes.data, int(threads),
        mp.ctypes.data if stats else None, mw.ctypes.data if stats else None)
    if stats:
        return order, release, nexec, err, mp, mw
    return order, release, nexec, err


class Graph:
    """One DependencyGraph (graph/mod.rs:45-677), for the reference's unit-test shapes."""

    def __init__(self, process_id, n):
        self.lib = load()
        self.h = self.lib.oracle_graph_new(process_id, n)
        self.rec = 0

    def __del__(self):
        try:
            self.lib.oracle_graph_free(self.h)
        except Exception:
            pass

    def _deps(self, deps):
        deps = list(deps)
        src = (ctypes.c_uint32 * max(len(deps), 1))(*[d[0] for d in deps])
        seq = (ctypes.c_uint64 * max(len(deps), 1))(*[d[1] for d in deps])
        return src, seq, len(deps)

    def handle_add(self, dot, deps, t_ms=0):
        src, seq, nd = self._deps(deps)
        r = self.lib.oracle_graph_handle_add(self.h, dot[0], dot[1], src, seq, nd, t_ms, self.rec)
        self.rec += 1
        if r:
            raise RuntimeError("oracle handle_add failed (%d)" % r)

    def index_only(self, dot, deps, t_ms=0):
        src, seq, nd = self._deps(deps)
        r = self.lib.oracle_graph_index_only(self.h, dot[0], dot[1], src, seq, nd, t_ms, self.rec)
        self.rec += 1
        if r:
            raise RuntimeError("oracle index_only failed (%d)" % r)

    def set_executed(self, src, frontier):
        self.lib.oracle_graph_set_executed(self.h, src, frontier)

    def find_scc(self, dot, first_find=True):
        ms = (ctypes.c_uint32 * 64)()
        mq = (ctypes.c_uint64 * 64)()
        nm = ctypes.c_uint32()
        ready = ctypes.c_uint64()
        nd = ctypes.c_uint32()
        kind = self.lib.oracle_graph_find_scc(self.h, dot[0], dot[1], 1 if first_find else 0, ms, mq,
                                              64, ctypes.byref(nm), ctypes.byref(ready),
                                              ctypes.byref(nd))
        missing = [(ms[i], mq[i]) for i in range(min(nm.value, 64))]
        return kind, missing, ready.value, nd.value

    def drain(self):
        """Executed commands so far: list of ((src, seq), rec, scc_start)."""
        out = []
        src = (ctypes.c_uint32 * 256)()
        seq = (ctypes.c_uint64 * 256)()
        rec = (ctypes.c_uint32 * 256)()
        st = (ctypes.c_uint8 * 256)()
        while True:
            m = self.lib.oracle_graph_drain(self.h, src, seq, rec, st, 256)
            out.extend(((src[i], seq[i]), rec[i], bool(st[i])) for i in range(m))
            if m < 256:
                return out

    def pending(self):
        src = (ctypes.c_uint32 * 256)()
        seq = (ctypes.c_uint64 * 256)()
        ws = (ctypes.c_uint32 * 256)()
        wq = (ctypes.c_uint64 * 256)()
        m = self.lib.oracle_graph_pending(self.h, src, seq, ws, wq, 256)
        return [((src[i], seq[i]), (ws[i], wq[i])) for i in range(m)]

    def metrics(self, kind):
        v = (ctypes.c_uint64 * 4096)()
        c = (ctypes.c_uint64 * 4096)()
        m = self.lib.oracle_graph_metrics(self.h, kind, v, c, 4096)
        return {int(v[i]): int(c[i]) for i in range(min(m, 4096))}
