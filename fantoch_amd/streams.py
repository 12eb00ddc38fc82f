"""Host-side commit-stream packing (numpy) for the tiled plane layout.

A commit stream is what one executor sees: the sequence of
GraphExecutionInfo::Add{dot, cmd, deps} (fantoch_ps/src/executor/graph/executor.rs:197-214)
delivered to it, each with the SysTime::millis() of its delivery.  Here an Add
is (dot, deps, t_ms[, kind]) with dot = (source, seq) and deps a collection of
dots; deps are canonicalised to ascending order without duplicates (C1).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import index, make_hdr, pack_dot, plane_words


class Planes:
    """Host copy of a batch: dot/hdr planes, dmax dep planes, optional lengths."""

    def __init__(self, num_streams, steps, dmax, n, dot=None, hdr=None, deps=None, lengths=None):
        self.S = int(num_streams)
        self.steps = int(steps)
        self.dmax = int(dmax)
        self.n = int(n)
        pw = plane_words(self.S, self.steps)
        self.plane = pw
        self.dot = np.zeros(pw, np.uint32) if dot is None else dot
        self.hdr = np.zeros(pw, np.uint32) if hdr is None else hdr
        self.deps = np.zeros(max(self.dmax, 1) * pw, np.uint32) if deps is None else deps
        self.lengths = lengths

    def stream(self, s):
        """Decodes stream s back into a list of (dot, deps, t, kind)."""
        L = self.steps if self.lengths is None else int(self.lengths[s])
        idx = index(np.arange(L), s, self.steps)
        out = []
        for i in range(L):
            at = int(idx[i])
            h = int(self.hdr[at])
            nd = (h >> 24) & 31
            deps = [_lib.unpack_dot(self.deps[j * self.plane + at]) for j in range(nd)]
            out.append((_lib.unpack_dot(self.dot[at]), deps, h & 0xFFFFFF, h >> 29))
        return out


def pack_streams(streams, n):
    """streams: list of lists of (dot, deps, t_ms) or (dot, deps, t_ms, kind)."""
    S = len(streams)
    steps = max([len(s) for s in streams] + [1])
    dmax = 1
    canon = []
    for st in streams:
        cs = []
        for add in st:
            dot, deps, t = add[0], add[1], add[2]
            kind = add[3] if len(add) > 3 else _lib.FX_KIND_ADD
            pd = sorted(set(pack_dot(*d) for d in deps))
            dmax = max(dmax, len(pd))
            cs.append((pack_dot(*dot), pd, int(t), int(kind)))
        canon.append(cs)
    p = Planes(S, steps, dmax, n, lengths=np.array([len(s) for s in streams], np.uint32))
    for s, cs in enumerate(canon):
        if not cs:
            continue
        idx = index(np.arange(len(cs)), s, steps)
        for i, (d, pd, t, kind) in enumerate(cs):
            at = int(idx[i])
            p.dot[at] = d
            p.hdr[at] = make_hdr(t, len(pd), kind)
            for j, x in enumerate(pd):
                p.deps[j * p.plane + at] = x
    return p


def synth_params(seed=1, instances=1, n=5, cmds=100, window=8, cycle_pct=30, horizon=64,
                 conflicts=(0, 2, 10, 50, 100), instance_base=0, conflict_block=0, clients=1, key_pool=0):
    p = _lib.SynthParams()
    p.seed = seed
    p.instances = instances
    p.instance_base = instance_base
    p.n = n
    p.cmds_per_process = cmds
    p.window = window
    p.cycle_pct = cycle_pct
    p.horizon = horizon
    p.num_conflicts = len(conflicts)
    for i, c in enumerate(conflicts):
        p.conflict_pct[i] = c
    p.conflict_block = conflict_block
    p.clients = clients
    p.key_pool = key_pool
    return p


def synth_shape(params):
    S, steps, dmax = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    _lib.check(_lib.load().fx_synth_shape(ctypes.byref(params), ctypes.byref(S), ctypes.byref(steps),
                                          ctypes.byref(dmax)), "fx_synth_shape")
    return S.value, steps.value, dmax.value


def synth_host(params):
    """Synthetic commit streams generated on the host (same bytes as the GPU generator)."""
    S, steps, dmax = synth_shape(params)
    p = Planes(S, steps, dmax, params.n)
    _lib.check(_lib.load().fx_synth_generate_host(
        ctypes.byref(params), p.dot.ctypes.data, p.hdr.ctypes.data, p.deps.ctypes.data),
        "fx_synth_generate_host")
    return p


def decode_orders(order, nexec, S, steps):
    """order plane -> per stream list of (rec, scc_start)."""
    out = []
    for s in range(S):
        k = int(nexec[s])
        idx = index(np.arange(k), s, steps)
        o = order[idx]
        out.append([(int(x) & 0x7FFFFFFF, bool(int(x) & _lib.FX_ORDER_SCC_START)) for x in o])
    return out


def decode_release(release, lengths, S, steps):
    out = []
    for s in range(S):
        L = steps if lengths is None else int(lengths[s])
        idx = index(np.arange(L), s, steps)
        out.append(release[idx].copy())
    return out
