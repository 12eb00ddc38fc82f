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
SRCS = [os.path.join(HERE, f) for f in ("graph_oracle.cpp", "sim_oracle.cpp", "pred_oracle.cpp")]
DEPS = SRCS + [os.path.join(HERE, "graph_oracle.hpp"),
               os.path.join(os.path.dirname(HERE), "include", "fantoch_amd.h")]

_lib = None


def build():
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", LIB] + SRCS +
                          ["-lpthread"])


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(f) for f in DEPS):
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
        lib.oracle_pred_batch.restype = ctypes.c_int
        lib.oracle_pred_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, u32, u32, u32, u32, vp, vp, vp, vp, u32]
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
        lib.oracle_graph_new_sharded.restype = vp
        lib.oracle_graph_new_sharded.argtypes = [u32, u32, u32, u32]
        lib.oracle_graph_handle_add_sharded.restype = ctypes.c_int
        lib.oracle_graph_handle_add_sharded.argtypes = [vp, u32, u64, P32, P64, P32, u32, u64, u32]
        lib.oracle_graph_executed_reply.restype = ctypes.c_int
        lib.oracle_graph_executed_reply.argtypes = [vp, u32, u64, u64]
        lib.oracle_graph_requests.restype = u32
        lib.oracle_graph_requests.argtypes = [vp, P32, P32, P64, u32]
        lib.oracle_graph_to_executors.restype = u32
        lib.oracle_graph_to_executors.argtypes = [vp, P32, P64, u32]
        lib.oracle_clone_new.restype = vp
        lib.oracle_clone_new.argtypes = [vp]
        lib.oracle_clone_free.argtypes = [vp]
        lib.oracle_clone_handle_executed.argtypes = [vp, P32, P64, u32]
        lib.oracle_clone_handle_request.argtypes = [vp, u32, P32, P64, u32]
        lib.oracle_clone_cleanup.argtypes = [vp]
        lib.oracle_clone_replies.restype = u32
        lib.oracle_clone_replies.argtypes = [vp, P32, P32, P32, P64, P32, P32, u32, P32, P64, P32, u32]
        lib.oracle_graph_waits.restype = u32
        lib.oracle_graph_waits.argtypes = [vp, P32, P64, P32, P64, u32]
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


def pred_batch_execute(planes, clock_lo, clock_hi, execute_at_commit=False, threads=1, ndeps=None):
    """PredecessorsGraph (pred/mod.rs) over every stream of a host batch with
    packed Caesar clock planes ((seq << 8 | process id) split in two u32
    planes).  Returns (order, release, nexec, err) in the GPU plane layout."""
    lib = load()
    pw = planes.plane
    order = np.zeros(pw, np.uint32)
    release = np.zeros(pw, np.uint32)
    nexec = np.zeros(planes.S, np.uint32)
    err = np.zeros(planes.S, np.uint32)
    lengths = None
    if planes.lengths is not None:
        lengths = np.ascontiguousarray(planes.lengths, np.uint32)
    clo = np.ascontiguousarray(clock_lo, np.uint32)
    chi = np.ascontiguousarray(clock_hi, np.uint32)
    nd = None if ndeps is None else np.ascontiguousarray(ndeps, np.uint32)
    lib.oracle_pred_batch(planes.dot.ctypes.data, planes.hdr.ctypes.data, planes.deps.ctypes.data, clo.ctypes.data,
                          chi.ctypes.data, nd.ctypes.data if nd is not None else None,
                          lengths.ctypes.data if lengths is not None else None, planes.S, planes.steps, planes.dmax, planes.n, 2 if execute_at_commit else 0, order.ctypes.data,
                          release.ctypes.data, nexec.ctypes.data, err.ctypes.data, int(threads))
    return order, release, nexec, err


class Graph:
    """One DependencyGraph (graph/mod.rs:45-677), for the reference's unit-test shapes."""

    def __init__(self, process_id, n, shard_id=0, shard_count=1):
        self.lib = load()
        if shard_count > 1:
            self.h = self.lib.oracle_graph_new_sharded(process_id, n, shard_id, shard_count)
        else:
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

    def handle_add_sharded(self, dot, deps, shards, t_ms=0):
        """handle_add (or RequestReply::Info) with each dep's shard bitmask."""
        src, seq, nd = self._deps(deps)
        sh = (ctypes.c_uint32 * max(nd, 1))(*shards)
        r = self.lib.oracle_graph_handle_add_sharded(self.h, dot[0], dot[1], src, seq, sh, nd, t_ms, self.rec)
        self.rec += 1
        if r:
            raise RuntimeError("oracle handle_add_sharded failed (%d)" % r)

    def executed_reply(self, dot, t_ms=0):
        """RequestReply::Executed{dot}."""
        if self.lib.oracle_graph_executed_reply(self.h, dot[0], dot[1], t_ms):
            raise RuntimeError("oracle executed_reply failed")

    def requests(self):
        """Drains out-requests: sorted [(target shard, dot)]."""
        cap = 4096
        sh, src, seq = (ctypes.c_uint32 * cap)(), (ctypes.c_uint32 * cap)(), (ctypes.c_uint64 * cap)()
        m = self.lib.oracle_graph_requests(self.h, sh, src, seq, cap)
        return [(sh[i], (src[i], seq[i])) for i in range(min(m, cap))]

    def to_executors(self):
        """Drains the dots added to the executed clock (partial replication)."""
        cap = 1 << 16
        src, seq = (ctypes.c_uint32 * cap)(), (ctypes.c_uint64 * cap)()
        m = self.lib.oracle_graph_to_executors(self.h, src, seq, cap)
        return [(src[i], seq[i]) for i in range(min(m, cap))]

    def waits(self, cap=1 << 16):
        """Every (waiting dot, missing parent) registration, ascending."""
        vs, vq = (ctypes.c_uint32 * cap)(), (ctypes.c_uint64 * cap)()
        ps, pq = (ctypes.c_uint32 * cap)(), (ctypes.c_uint64 * cap)()
        m = self.lib.oracle_graph_waits(self.h, vs, vq, ps, pq, cap)
        return [((vs[i], vq[i]), (ps[i], pq[i])) for i in range(min(m, cap))]

    def clone(self):
        """An executor with index > 0 sharing this graph's VertexIndex."""
        return GraphClone(self)

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

    def pending(self, cap=256):
        src = (ctypes.c_uint32 * cap)()
        seq = (ctypes.c_uint64 * cap)()
        ws = (ctypes.c_uint32 * cap)()
        wq = (ctypes.c_uint64 * cap)()
        m = self.lib.oracle_graph_pending(self.h, src, seq, ws, wq, cap)
        return [((src[i], seq[i]), (ws[i], wq[i])) for i in range(m)]

    def metrics(self, kind):
        v = (ctypes.c_uint64 * 4096)()
        c = (ctypes.c_uint64 * 4096)()
        m = self.lib.oracle_graph_metrics(self.h, kind, v, c, 4096)
        return {int(v[i]): int(c[i]) for i in range(min(m, 4096))}


class GraphClone:
    """Executor index > 0 of a partial-replication process (mod.rs:211-355)."""

    def __init__(self, main):
        self.main = main  # keeps the shared graph alive
        self.lib = main.lib
        self.h = self.lib.oracle_clone_new(main.h)

    def __del__(self):
        try:
            self.lib.oracle_clone_free(self.h)
        except Exception:
            pass

    def handle_executed(self, dots):
        src, seq, n = self.main._deps(dots)
        self.lib.oracle_clone_handle_executed(self.h, src, seq, n)

    def handle_request(self, from_shard, dots):
        src, seq, n = self.main._deps(dots)
        self.lib.oracle_clone_handle_request(self.h, from_shard, src, seq, n)

    def cleanup(self):
        self.lib.oracle_clone_cleanup(self.h)

    def replies(self):
        """Drains [(to shard, 'info' | 'executed', dot, [(dep, shards)])]."""
        cap, dcap = 4096, 1 << 16
        to, kind, src, rec, nd = [(ctypes.c_uint32 * cap)() for _ in range(5)]
        seq = (ctypes.c_uint64 * cap)()
        ds, dsh = (ctypes.c_uint32 * dcap)(), (ctypes.c_uint32 * dcap)()
        dq = (ctypes.c_uint64 * dcap)()
        m = self.lib.oracle_clone_replies(self.h, to, kind, src, seq, rec, nd, cap, ds, dq, dsh, dcap)
        out, k = [], 0
        for i in range(m):
            deps = [((ds[k + j], dq[k + j]), dsh[k + j]) for j in range(nd[i])]
            k += nd[i]
            out.append((to[i], "info" if kind[i] else "executed", (src[i], seq[i]), deps))
        return out


# ------------------------------------------------------------ simulator
ROOT = os.path.dirname(HERE)
PLANET_DIR = os.path.join(ROOT, "fantoch_amd", "data", "latency_gcp")


class SimSpec(ctypes.Structure):
    """fx_sim_spec (include/fantoch_amd.h)."""
    _fields_ = [("seed", ctypes.c_uint64), ("instance", ctypes.c_uint64),
                ("protocol", ctypes.c_uint32), ("n", ctypes.c_uint32), ("f", ctypes.c_uint32),
                ("gc_interval_ms", ctypes.c_uint32), ("executed_notification_ms", ctypes.c_uint32),
                ("clients_per_region", ctypes.c_uint32), ("commands_per_client", ctypes.c_uint32),
                ("keys_per_command", ctypes.c_uint32), ("conflict_rate", ctypes.c_uint32),
                ("pool_size", ctypes.c_uint32), ("read_only_pct", ctypes.c_uint32),
                ("extra_sim_time_ms", ctypes.c_int32), ("reorder_messages", ctypes.c_uint32),
                ("nfr", ctypes.c_uint32), ("num_client_regions", ctypes.c_uint32),
                ("process_regions", ctypes.c_uint8 * 8), ("client_regions", ctypes.c_uint8 * 20)]


class SimOut(ctypes.Structure):
    _fields_ = [("executed", ctypes.c_void_p), ("executed_len", ctypes.c_void_p),
                ("exec_cap", ctypes.c_uint32), ("latency", ctypes.c_void_p), ("issued", ctypes.c_void_p),
                ("R", ctypes.c_uint32), ("lat_bins", ctypes.c_uint32), ("fast", ctypes.c_void_p),
                ("slow", ctypes.c_void_p), ("stable", ctypes.c_void_p), ("chain", ctypes.c_void_p),
                ("delay", ctypes.c_void_p), ("chain_bins", ctypes.c_uint32),
                ("delay_bins", ctypes.c_uint32), ("end_ms", ctypes.c_uint64),
                ("events", ctypes.c_uint64), ("trace", ctypes.c_uint64), ("status", ctypes.c_int32),
                ("pad", ctypes.c_int32), ("monitor_hash", ctypes.c_void_p),
                ("fast_reads", ctypes.c_void_p), ("slow_reads", ctypes.c_void_p)]


def _sim_lib():
    lib = load()
    if not getattr(lib, "_sim_bound", False):
        lib.oracle_planet_regions.restype = ctypes.c_int
        lib.oracle_planet_regions.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32]
        lib.oracle_planet_matrix.restype = ctypes.c_int
        lib.oracle_planet_matrix.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_uint32]
        lib.oracle_sort_processes.restype = ctypes.c_int
        lib.oracle_sort_processes.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        lib.oracle_sim_run.restype = ctypes.c_int
        lib.oracle_sim_run.argtypes = [ctypes.c_char_p, ctypes.POINTER(SimSpec), ctypes.POINTER(SimOut)]
        lib.oracle_sim_batch.restype = ctypes.c_int
        lib.oracle_sim_batch.argtypes = [ctypes.c_char_p, ctypes.POINTER(SimSpec), ctypes.c_uint32,
                                         ctypes.POINTER(SimOut), ctypes.c_int]
        lib.oracle_sim_capture.restype = ctypes.c_int
        lib.oracle_sim_capture.argtypes = [ctypes.c_char_p, ctypes.POINTER(SimSpec), ctypes.c_uint64] + \
            [ctypes.c_void_p] * 7
        lib._sim_bound = True
    return lib


def planet_regions(planet_dir=PLANET_DIR):
    buf = ctypes.create_string_buffer(4096)
    r = _sim_lib().oracle_planet_regions(planet_dir.encode(), buf, 4096)
    if r < 0:
        raise RuntimeError("cannot load planet %s" % planet_dir)
    return buf.value.decode().split()


def planet_matrix(planet_dir=PLANET_DIR):
    R = len(planet_regions(planet_dir))
    lat = np.zeros((R, R), np.int64)
    srt = np.zeros((R, R), np.uint32)
    if _sim_lib().oracle_planet_matrix(planet_dir.encode(), lat.ctypes.data, srt.ctypes.data, R):
        raise RuntimeError("planet matrix")
    return lat, srt


def sort_processes(region, procs, planet_dir=PLANET_DIR):
    """util.rs:153-185 over [(id, region index)] -> sorted ids."""
    ids = np.array([p[0] for p in procs], np.uint32)
    regs = np.array([p[1] for p in procs], np.uint32)
    out = np.zeros(len(procs), np.uint32)
    _sim_lib().oracle_sort_processes(planet_dir.encode(), region, ids.ctypes.data, regs.ctypes.data,
                                     len(procs), out.ctypes.data)
    return [int(x) for x in out]


def make_spec(protocol, n, f, process_regions, client_regions, clients_per_region=1,
              commands_per_client=100, keys_per_command=1, conflict_rate=2, pool_size=1,
              read_only_pct=0, gc_interval_ms=10, executed_notification_ms=10,
              extra_sim_time_ms=-1, reorder=False, nfr=False, seed=0, instance=0):
    s = SimSpec()
    s.seed, s.instance, s.protocol, s.n, s.f = seed, instance, protocol, n, f
    s.gc_interval_ms, s.executed_notification_ms = gc_interval_ms, executed_notification_ms
    s.clients_per_region, s.commands_per_client = clients_per_region, commands_per_client
    s.keys_per_command, s.conflict_rate, s.pool_size = keys_per_command, conflict_rate, pool_size
    s.read_only_pct, s.extra_sim_time_ms = read_only_pct, extra_sim_time_ms
    s.reorder_messages, s.nfr = int(bool(reorder)), int(bool(nfr))
    s.num_client_regions = len(client_regions)
    for i, r in enumerate(process_regions):
        s.process_regions[i] = r
    for i, r in enumerate(client_regions):
        s.client_regions[i] = r
    return s


class _OutBufs:
    def __init__(self, spec, R, exec_cap, lat_bins, chain_bins, delay_bins):
        n = spec.n
        self.executed = np.zeros((n, exec_cap), np.uint32)
        self.executed_len = np.zeros(n, np.uint64)
        self.latency = np.zeros((R, lat_bins), np.uint64)
        self.issued = np.zeros(R, np.uint64)
        self.fast = np.zeros(n, np.uint64)
        self.slow = np.zeros(n, np.uint64)
        self.stable = np.zeros(n, np.uint64)
        self.chain = np.zeros(chain_bins, np.uint64)
        self.delay = np.zeros(delay_bins, np.uint64)
        self.monitor_hash = np.zeros(n, np.uint64)
        self.fast_reads = np.zeros(n, np.uint64)
        self.slow_reads = np.zeros(n, np.uint64)
        o = SimOut()
        o.executed, o.executed_len, o.exec_cap = self.executed.ctypes.data, self.executed_len.ctypes.data, exec_cap
        o.latency, o.issued, o.R, o.lat_bins = self.latency.ctypes.data, self.issued.ctypes.data, R, lat_bins
        o.fast, o.slow, o.stable = self.fast.ctypes.data, self.slow.ctypes.data, self.stable.ctypes.data
        o.chain, o.delay = self.chain.ctypes.data, self.delay.ctypes.data
        o.chain_bins, o.delay_bins = chain_bins, delay_bins
        o.monitor_hash = self.monitor_hash.ctypes.data
        o.fast_reads, o.slow_reads = self.fast_reads.ctypes.data, self.slow_reads.ctypes.data
        self.out = o

    def result(self):
        o = self.out
        return {"executed": [self.executed[p, :int(self.executed_len[p])].copy()
                             for p in range(self.executed.shape[0])],
                "latency": self.latency, "issued": self.issued, "fast": self.fast,
                "slow": self.slow, "stable": self.stable, "chain": self.chain, "delay": self.delay,
                "end_ms": int(o.end_ms), "events": int(o.events), "trace": int(o.trace),
                "status": int(o.status), "monitor_hash": self.monitor_hash,
                "fast_reads": self.fast_reads, "slow_reads": self.slow_reads}


def spec_from(s):
    """Copies a product-side fx_sim_spec (any ctypes struct with the same field
    names) into the oracle's SimSpec."""
    o = SimSpec()
    for name, _ in SimSpec._fields_:
        v = getattr(s, name)
        if name in ("process_regions", "client_regions"):
            arr = getattr(o, name)
            for i in range(len(v)):
                arr[i] = v[i]
        else:
            setattr(o, name, v)
    return o


def sim_run(spec, exec_cap=None, lat_bins=8192, chain_bins=256, delay_bins=8192,
            planet_dir=PLANET_DIR):
    """Runs one simulated instance (Runner::run) through the C++ oracle."""
    R = len(planet_regions(planet_dir))
    if exec_cap is None:
        exec_cap = spec.clients_per_region * spec.num_client_regions * spec.commands_per_client + 8
    b = _OutBufs(spec, R, exec_cap, lat_bins, chain_bins, delay_bins)
    _sim_lib().oracle_sim_run(planet_dir.encode(), ctypes.byref(spec), ctypes.byref(b.out))
    r = b.result()
    if r["status"]:
        raise RuntimeError("oracle sim failed (status %d)" % r["status"])
    return r


def sim_batch(specs, threads=1, exec_cap=None, lat_bins=8192, chain_bins=256, delay_bins=8192,
              planet_dir=PLANET_DIR):
    """Runs many instances on `threads` std::threads; returns a list of results."""
    R = len(planet_regions(planet_dir))
    arr = (SimSpec * len(specs))(*specs)
    bufs = []
    outs = (SimOut * len(specs))()
    for i, s in enumerate(specs):
        cap = exec_cap or s.clients_per_region * s.num_client_regions * s.commands_per_client + 8
        b = _OutBufs(s, R, cap, lat_bins, chain_bins, delay_bins)
        bufs.append(b)
        outs[i] = b.out
    _sim_lib().oracle_sim_batch(planet_dir.encode(), arr, len(specs), outs, int(threads))
    res = []
    for i, b in enumerate(bufs):
        b.out = outs[i]
        res.append(b.result())
    return res


def pack(d):
    return (int(d[0]) << 24) | int(d[1])


def unpack(x):
    return (int(x) >> 24, int(x) & 0xFFFFFF)


def quorum_deps(fq, reports, threshold):
    """QuorumDeps (quorum.rs:16-103): reports = [set of dots] from processes 1..;
    returns (union, all, check_threshold(threshold), check_equal)."""
    lib = load()
    lib.oracle_quorum_deps.restype = ctypes.c_int
    lens = np.array([len(r) for r in reports] + [0], np.uint32)
    flat = np.array([pack(d) for r in reports for d in sorted(r)] + [0], np.uint32)
    out = np.zeros(256, np.uint32)
    nu, al, th, eq = (ctypes.c_uint32() for _ in range(4))
    lib.oracle_quorum_deps(ctypes.c_uint32(fq), ctypes.c_uint32(len(reports)),
                           ctypes.c_void_p(lens.ctypes.data), ctypes.c_void_p(flat.ctypes.data),
                           ctypes.c_uint32(threshold), ctypes.c_void_p(out.ctypes.data),
                           ctypes.c_uint32(256), ctypes.byref(nu), ctypes.byref(al), ctypes.byref(th),
                           ctypes.byref(eq))
    return {unpack(x) for x in out[:nu.value]}, bool(al.value), bool(th.value), bool(eq.value)


def key_deps_script(ops, nfr=False):
    """ops: ("add", dot, keys, read_only) | ("noop", dot) | ("deps", keys, read_only) |
    ("noop_deps",) -> list of dep sets (one per op)."""
    lib = load()
    kind, dot, nk, keys, ro = [], [], [], [], []
    for op in ops:
        if op[0] == "add":
            kind.append(0); dot.append(pack(op[1])); nk.append(len(op[2])); keys += op[2]; ro.append(int(op[3]))
        elif op[0] == "noop":
            kind.append(1); dot.append(pack(op[1])); nk.append(0); ro.append(0)
        elif op[0] == "deps":
            kind.append(2); dot.append(0); nk.append(len(op[1])); keys += op[1]; ro.append(int(op[2]))
        else:
            kind.append(3); dot.append(0); nk.append(0); ro.append(0)
    cap = 64
    a = lambda v: np.array(v + [0], np.uint32)
    kind_a, dot_a, nk_a, keys_a, ro_a = a(kind), a(dot), a(nk), a(keys), a(ro)
    out = np.zeros(len(ops) * cap, np.uint32)
    olen = np.zeros(len(ops), np.uint32)
    lib.oracle_key_deps_script(ctypes.c_uint32(int(nfr)), ctypes.c_uint32(len(ops)),
                               *[ctypes.c_void_p(x.ctypes.data) for x in (kind_a, dot_a, nk_a, keys_a, ro_a)],
                               ctypes.c_uint32(cap), ctypes.c_void_p(out.ctypes.data),
                               ctypes.c_void_p(olen.ctypes.data))
    return [{unpack(x) for x in out[i * cap:i * cap + olen[i]]} for i in range(len(ops))]


def gc_script(n, ops):
    """ops: ("add", dot) | ("update", from, [clock n]) | ("stable",) ->
    list of (stable ranges or None, frontier after the op)."""
    lib = load()
    kind = np.array([{"add": 0, "update": 1, "stable": 2}[o[0]] for o in ops], np.uint32)
    arg = np.array([pack(o[1]) if o[0] == "add" else (o[1] if o[0] == "update" else 0) for o in ops], np.uint32)
    clocks = np.zeros((len(ops), n), np.uint64)
    for i, o in enumerate(ops):
        if o[0] == "update":
            clocks[i] = o[2]
    cap = 16
    out = np.zeros((len(ops), cap, 3), np.uint64)
    olen = np.zeros(len(ops), np.uint32)
    fr = np.zeros((len(ops), n), np.uint64)
    lib.oracle_gc_script(ctypes.c_uint32(n), ctypes.c_uint32(len(ops)),
                         *[ctypes.c_void_p(x.ctypes.data) for x in (kind, arg, clocks)],
                         ctypes.c_uint32(cap), ctypes.c_void_p(out.ctypes.data),
                         ctypes.c_void_p(olen.ctypes.data), ctypes.c_void_p(fr.ctypes.data))
    res = []
    for i, o in enumerate(ops):
        st = [tuple(int(v) for v in out[i, j]) for j in range(olen[i])] if o[0] == "stable" else None
        res.append((st, [int(v) for v in fr[i]]))
    return res


def workload_keys(spec, client, count):
    """Keys (and read-only flags) of the first `count` commands of `client`."""
    lib = load()
    keys = np.zeros(count * spec.keys_per_command, np.uint32)
    ro = np.zeros(count, np.uint32)
    lib.oracle_workload_keys(ctypes.byref(spec), ctypes.c_uint64(client), ctypes.c_uint32(count),
                             ctypes.c_void_p(keys.ctypes.data), ctypes.c_void_p(ro.ctypes.data))
    return keys.reshape(count, spec.keys_per_command), ro


def sim_capture_raw(spec, cap=None, planet_dir=PLANET_DIR):
    """One instance through the simulator oracle, capturing each process's
    executor input (the Adds its GraphExecutor receives, in handle order).
    Returns dict of arrays: dot, t_ms, nd [n][cap], deps [n][cap][8], len [n],
    executed [n][cap] (the simulation's execution order), exec_len [n]."""
    lib = _sim_lib()
    n = spec.n
    if cap is None:
        cap = spec.clients_per_region * spec.num_client_regions * spec.commands_per_client
    out = {"dot": np.zeros((n, cap), np.uint32), "t_ms": np.zeros((n, cap), np.uint32),
           "nd": np.zeros((n, cap), np.uint32), "deps": np.zeros((n, cap, 8), np.uint32),
           "len": np.zeros(n, np.uint64), "executed": np.zeros((n, cap), np.uint32),
           "exec_len": np.zeros(n, np.uint64)}
    st = lib.oracle_sim_capture(planet_dir.encode(), ctypes.byref(spec), cap, out["dot"].ctypes.data,
                                out["t_ms"].ctypes.data, out["nd"].ctypes.data, out["deps"].ctypes.data,
                                out["len"].ctypes.data, out["executed"].ctypes.data, out["exec_len"].ctypes.data)
    if st != 0:
        raise RuntimeError("oracle_sim_capture status %d" % st)
    return out


def sim_capture(spec, planet_dir=PLANET_DIR):
    """sim_capture_raw as lists: (streams, executed), streams[p] = [(dot, deps,
    t_ms)] with dots as (source, seq), executed[p] = packed dots in order."""
    r = sim_capture_raw(spec, planet_dir=planet_dir)
    streams = []
    for p in range(spec.n):
        k = int(r["len"][p])
        streams.append([(unpack(r["dot"][p, i]), [unpack(x) for x in r["deps"][p, i, :r["nd"][p, i]]],
                         int(r["t_ms"][p, i])) for i in range(k)])
    return streams, [r["executed"][p, :int(r["exec_len"][p])].copy() for p in range(spec.n)]
