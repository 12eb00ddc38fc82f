"""`GraphExecutor`: the reference's Executor trait over the C-ABI (runs on the GPU).

Mirrors fantoch_ps/src/executor/graph/executor.rs:31-114 (trait surface in
fantoch/src/executor/mod.rs:27-89): `handle(Add)`, `to_clients()`,
`to_clients_iter()`, `metrics()`, `monitor()`, `parallel()`.  Keys are u32
ids (canonical C7); a reference panic is an FxError here.
"""
import ctypes

from . import _lib
from ._lib import CDot, CRifl, check

EXECUTION_DELAY = 0
CHAIN_SIZE = 1


class GraphExecutor:
    def __init__(self, process_id, shard_id, n, f=1, execute_at_commit=False, monitor=True, shard_count=1):
        lib = _lib.load()
        cfg = _lib.Config(n, f, shard_count, 1 if execute_at_commit else 0, 1 if monitor else 0)
        h = lib.fx_graph_executor_new(process_id, shard_id, ctypes.byref(cfg))
        if not h:
            raise _lib.FxError(_lib.FX_ERR_NO_DEVICE if lib.fx_device_count() <= 0
                               else _lib.FX_ERR_INVALID_ARG, "fx_graph_executor_new")
        self._h = h
        self.n = n
        # per-handle call buffers: the simulator's pattern calls handle_add and
        # a drain after every commit, so neither allocates ctypes arrays per call
        self._add = lib.fx_graph_executor_handle_add
        self._drain = lib.fx_graph_executor_drain_dots
        self._karr = (ctypes.c_uint32 * 16)()
        self._darr = (CDot * 64)()
        self._du32 = (ctypes.c_uint32 * 128).from_buffer(self._darr)  # the same words, flat
        self._dbuf = (CDot * 256)()
        self._dstart = (ctypes.c_uint8 * 256)()
        self._got = ctypes.c_uint32()
        self._gotref = ctypes.byref(self._got)

    def close(self):
        if self._h:
            _lib.load().fx_graph_executor_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def parallel():
        return bool(_lib.load().fx_graph_executor_parallel())

    def set_executor_index(self, index):
        check(_lib.load().fx_graph_executor_set_executor_index(self._h, index))

    def handle_add(self, dot, rifl, keys, deps, time_ms, read_only=False):
        """handle(GraphExecutionInfo::Add{dot, cmd, deps}, time)."""
        keys = list(keys)
        deps = list(deps)
        if len(keys) <= 16:
            karr = self._karr
            for i, k in enumerate(keys):
                karr[i] = k
        else:
            karr = (ctypes.c_uint32 * len(keys))(*keys)
        if len(deps) <= 64:
            darr = self._darr
            self._du32[0:2 * len(deps)] = [int(x) for d in deps for x in d]
        else:
            darr = (CDot * len(deps))(*[CDot(int(s), int(q)) for s, q in deps])
        st = self._add(self._h, CDot(*dot), CRifl(*rifl), karr, len(keys), 1 if read_only else 0, darr,
                       len(deps), int(time_ms))
        if st:
            check(st, "handle_add")

    # ---- partial replication (shard_count > 1, graph/mod.rs:82-406)
    def handle_add_sharded(self, dot, rifl, keys, deps, shards, time_ms, read_only=False, cmd_shards=0):
        """handle(Add) / RequestReply::Info with each dep's shard bitmask;
        cmd_shards = the command's own shard set (0 = this shard only)."""
        keys = list(keys)
        karr = (ctypes.c_uint32 * max(len(keys), 1))(*keys)
        deps = list(deps)
        darr = (CDot * max(len(deps), 1))(*[CDot(int(s), int(q)) for s, q in deps])
        sarr = (ctypes.c_uint32 * max(len(deps), 1))(*[int(m) for m in shards])
        check(_lib.load().fx_graph_executor_handle_add_sharded(
            self._h, CDot(*dot), CRifl(*rifl), karr, len(keys), 1 if read_only else 0, darr, sarr,
            len(deps), int(time_ms), int(cmd_shards)), "handle_add_sharded")

    def handle_executed(self, dots, time_ms):
        """RequestReply::Executed for each dot."""
        dots = list(dots)
        darr = (CDot * max(len(dots), 1))(*[CDot(int(s), int(q)) for s, q in dots])
        check(_lib.load().fx_graph_executor_handle_executed(self._h, darr, len(dots), int(time_ms)),
              "handle_executed")

    def requests(self):
        """Drains out-requests: sorted [(target shard, dot)]."""
        out = []
        sh = (ctypes.c_uint64 * 256)()
        buf = (CDot * 256)()
        got = ctypes.c_uint32()
        while True:
            check(_lib.load().fx_graph_executor_requests(self._h, sh, buf, 256, ctypes.byref(got)), "requests")
            out += [(sh[i], (buf[i].source, buf[i].seq)) for i in range(got.value)]
            if got.value < 256:
                return out

    def to_executors(self):
        """Drains the dots added to the executed clock (Executed info for the other executors)."""
        out = []
        buf = (CDot * 256)()
        got = ctypes.c_uint32()
        while True:
            check(_lib.load().fx_graph_executor_to_executors(self._h, buf, 256, ctypes.byref(got)),
                  "to_executors")
            out += [(buf[i].source, buf[i].seq) for i in range(got.value)]
            if got.value < 256:
                return out

    def clone(self):
        """Executor index > 0 sharing this handle's VertexIndex (partial replication)."""
        return ExecutorClone(self)

    def index_only(self, dot, rifl, keys, deps, time_ms=0):
        keys = list(keys)
        karr = (ctypes.c_uint32 * max(len(keys), 1))(*keys)
        deps = list(deps)
        darr = (CDot * max(len(deps), 1))(*[CDot(int(s), int(q)) for s, q in deps])
        check(_lib.load().fx_graph_executor_index_only(
            self._h, CDot(*dot), CRifl(*rifl), karr, len(keys), darr, len(deps), int(time_ms)),
            "index_only")

    def set_executed_frontier(self, frontier):
        arr = (ctypes.c_uint64 * len(frontier))(*frontier)
        check(_lib.load().fx_graph_executor_set_executed_frontier(self._h, arr, len(frontier)))

    def to_clients_iter(self):
        """Drains ExecutorResults: list of (rifl, key)."""
        out = []
        buf = (_lib.ExecutorResultC * 256)()
        got = ctypes.c_uint32()
        while True:
            check(_lib.load().fx_graph_executor_to_clients(self._h, buf, 256, ctypes.byref(got)),
                  "to_clients")
            for i in range(got.value):
                r = buf[i]
                out.append(((r.rifl.source, r.rifl.seq), r.key))
            if got.value < 256:
                return out

    def drain_dots(self):
        """Executed dots in execution order: list of ((source, seq), scc_start)."""
        out = []
        buf, start, got = self._dbuf, self._dstart, self._got
        while True:
            st = self._drain(self._h, buf, start, 256, self._gotref)
            if st:
                check(st, "drain_dots")
            n = got.value
            for i in range(n):
                d = buf[i]
                out.append(((d.source, d.seq), bool(start[i])))
            if n < 256:
                return out

    def metrics(self, kind):
        """{value: count} of ExecutionDelay (0) or ChainSize (1)."""
        got = ctypes.c_uint32()
        lib = _lib.load()
        check(lib.fx_graph_executor_metrics(self._h, kind, None, None, 0, ctypes.byref(got)))
        n = got.value
        v = (ctypes.c_uint64 * max(n, 1))()
        c = (ctypes.c_uint64 * max(n, 1))()
        check(lib.fx_graph_executor_metrics(self._h, kind, v, c, n, ctypes.byref(got)))
        return {int(v[i]): int(c[i]) for i in range(n)}

    def monitor(self, key):
        got = ctypes.c_uint32()
        lib = _lib.load()
        check(lib.fx_graph_executor_monitor(self._h, key, None, 0, ctypes.byref(got)))
        n = got.value
        buf = (CRifl * max(n, 1))()
        check(lib.fx_graph_executor_monitor(self._h, key, buf, n, ctypes.byref(got)))
        return [(buf[i].source, buf[i].seq) for i in range(n)]

    def pending(self):
        """[(dot, waiting_on)] of the pending vertices, ascending."""
        got = ctypes.c_uint32()
        lib = _lib.load()
        check(lib.fx_graph_executor_pending(self._h, None, None, 0, ctypes.byref(got)))
        n = got.value
        buf = (CDot * max(n, 1))()
        wb = (CDot * max(n, 1))()
        check(lib.fx_graph_executor_pending(self._h, buf, wb, n, ctypes.byref(got)))
        return [((buf[i].source, buf[i].seq), (wb[i].source, wb[i].seq))
                for i in range(min(got.value, n))]

    def transfer_stats(self):
        """(host-to-device, device-to-host) bytes moved by this handle so far."""
        h2d, d2h = ctypes.c_uint64(), ctypes.c_uint64()
        check(_lib.load().fx_graph_executor_transfer_stats(self._h, ctypes.byref(h2d),
                                                           ctypes.byref(d2h)))
        return h2d.value, d2h.value

    def persist_stats(self):
        """fx_graph_executor_persist_stats: the persistent mode's counters
        (include/fantoch_amd.h FX_PERSIST_STATS; the kernel's words only with
        FX_HANDLE_STATS=1 in the environment when the handle was made)."""
        lib = _lib.load()
        n = 15
        out = (ctypes.c_uint64 * n)()
        check(lib.fx_graph_executor_persist_stats(self._h, out, n))
        return [int(x) for x in out]

    def debug_hooks(self, skip_status_flush=0, hold_ms=0):
        """fx_graph_executor_debug_hooks (tests only): from the persistent
        kernel's next launch, skip the status of its k-th flush and/or ignore
        stop requests until it has been idle hold_ms."""
        check(_lib.load().fx_graph_executor_debug_hooks(self._h, skip_status_flush, hold_ms))


class ExecutorClone:
    """Executor index > 0 of a partial-replication process: GraphExecutionInfo::
    Executed, Request serving and cleanup (graph/mod.rs:183-355)."""

    def __init__(self, main):
        self.main = main  # freed after the clone
        h = _lib.load().fx_graph_executor_clone(main._h)
        if not h:
            raise _lib.FxError(_lib.FX_ERR_INVALID_ARG, "fx_graph_executor_clone")
        self._h = h

    def close(self):
        if self._h:
            _lib.load().fx_graph_executor_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _dots(self, dots):
        dots = list(dots)
        return (CDot * max(len(dots), 1))(*[CDot(int(s), int(q)) for s, q in dots]), len(dots)

    def handle_executed(self, dots):
        arr, n = self._dots(dots)
        check(_lib.load().fx_graph_executor_handle_executed_info(self._h, arr, n), "handle_executed_info")

    def handle_request(self, from_shard, dots):
        arr, n = self._dots(dots)
        check(_lib.load().fx_graph_executor_handle_request(self._h, int(from_shard), arr, n), "handle_request")

    def cleanup(self):
        check(_lib.load().fx_graph_executor_cleanup(self._h), "cleanup")

    def replies(self, with_cmd_shards=False):
        """Drains [(to shard, 'info' | 'executed', dot, [(dep, shards)])] (plus
        each Info's command shard set when with_cmd_shards)."""
        out = []
        buf = (_lib.RequestReplyC * 256)()
        deps = (CDot * 8192)()
        sh = (ctypes.c_uint32 * 8192)()
        got = ctypes.c_uint32()
        while True:
            check(_lib.load().fx_graph_executor_request_replies(self._h, buf, 256, deps, sh, 8192,
                                                                 ctypes.byref(got)), "request_replies")
            for i in range(got.value):
                r = buf[i]
                d = [((deps[r.first_dep + j].source, deps[r.first_dep + j].seq), sh[r.first_dep + j])
                     for j in range(r.ndeps)]
                row = (r.to_shard, "info" if r.kind else "executed", (r.dot.source, r.dot.seq), d)
                out.append(row + (int(r.cmd_shards),) if with_cmd_shards else row)
            if got.value < 256:
                return out
