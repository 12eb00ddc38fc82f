"""Execution logs of the run mode: write, read (C-ABI) and replay on the GPU executor.

The file is what execution_logger_task writes
(fantoch/src/run/task/server/execution_logger.rs:11-55): LengthDelimitedCodec
frames (4-byte big-endian length) around `bincode::serialize` of each
GraphExecutionInfo (fantoch_ps/src/executor/graph/executor.rs:197-214) — see
fantoch_amd/csrc/exec_log.cpp for the byte layout.  `replay` mirrors
fantoch_ps/src/bin/graph_executor_replay.rs:13-38: a GraphExecutor with
process_id 1, shard 0 and Config::new(n, f) handles every Add in file order.

Reading is host-side (the C-ABI decoder); executing always goes through the
GPU executor — there is no CPU path here.
"""
import ctypes
import struct

import numpy as np

from . import _lib
from ._lib import check
from .executor import GraphExecutor

# KVOp (fantoch/src/kvs.rs:13-17)
GET = ("get",)
DELETE = ("delete",)


def put(value):
    return ("put", value)


# ------------------------------------------------------------------ writer
def _u8(v):
    return struct.pack("<B", v)


def _u32(v):
    return struct.pack("<I", v)


def _u64(v):
    return struct.pack("<Q", v)


def _str(s):
    b = s.encode() if isinstance(s, str) else bytes(s)
    return _u64(len(b)) + b


def _dot(d):
    return _u8(d[0]) + _u64(d[1])


def _ops(ops):
    out = [_u64(len(ops))]
    for op in ops:
        if op[0] == "get":
            out.append(_u32(0))
        elif op[0] == "put":
            out.append(_u32(1) + _str(op[1]))
        elif op[0] == "delete":
            out.append(_u32(2))
        else:
            raise ValueError(op)
    return b"".join(out)


def encode_command(rifl, shard_to_ops):
    """bincode of Command (fantoch/src/command.rs:13-22): rifl, shard_to_ops,
    shard_to_keys (derived, command.rs:33-58) and the empty `_empty_keys`."""
    out = [_u64(rifl[0]), _u64(rifl[1]), _u64(len(shard_to_ops))]
    for shard, kops in shard_to_ops.items():
        out.append(_u64(shard) + _u64(len(kops)))
        for key, ops in kops.items():
            out.append(_str(key) + _ops(ops))
    out.append(_u64(len(shard_to_ops)))
    for shard, kops in shard_to_ops.items():
        out.append(_u64(shard) + _u64(len(kops)) + b"".join(_str(k) for k in kops))
    out.append(_u64(0))
    return b"".join(out)


def _dependency(dep):
    dot, shards = dep if isinstance(dep[0], tuple) else (dep, None)
    if shards is None:
        return _dot(dot) + _u8(0)
    shards = sorted(shards)  # BTreeSet
    return _dot(dot) + _u8(1) + _u64(len(shards)) + b"".join(_u64(s) for s in shards)


def encode_add(dot, rifl, shard_to_ops, deps):
    """GraphExecutionInfo::Add{dot, cmd, deps} (tag 0); deps: dots or (dot, shards|None)."""
    deps = list(deps)
    return (_u32(0) + _dot(dot) + encode_command(rifl, shard_to_ops) + _u64(len(deps))
            + b"".join(_dependency(d) for d in deps))


def encode_request(from_shard, dots):
    return _u32(1) + _u64(from_shard) + _u64(len(dots)) + b"".join(_dot(d) for d in dots)


def encode_executed(dots):
    return _u32(3) + _u64(len(dots)) + b"".join(_dot(d) for d in dots)


def frame(payload):
    """LengthDelimitedCodec default framing: u32 big-endian length, then the payload."""
    return struct.pack(">I", len(payload)) + payload


def write_log(path, payloads):
    with open(path, "wb") as fh:
        for p in payloads:
            fh.write(frame(p))


# ------------------------------------------------------------------ reader
class ExecutionLog:
    """Decoded Adds of one log, in file order (numpy arrays + offsets)."""

    def __init__(self, summary, adds, keys, deps):
        self.summary = summary
        self.adds = adds
        self.keys = keys
        self.deps = deps

    def __len__(self):
        return len(self.adds)

    def __iter__(self):
        """(dot, rifl, keys, deps, read_only) per Add."""
        for a in self.adds:
            k0, d0 = int(a.key_off), int(a.dep_off)
            keys = [int(k) for k in self.keys[k0:k0 + a.nkeys]]
            deps = [(int(self.deps[i].source), int(self.deps[i].seq))
                    for i in range(d0, d0 + a.ndeps)]
            yield ((a.dot.source, a.dot.seq), (a.rifl.source, a.rifl.seq), keys, deps,
                   bool(a.read_only))


def _summary_dict(s):
    return {f: int(getattr(s, f)) for f, _ in _lib.LogSummary._fields_}


def read_log(data, shard_id=0):
    """Decodes a log (path or bytes) through fx_exec_log_scan/decode."""
    if not isinstance(data, (bytes, bytearray)):
        with open(data, "rb") as fh:
            data = fh.read()
    lib = _lib.load()
    buf = (ctypes.c_uint8 * max(len(data), 1)).from_buffer_copy(bytes(data) or b"\0")
    s = _lib.LogSummary()
    check(lib.fx_exec_log_scan(buf, len(data), shard_id, ctypes.byref(s)), "fx_exec_log_scan")
    adds = (_lib.LogAdd * max(s.adds, 1))()
    keys = np.zeros(max(s.keys, 1), dtype=np.uint32)
    deps = (_lib.CDot * max(s.deps, 1))()
    s2 = _lib.LogSummary()
    check(lib.fx_exec_log_decode(buf, len(data), shard_id, adds, s.adds,
                                 keys.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), s.keys,
                                 deps, s.deps, ctypes.byref(s2)), "fx_exec_log_decode")
    return ExecutionLog(_summary_dict(s2), list(adds)[:s.adds], keys[:s.keys], deps)


def replay(data, n, f=1, now_ms=None, monitor=True):
    """graph_executor_replay: every Add of the log into GraphExecutor(1, 0, Config::new(n, f)).

    now_ms(i) gives SysTime::millis for the i-th Add (the reference uses RunTime, the wall
    clock; default 0).  Returns the executor, whose drain_dots() / to_clients_iter() /
    metrics() / monitor() hold the replay's result."""
    log = read_log(data)
    if log.summary["others"]:
        raise _lib.FxError(_lib.FX_ERR_UNSUPPORTED, "replay: partial-replication records in log")
    ex = GraphExecutor(1, 0, n, f=f, monitor=monitor)
    for i, (dot, rifl, keys, deps, ro) in enumerate(log):
        ex.handle_add(dot, rifl, keys, deps, now_ms(i) if now_ms else 0, read_only=ro)
    return ex


def renumbering(log):
    """Per-source rank of every sequence the log names (Add dots and deps):
    {source: sorted sequences}.  A whole log is known up front, so its dots can
    be renumbered by rank, which keeps every per-source comparison the executor
    makes (AEClock frontier / membership, dot order) and fits any u32 sequence
    into the stream format's 24 bits."""
    seqs = {}
    for dot, _rifl, _keys, deps, _ro in log:
        seqs.setdefault(dot[0], set()).add(dot[1])
        for s, q in deps:
            seqs.setdefault(s, set()).add(q)
    out = {s: sorted(v) for s, v in seqs.items()}
    if any(len(v) > _lib.FX_SEQ_MASK for v in out.values()):
        raise _lib.FxError(_lib.FX_ERR_DOT_RANGE, "log_stream: more than 2^24 - 1 sequences of one source")
    return out


def log_stream(log, now_ms=None, ranks=None):
    """A decoded log as one commit stream for the batched executor: [(dot, deps,
    t_ms)], dots renumbered per source by rank (`renumbering`)."""
    import bisect
    ranks = ranks if ranks is not None else renumbering(log)

    def local(d):
        return (d[0], bisect.bisect_left(ranks[d[0]], d[1]) + 1)
    return [(local(dot), [local(d) for d in deps], now_ms(i) if now_ms else 0)
            for i, (dot, _rifl, _keys, deps, _ro) in enumerate(log)]


def replay_batch(logs, n, execute_at_commit=False):
    """Replays many logs at once: one stream per log through fx_batch_execute (the
    batched GraphExecutor), e.g. the per-process logs of one run.  Returns
    ([[dot, ...] per log in execution order], BatchResult)."""
    from . import device as fd
    from . import streams as fs
    decoded = [l if isinstance(l, ExecutionLog) else read_log(l) for l in logs]
    for l in decoded:
        if l.summary["others"]:
            raise _lib.FxError(_lib.FX_ERR_UNSUPPORTED, "replay_batch: partial-replication records")
    planes = fs.pack_streams([log_stream(l) for l in decoded], n)
    res = fd.run_batch(planes, execute_at_commit=execute_at_commit)
    check(res.status, "replay_batch")
    orders = fs.decode_orders(res.order, res.nexec, planes.S, planes.steps)
    adds = [list(l) for l in decoded]
    return [[adds[s][rec][0] for rec, _ in orders[s]] for s in range(planes.S)], res
