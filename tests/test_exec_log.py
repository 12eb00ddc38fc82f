"""Execution-log reader: bincode-1 GraphExecutionInfo
frames as written by execution_logger_task and replayed by
graph_executor_replay (fantoch_ps/src/bin/graph_executor_replay.rs:13-38).

The reference holds no execution-log files, so the byte layout is pinned by a
hand-assembled frame (bincode 1.3.3 default options + LengthDelimitedCodec
defaults) and the replay by the oracle: parity of real logs is unpinned."""
import struct

import pytest

from fantoch_amd import _lib
from fantoch_amd import exec_log as L
from fantoch_amd import streams as fs
from oracle import oracle_lib
import kat_shapes as K


def test_add_bytes_match_bincode_layout():
    # Add{dot:(1,1), cmd:{rifl:(7,9), {0:{"A":[Get]}}}, deps:{((2,1), None)}}
    got = L.frame(L.encode_add((1, 1), (7, 9), {0: {"A": [L.GET]}}, [(2, 1)]))
    exp = bytes.fromhex(
        "00000000"                      # variant Add
        "01" "0100000000000000"         # dot (u8 source, u64 seq)
        "0700000000000000" "0900000000000000"  # rifl
        "0100000000000000"              # shard_to_ops: 1 shard
        "0000000000000000" "0100000000000000"  # shard 0, 1 key
        "0100000000000000" "41"         # "A"
        "0100000000000000" "00000000"   # Arc<Vec<KVOp>> = [Get]
        "0100000000000000" "0000000000000000" "0100000000000000" "0100000000000000" "41"
        "0000000000000000"              # _empty_keys
        "0100000000000000"              # deps: 1
        "02" "0100000000000000" "00")   # Dependency{dot:(2,1), shards: None}
    assert got == struct.pack(">I", len(exp)) + exp


def test_roundtrip_fields_and_interning():
    payloads = [
        L.encode_add((1, 1), (10, 1), {0: {"x": [L.put("v")], "y": [L.GET]}, 1: {"z": [L.GET]}},
                     [(2, 3), ((3, 4), {0, 1})]),
        L.encode_request(1, [(1, 1)]),
        L.encode_add((2, 5), (11, 2), {0: {"y": [L.GET]}}, []),
        L.encode_executed([(1, 1), (2, 5)]),
        L.encode_add((3, 2**32 - 1), (12, 3), {0: {"x": [L.DELETE]}}, [(1, 1)]),
    ]
    log = L.read_log(b"".join(L.frame(p) for p in payloads))
    assert log.summary == {"records": 5, "adds": 3, "others": 2, "keys": 4, "deps": 3,
                           "distinct_keys": 2}
    got = list(log)
    assert got[0] == ((1, 1), (10, 1), [0, 1], [(2, 3), (3, 4)], False)
    assert got[1] == ((2, 5), (11, 2), [1], [], True)
    assert got[2] == ((3, 2**32 - 1), (12, 3), [0], [(1, 1)], False)
    # the keys of another shard
    log1 = L.read_log(b"".join(L.frame(p) for p in payloads), shard_id=1)
    assert [k for _, _, k, _, _ in log1] == [[0], [], []]


def test_empty_log():
    log = L.read_log(b"")
    assert len(log) == 0 and log.summary["records"] == 0


@pytest.mark.parametrize("mutate", ["truncated", "trailing", "bad_tag", "bad_op", "seq_range",
                                    "bad_option"])
def test_malformed_logs_are_rejected(mutate):
    good = L.encode_add((1, 1), (1, 1), {0: {"A": [L.GET]}}, [(2, 1)])
    if mutate == "truncated":
        data = L.frame(good)[:-1]
    elif mutate == "trailing":
        data = L.frame(good + b"\0")
    elif mutate == "bad_tag":
        data = L.frame(b"\x04\0\0\0")
    elif mutate == "bad_op":
        data = L.frame(good.replace(b"\x41" + b"\x01" + b"\0" * 7 + b"\0\0\0\0",
                                    b"\x41" + b"\x01" + b"\0" * 7 + b"\x09\0\0\0", 1))
    elif mutate == "seq_range":
        data = L.frame(L.encode_add((1, 2**32), (1, 1), {}, []))
    else:
        data = L.frame(good[:-1] + b"\x02")
    with pytest.raises(_lib.FxError) as e:
        L.read_log(data)
    assert e.value.status == _lib.FX_ERR_LOG_FORMAT


def synth_log(seed=3, n=3, cmds=120):
    """A log of one synthetic commit stream (with cycles and missing deps)."""
    p = fs.synth_params(seed=seed, n=n, instances=1, cmds=cmds, window=8, cycle_pct=40)
    stream = fs.synth_host(p).stream(1)
    payloads = []
    for i, (dot, deps, t, _kind) in enumerate(stream):
        key = "CONFLICT0" if i % 3 else "client%d" % dot[0]
        payloads.append(L.encode_add(dot, (dot[0], dot[1]), {0: {key: [L.put("v")]}},
                                     [(d, None) for d in deps]))
    return stream, b"".join(L.frame(x) for x in payloads)


def test_decoded_stream_matches_the_source_stream():
    stream, data = synth_log()
    log = L.read_log(data)
    assert [(d, sorted(deps)) for d, _, _, deps, _ in log] == \
        [(dot, sorted(deps)) for dot, deps, _, _ in stream]
    # the oracle executes the decoded log exactly like the source stream
    g1, g2 = oracle_lib.Graph(1, 3), oracle_lib.Graph(1, 3)
    for (dot, _, _, deps, _), (_, sdeps, _, _) in zip(log, stream):
        g1.handle_add(dot, sorted(deps))
        g2.handle_add(dot, sdeps)
    assert g1.drain() == g2.drain()


@pytest.mark.gpu
def test_replay_simple_kat(gpu):  # graph/mod.rs:714-752 as a log
    payloads = [L.encode_add(dot, dot, {0: {"A": [L.GET]}}, deps) for dot, deps in K.SIMPLE["adds"]]
    ex = L.replay(b"".join(L.frame(p) for p in payloads), K.SIMPLE["n"], 1)
    assert [d for d, _ in ex.drain_dots()] == K.SIMPLE["ready_after"][-1]


@pytest.mark.gpu
def test_replay_matches_oracle(gpu):
    stream, data = synth_log(seed=11, n=5, cmds=200)
    ex = L.replay(data, 5, 2)
    g = oracle_lib.Graph(1, 5)
    for dot, deps, _, _ in stream:
        g.handle_add(dot, deps)
    assert [d for d, _ in ex.drain_dots()] == [d for d, _, _ in g.drain()]


@pytest.mark.gpu
def test_replay_refuses_partial_replication_records(gpu):
    data = L.frame(L.encode_executed([(1, 1)]))
    with pytest.raises(_lib.FxError) as e:
        L.replay(data, 3)
    assert e.value.status == _lib.FX_ERR_UNSUPPORTED


@pytest.mark.gpu
def test_replay_batch_matches_single_replay_and_oracle(gpu):
    logs, exp = [], []
    for seed, n in ((5, 3), (6, 3), (7, 3)):
        stream, data = synth_log(seed=seed, n=n, cmds=150)
        logs.append(data)
        g = oracle_lib.Graph(1, n)
        for dot, deps, _, _ in stream:
            g.handle_add(dot, deps)
        exp.append([d for d, _, _ in g.drain()])
    got, res = L.replay_batch(logs, 3)
    assert (res.err == 0).all()
    assert got == exp
    assert got[0] == [d for d, _ in L.replay(logs[0], 3).drain_dots()]


def stretched_log(seed, n, cmds):
    """synth_log with every sequence s mapped to 2^31 + 7919 s (gaps, and far
    beyond the stream format's 24 bits)."""
    stream, _ = synth_log(seed=seed, n=n, cmds=cmds)
    big = lambda d: (d[0], 2**31 + 7919 * d[1])
    payloads = [L.encode_add(big(dot), (dot[0], dot[1]), {0: {"k": [L.GET]}}, [(big(d), None) for d in deps])
                for dot, deps, _, _ in stream]
    return stream, big, b"".join(L.frame(x) for x in payloads)


def test_log_renumbering_preserves_the_execution_order():
    """Rank renumbering per source (log_stream) executes exactly like the
    original sequences: the oracle over both, mapped back."""
    stream, big, data = stretched_log(8, 3, 150)
    log = L.read_log(data)
    ranks = L.renumbering(log)
    local = L.log_stream(log, ranks=ranks)
    assert max(q for (_, q), _, _ in local) < 2**24
    g1, g2 = oracle_lib.Graph(1, 3), oracle_lib.Graph(1, 3)
    for (dot, deps, _, _), (ldot, ldeps, _) in zip(stream, local):
        g1.handle_add(dot, deps)
        g2.handle_add(ldot, sorted(ldeps))
    back = lambda d: (d[0], (ranks[d[0]][d[1] - 1] - 2**31) // 7919)
    assert [back(d) for d, _, _ in g2.drain()] == [d for d, _, _ in g1.drain()]


@pytest.mark.gpu
def test_replay_batch_of_u32_sequences(gpu):
    stream, big, data = stretched_log(9, 3, 150)
    g = oracle_lib.Graph(1, 3)
    for dot, deps, _, _ in stream:
        g.handle_add(dot, deps)
    got, res = L.replay_batch([data], 3)
    assert (res.err == 0).all()
    assert got[0] == [big(d) for d, _, _ in g.drain()]
