"""Partial replication (shard_count > 1): the oracle's restatement of
tarjan.rs:148-166 / mod.rs:277-406 / index.rs:168-202 on a hand-derived known
answer and on seeded request/reply scenarios (CPU), and the GPU executor
handle (FX_FLAG_PARTIAL on the HBM wide tables) against it step by step."""
import pytest

import partial_shapes as P


def expect_of(kat):
    return [(e["executed"], e["requests"], e["to_executors"]) for e in kat["expect"]]


def test_oracle_partial_kat():
    b = P.OracleBackend(P.KAT["n"], P.KAT["shards"], P.KAT["shard"])
    assert P.run_kat(b) == expect_of(P.KAT)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_partial_scenario_terminates(seed):
    hist, order = P.scenario(seed)
    b = P.OracleBackend(2, 2, 0)
    log = P.drive(hist, order, b, seed=seed)
    executed = [d for step in log for d in step[0]]
    requested = [d for step in log for _, d in step[1]]
    mine = {hist[i][0] for i in order}
    # every command of this shard executes exactly once; requests name only
    # commands this shard does not replicate, each once (PendingIndex::index
    # asks on the first miss only)
    assert len(executed) == len(set(executed)) and mine <= set(executed)
    assert len(requested) == len(set(requested)) and not (set(requested) & mine)
    assert requested, "the scenario should exercise out-requests"
    assert b.waits() == []


@pytest.mark.gpu
def test_gpu_partial_kat():
    b = P.GpuBackend(P.KAT["n"], P.KAT["shards"], P.KAT["shard"])
    assert P.run_kat(b) == expect_of(P.KAT)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,shards", [(1, 2, 2), (2, 2, 2), (3, 2, 3), (4, 4, 2)])
def test_gpu_partial_scenarios_match_oracle(seed, n, shards):
    hist, order = P.scenario(seed, n=n, shards=shards, shard=seed % shards)
    o = P.OracleBackend(n, shards, seed % shards)
    g = P.GpuBackend(n, shards, seed % shards)
    lo = P.drive(hist, order, o, seed=seed)
    lg = P.drive(hist, order, g, seed=seed)
    assert len(lo) == len(lg)
    for k, (a, b) in enumerate(zip(lo, lg)):
        assert a == b, k
    assert o.waits() == g.waits() == []


def test_oracle_clone_serves_requests():
    hist, order = P.scenario(5, n=2, shards=2, shard=0)
    b = P.OracleServing(2, 2, 0)
    log = P.drive_serving(hist, order, b, seed=5)
    kinds = [r[1] for step in log for r in step]
    assert "info" in kinds and "executed" in kinds
    # every request is answered once its dot is delivered (the final cleanup
    # runs after the last Add; an Info dot was pending, an Executed one executed)
    assert b.c.replies() == []


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [5, 6])
def test_gpu_clone_serves_requests_like_oracle(seed):
    hist, order = P.scenario(seed, n=2, shards=2, shard=0)
    lo = P.drive_serving(hist, order, P.OracleServing(2, 2, 0), seed=seed)
    lg = P.drive_serving(hist, order, P.GpuServing(2, 2, 0), seed=seed)
    assert len(lo) == len(lg)
    for k, (a, b) in enumerate(zip(lo, lg)):
        assert a == b, k


@pytest.mark.gpu
def test_gpu_request_from_replicating_shard_is_an_error():
    """process_requests panics when the requesting shard replicates the
    pending command (graph/mod.rs:308-316, Command::replicated_by): here an
    FX_ERR_INVALID_ARG; a request from a shard that does not replicate it gets
    an Info carrying the command's shard set (the reference ships the cmd)."""
    from fantoch_amd import _lib
    from fantoch_amd.executor import GraphExecutor
    ex = GraphExecutor(1, 0, 2, shard_count=3, monitor=False)
    # (1, 1) waits on (3, 1), a command of shard 1: it stays pending
    ex.handle_add_sharded((1, 1), (1, 1), [0], [(3, 1)], [0b010], 1, cmd_shards=0b101)
    c = ex.clone()
    c.handle_request(1, [(1, 1)])  # shard 1 does not replicate (1, 1)
    rep = c.replies(with_cmd_shards=True)
    assert [(r[0], r[1], r[2], r[4]) for r in rep] == [(1, "info", (1, 1), 0b101)]
    with pytest.raises(_lib.FxError) as e:
        c.handle_request(2, [(1, 1)])  # shard 2 replicates it
    assert e.value.status == _lib.FX_ERR_INVALID_ARG
    c.close()


@pytest.mark.gpu
def test_gpu_info_reply_feeds_back_into_requesting_shard():
    """RequestReply::Info round trip (graph/mod.rs:390-393): shard 0's clone
    answers shard 1's request for a pending command of shards {0, 2} with an
    Info carrying that shard set; shard 1's executor takes it back through
    handle_add_sharded with the set as it came (a command it does not
    replicate) and executes it exactly as the oracle does."""
    from fantoch_amd.executor import GraphExecutor
    from oracle import oracle_lib
    n = 2
    ex0 = GraphExecutor(1, 0, n, shard_count=3, monitor=False)
    # (1, 1), a command of shards {0, 2}, waits on (5, 1) of shard 2
    ex0.handle_add_sharded((1, 1), (1, 1), [0], [(5, 1)], [0b100], 1, cmd_shards=0b101)
    c = ex0.clone()
    c.handle_request(1, [(1, 1)])
    rep = c.replies(with_cmd_shards=True)
    assert [(r[0], r[1], r[2], r[4]) for r in rep] == [(1, "info", (1, 1), 0b101)]
    deps = rep[0][3]
    # shard 1 (processes 3, 4): its own command (3, 1) depends on (1, 1)
    ex1 = GraphExecutor(3, 1, n, shard_count=3, monitor=False)
    o1 = oracle_lib.Graph(3, n, shard_id=1, shard_count=3)
    steps = [("add", (3, 1), [(1, 1)], [0b101], 0b010),
             ("add", (1, 1), [d for d, _ in deps], [m for _, m in deps], rep[0][4]),  # the Info
             ("executed", (5, 1))]
    lg, lo = [], []
    for t, st in enumerate(steps, 1):
        if st[0] == "add":
            ex1.handle_add_sharded(st[1], st[1], [0], st[2], st[3], t, cmd_shards=st[4])
            o1.handle_add_sharded(st[1], st[2], st[3], t)
        else:
            ex1.handle_executed([st[1]], t)
            o1.executed_reply(st[1], t)
        lg.append(([d for d, _ in ex1.drain_dots()], ex1.requests()))
        lo.append(([d for d, _, _ in o1.drain()], o1.requests()))
    assert lg == lo
    assert (3, 1) in [d for step in lg for d in step[0]]
    ex1.close()
    c.close()
    ex0.close()
