"""BASELINE configs[3] on real protocol commit streams: Atlas / EPaxos at n = 5,
64 closed-loop clients per region, 100 % conflicts.  The simulator oracle
(oracle/sim_oracle.cpp, a restatement of fantoch/src/sim + atlas.rs /
epaxos.rs) captures the Add stream each process's GraphExecutor receives;
the GPU batched executor then runs those streams, and its execution order
must equal the order the executor produced inside the simulation, process by
process (SCCs of hundreds of commands, hundreds pending).

The CPU tests check the capture itself: the standalone oracle executor over a
captured stream reproduces the simulation's order (so the captured stream is
exactly the executor's input)."""
import numpy as np
import pytest

from fantoch_amd import _lib
from fantoch_amd import sim as S
from fantoch_amd import streams as fs
from oracle import oracle_lib as O

CASES = [("atlas", 1), ("epaxos", 2)]


def capture(proto, f, cmds, seed=3):
    pl = S.Planet()
    r5 = pl.ids(S.GCP5[:5])
    p = S.ATLAS if proto == "atlas" else S.EPAXOS
    s = S.spec(p, 5, f, r5, r5, clients_per_region=64, commands_per_client=cmds, conflict_rate=100, seed=seed)
    return O.sim_capture(O.spec_from(s))


def order_dots(planes, order, nexec, s):
    k = int(nexec[s])
    o = order[_lib.index(np.arange(k), s, planes.steps)] & 0x7FFFFFFF
    return planes.dot[_lib.index(o.astype(np.int64), s, planes.steps)]


@pytest.mark.parametrize("proto,f", CASES)
def test_captured_stream_replays_to_the_sim_order(proto, f):
    streams, executed = capture(proto, f, cmds=4)
    planes = fs.pack_streams(streams, 5)
    o_order, _o_rel, o_nexec, o_err = O.batch_execute(planes, threads=5)
    assert not o_err.any()
    for p in range(5):
        assert len(executed[p]) > 0
        assert np.array_equal(order_dots(planes, o_order, o_nexec, p), executed[p]), p


@pytest.mark.gpu
@pytest.mark.parametrize("proto,f", CASES)
def test_config3_protocol_streams_on_gpu(proto, f):
    from fantoch_amd import device as fd
    streams, executed = capture(proto, f, cmds=30)
    planes = fs.pack_streams(streams, 5)
    res = fd.run_batch(planes, nbins_chain=1024, nbins_delay=8192)
    assert res.status == _lib.FX_OK and np.all(res.err == 0)
    chain_max = 0
    for p in range(5):
        assert np.array_equal(order_dots(planes, res.order, res.nexec, p), executed[p]), p
        k = int(res.nexec[p])
        starts = np.flatnonzero(res.order[_lib.index(np.arange(k), p, planes.steps)] & _lib.FX_ORDER_SCC_START)
        chain_max = max(chain_max, int(np.diff(np.append(starts, k)).max()))
    assert chain_max > 5  # SCCs far beyond n: the worst-case graph of configs[3]
    assert res.tier_counts[_lib.FX_TIER_WIDE] + res.tier_counts[_lib.FX_TIER_WIDE_HBM] > 0
