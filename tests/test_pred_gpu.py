"""GPU predecessors executor (fx_pred_run / fx_pred_execute) vs the oracle
(oracle/pred_oracle.cpp), bit for bit: order plane, release plane, nexec,
status and the ExecutionDelay histogram.  GPU only."""
import itertools

import numpy as np
import pytest

import pred_shapes as P
from fantoch_amd import _lib
from fantoch_amd import device as fd
from oracle import oracle_lib as O

pytestmark = pytest.mark.gpu


def check(streams, n, **kw):
    planes, clo, chi, nd = P.pack_pred_streams(streams, n)
    res = fd.run_pred(planes, clo, chi, ndeps=nd, **kw)
    o_order, o_rel, o_nexec, o_err = O.pred_batch_execute(
        planes, clo, chi, threads=8, ndeps=nd, execute_at_commit=kw.get("execute_at_commit", False))
    assert res.status == (int(o_err[o_err != 0][0]) if np.any(o_err) else 0)
    assert np.array_equal(res.err, o_err)
    assert np.array_equal(res.nexec, o_nexec)
    for s in range(planes.S):
        rows = _lib.index(np.arange(int(o_nexec[s])), s, planes.steps)
        assert np.array_equal(res.order[rows], o_order[rows]), "order differs on stream %d" % s
        L = planes.steps if planes.lengths is None else int(planes.lengths[s])
        rr = _lib.index(np.arange(L), s, planes.steps)
        assert np.array_equal(res.release[rr], o_rel[rr]), "release differs on stream %d" % s
    return planes, res


def test_simple_kat():
    planes, res = check([P.SIMPLE], 2)
    order = [int(x) & 0x7FFFFFFF for x in res.order[_lib.index(np.arange(2), 0, planes.steps)]]
    assert order == P.SIMPLE_ORDER


def test_random_kat_permutations():
    streams = []
    for args in P.random_cases():
        for perm in itertools.permutations(range(len(args))):
            streams.append([(args[i][0], args[i][1], t, (args[i][2], 1)) for t, i in enumerate(perm)])
    planes, res = check(streams, 2)
    assert np.all(res.nexec == planes.lengths)


@pytest.mark.parametrize("tier", [None, 0, 1, 2])
@pytest.mark.parametrize("n,events,keys,window", [(3, 40, 8, 0), (5, 30, 16, 12), (2, 80, 4, 0), (4, 16, 32, 4)])
def test_random_streams(tier, n, events, keys, window):
    """tier None: the escalation chain; a fixed tier: streams that outgrow it
    report FX_ERR_CAPACITY (the oracle's err then differs: compared only where
    both finished)."""
    streams = P.random_streams(7, 24, n, events, keys=keys, window=window)
    if tier is None or tier == _lib.FX_PRED_TIER_HBM:
        check(streams, n, tier=tier)
        return
    planes, clo, chi, nd = P.pack_pred_streams(streams, n)
    res = fd.run_pred(planes, clo, chi, ndeps=nd, tier=tier)
    o_order, o_rel, o_nexec, o_err = O.pred_batch_execute(planes, clo, chi, threads=8, ndeps=nd)
    ok = res.err == 0
    assert np.all((res.err == 0) | (res.err == _lib.FX_ERR_CAPACITY))
    for s in np.flatnonzero(ok):
        rows = _lib.index(np.arange(int(o_nexec[s])), s, planes.steps)
        assert res.nexec[s] == o_nexec[s] and np.array_equal(res.order[rows], o_order[rows])


def test_execute_at_commit_and_errors():
    check([P.SIMPLE], 2, execute_at_commit=True)
    dup = [((1, 1), [(2, 1)], 0, (2, 1)), ((1, 1), [], 1, (3, 1))]
    planes, res = check([dup, P.SIMPLE], 2)
    assert res.err[0] == _lib.FX_ERR_DOUBLE_INDEX
    # a dot committed again after it executed (pred/mod.rs:123 asserts the
    # committed clock's add): an error, not a second execution
    again = [((1, 1), [], 0, (1, 1)), ((2, 1), [(1, 1)], 1, (2, 1)), ((1, 1), [], 2, (3, 1))]
    planes, res = check([again, P.SIMPLE], 2)
    assert res.err[0] == _lib.FX_ERR_DOUBLE_INDEX and res.nexec[0] == 2


def test_very_wide_deps():
    """~220 deps per commit: the LDS tables shrink to 128 vertices, the
    streams outgrow them and rerun on the HBM tables."""
    streams = P.random_streams(3, 8, 2, 110, keys=3, reverse_pct=80)
    planes, res = check(streams, 2)
    assert planes.dmax > 200 and res.reruns >= 8 and np.all(res.nexec == planes.lengths)


def synth_pred_case(seed=5, instances=40, cmds=100):
    """The pred bench's workload at a small size: configs[1]-shaped synthetic
    streams (n = 5, so dmax = 5), Caesar clock (seq, process id) of each dot."""
    from fantoch_amd import streams as fs
    p = fs.synth_params(seed=seed, instances=instances, n=5, cmds=cmds, window=8, cycle_pct=30,
                        conflicts=(0, 2, 10, 50, 100), conflict_block=instances // 5)
    planes = fs.synth_host(p)
    dot = planes.dot.astype(np.uint32)
    clo = ((dot & np.uint32(0xFFFFFF)) << np.uint32(8)) | ((dot >> np.uint32(24)) & np.uint32(0xFF))
    return planes, clo, np.zeros_like(clo)


@pytest.mark.parametrize("tier", [None, _lib.FX_PRED_TIER_SMALL])
def test_synth_streams_bench_shape(tier):
    """n = 5 and dmax = 5 select the SMALL tier's compiled-in layout
    (k_pred<false, 5, 5>); bit-exact with the oracle where the tier finished."""
    planes, clo, chi = synth_pred_case()
    assert planes.n == 5 and planes.dmax == 5
    res = fd.run_pred(planes, clo, chi, tier=tier)
    o_order, o_rel, o_nexec, o_err = O.pred_batch_execute(planes, clo, chi, threads=8)
    ok = res.err == 0
    assert np.all(ok | (res.err == _lib.FX_ERR_CAPACITY)) and ok.sum() > planes.S // 2
    if tier is None:
        assert np.array_equal(res.err, o_err)
    for s in np.flatnonzero(ok):
        assert res.nexec[s] == o_nexec[s]
        rows = _lib.index(np.arange(int(o_nexec[s])), s, planes.steps)
        assert np.array_equal(res.order[rows], o_order[rows]), "order differs on stream %d" % s
        rr = _lib.index(np.arange(planes.steps), s, planes.steps)
        assert np.array_equal(res.release[rr], o_rel[rr]), "release differs on stream %d" % s
