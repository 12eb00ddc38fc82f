"""The wide tiers (graph_wide.hip: the graph as LDS / HBM tables, one
wavefront per stream) vs the CPU oracle, bit for bit, and BASELINE configs[3]
(64 clients per region, 100 % conflicts, SCCs of hundreds of commands) through
the escalation chain.  GPU only."""
import itertools

import numpy as np
import pytest

import kat_shapes as K
from fantoch_amd import _lib
from fantoch_amd import device as fd
from fantoch_amd import streams as fs
from test_gpu_parity import assert_parity, kat_stream, oracle_hists

pytestmark = pytest.mark.gpu
WIDE = [_lib.FX_TIER_WIDE, _lib.FX_TIER_WIDE_HBM]


@pytest.mark.parametrize("tier", WIDE)
@pytest.mark.parametrize("case", [
    dict(n=5, instances=12, cmds=150, window=6, cycle_pct=30, conflicts=(0, 2, 10, 50, 100)),
    dict(n=3, instances=16, cmds=200, window=24, cycle_pct=60, conflicts=(100,)),
    dict(n=7, instances=6, cmds=100, window=8, cycle_pct=30, conflicts=(50, 100)),
])
def test_wide_tier_standalone(tier, case):
    planes = fs.synth_host(fs.synth_params(seed=21, **case))
    res = fd.run_batch(planes, tiered=False, tier=tier)
    assert res.status == _lib.FX_OK
    assert_parity(planes, res)


@pytest.mark.parametrize("tier", WIDE)
def test_wide_tier_kats(tier):
    streams = []
    for args in K.random_cases():
        for perm in itertools.permutations(args):
            streams.append(kat_stream(list(perm)))
    for perm in itertools.permutations(K.CYCLE["args"]):
        streams.append(kat_stream(list(perm)))
    planes = fs.pack_streams(streams, 3)
    res = fd.run_batch(planes, tiered=False, tier=tier)
    assert_parity(planes, res)
    assert np.all(res.nexec == planes.lengths)
    f = K.SCCS_MISSING
    stream = [(dot, deps, 0, _lib.FX_KIND_INDEX_ONLY) for dot, deps in f["indexed"]]
    stream.append((f["root"][0], f["root"][1], 0))
    planes = fs.pack_streams([stream], f["n"])
    front = np.zeros((1, 8), np.uint32)
    front[0, :5] = f["executed"]
    res = fd.run_batch(planes, tiered=False, tier=tier, init_frontier=front)
    assert_parity(planes, res, init_frontier=front)


def test_wide_tier_execute_at_commit():
    planes = fs.synth_host(fs.synth_params(seed=4, n=5, instances=4, cmds=50, window=6, cycle_pct=30))
    res = fd.run_batch(planes, tiered=False, tier=_lib.FX_TIER_WIDE, execute_at_commit=True)
    assert_parity(planes, res, execute_at_commit=True)


@pytest.mark.parametrize("clients,cmds,window", [(16, 320, 80), (64, 640, 320)])
def test_config3_many_clients_escalation(clients, cmds, window):
    """configs[3] shape: n = 5, C clients per process, 100 % conflicts, 30 %
    concurrent cycles: pending sets and SCCs far beyond tiers 0-2, so
    fx_batch_run_tiered escalates to the wide tier; zero capacity errors."""
    p = fs.synth_params(seed=3, instances=1, n=5, cmds=cmds, window=window, cycle_pct=30, conflicts=(100,),
                        clients=clients)
    planes = fs.synth_host(p)
    res = fd.run_batch(planes, nbins_chain=1024, nbins_delay=8192)
    assert res.status == _lib.FX_OK and np.all(res.err == 0)
    o_order, o_rel, o_nexec = assert_parity(planes, res)
    assert np.all(res.nexec == planes.steps)
    chain, delay = oracle_hists(planes, o_order, o_rel, o_nexec, 1024, 8192)
    assert np.array_equal(res.chain, chain) and np.array_equal(res.delay, delay)
    assert np.nonzero(chain)[0].max() > 5 * clients // 2  # SCCs far beyond n
    assert res.tier_counts[_lib.FX_TIER_WIDE] > 0


def test_wide_lds_index_collision_escalates():
    """The packed LDS tables index 256 seqs per source: two pending dots of one
    source 256 seqs apart share a slot, the LDS tier stops the stream with
    FX_ERR_CAPACITY and the tiered driver reruns it on the HBM tables, where
    the output equals the oracle's.  (1, 1) waits on the missing (2, 1); every
    later (1, s) depends on (1, s - 1), so (1, 1) ... (1, 257) are all pending
    when (1, 257) arrives; (2, 1) then releases the whole chain."""
    stream = [((1, 1), [(2, 1)], 0)]
    stream += [((1, s), [(1, s - 1)], s) for s in range(2, 258)]
    stream.append(((2, 1), [], 300))
    planes = fs.pack_streams([stream], 2)
    res = fd.run_batch(planes, tiered=False, tier=_lib.FX_TIER_WIDE)
    assert int(res.err[0]) == _lib.FX_ERR_CAPACITY
    res = fd.run_batch(planes, tier=_lib.FX_TIER_WIDE)
    assert res.status == _lib.FX_OK and int(res.err[0]) == 0
    assert_parity(planes, res)
    assert int(res.nexec[0]) == len(stream)
    assert res.tier_counts[_lib.FX_TIER_WIDE_HBM] == 1


def test_wide_lds_chain_one_below_the_index_span():
    """The same chain 255 seqs long fits the LDS tier's index (no collision)
    and runs there, bit-exact."""
    stream = [((1, 1), [(2, 1)], 0)]
    stream += [((1, s), [(1, s - 1)], s) for s in range(2, 257)]
    stream.append(((2, 1), [], 300))
    planes = fs.pack_streams([stream], 2)
    res = fd.run_batch(planes, tiered=False, tier=_lib.FX_TIER_WIDE)
    assert int(res.err[0]) == 0
    assert_parity(planes, res)
    assert int(res.nexec[0]) == len(stream)
