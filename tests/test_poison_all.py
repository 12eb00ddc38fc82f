"""Register poisoning for every GPU kernel, not only k_sim.

tests/test_sim_poison.py fills every SIMD's register file with garbage before
the all-on-chip simulator runs (tagged values under two tags, and zeros), so a
read of a register the kernel never wrote -- or read one wait state too soon,
round 3's k_sim defect -- returns that garbage instead of an earlier kernel's
leftovers.  The same defect class (reads of lanes or registers a kernel did not
write) bit the executor's group tier in round 2 (DESIGN.md "The fast-path bug").
Here the same fills run before:

* k_simx, the large-instance simulator: BASELINE configs[3] (64 clients per
  region, 100 % conflicts) and the reference's protocol simulations
  (fantoch_ps/src/protocol/mod.rs:702-768 sim_test, reordering, NFR);
* every batched executor tier launched standalone (group, LDS / HBM slots,
  lane, wave, lane-register, split, wide LDS / HBM tables) and the quiescent-cut
  driver;
* the predecessors executor (k_pred) on each tier;
* the persistent handle's first launch.

Each run must stay bit-exact with the oracle (graph/mod.rs:1045-1113
check_termination's contract: the same per-key order whatever ran before).
GPU only."""
import functools
import os

import numpy as np
import pytest

import pred_shapes as P
from fantoch_amd import _lib
from fantoch_amd import device as fd
from fantoch_amd import sim as S
from fantoch_amd import streams as fs
from fantoch_amd.executor import GraphExecutor
from oracle import oracle_lib as O
from test_gpu_parity import assert_parity
from test_sim_large import assert_instance_parity, planet, sim_test_specs
from test_sim_poison import FILLS, poisoner

pytestmark = pytest.mark.gpu
FILL_IDS = ["tag%02x" % t if m == 1 else "zero" for m, t in FILLS]


@functools.lru_cache(maxsize=None)
def _oracle_sim(key):
    specs = _SIM_CASES[key]()
    return specs, O.sim_batch([O.spec_from(s) for s in specs], threads=8)


def _config3(protocol, f):
    def make():
        regs = sorted(planet().ids(S.GCP5))
        return [S.spec(protocol, 5, f, regs, regs, clients_per_region=64, commands_per_client=20,
                       conflict_rate=100, seed=12, instance=i) for i in range(2)]
    return make


_SIM_CASES = {
    "config3_atlas": _config3(S.ATLAS, 1),
    "config3_epaxos": _config3(S.EPAXOS, 2),
    "sim_atlas_5_2": lambda: sim_test_specs(S.ATLAS, 5, 2, seeds=(3,)),
    "sim_atlas_5_2_nfr": lambda: sim_test_specs(S.ATLAS, 5, 2, 20, 1, True, seeds=(3,)),
    "sim_epaxos_5_2": lambda: sim_test_specs(S.EPAXOS, 5, 2, seeds=(3,)),
    "sim_epaxos_7_3_nfr": lambda: sim_test_specs(S.EPAXOS, 7, 3, 100, 1, True, seeds=(3,)),
}


# k_simx launch variants: the default launch, its arena filled with 0xA5 bytes
# instead of zeroed (FX_SIM_FLAG_ARENA_FILL: the kernel must initialise every
# arena word it reads), and the run-time-geometry build for
# the shapes that otherwise run the configs[3] build (FX_SIM_FLAG_GENERIC)
_SIMX_VARIANTS = {"default": {}, "arena_fill": dict(arena_fill=True), "generic": dict(generic=True)}


@pytest.mark.parametrize("variant", sorted(_SIMX_VARIANTS))
@pytest.mark.parametrize("fill", FILLS, ids=FILL_IDS)
@pytest.mark.parametrize("case", sorted(_SIM_CASES))
def test_poisoned_k_simx(case, fill, variant):
    if variant == "generic" and not case.startswith("config3"):
        pytest.skip("the sim_test shapes run the generic build already")
    specs, orc = _oracle_sim(case)
    res = S.run(specs, planet(), large=True, before_launch=poisoner(*fill), **_SIMX_VARIANTS[variant])
    bad = ["instance %d err %d site %d events %d" % (i, int(e), int(res.stats[i, _lib.FX_SIM_STAT_ERR_SITE]),
                                                    res.events(i)) for i, e in enumerate(res.err) if e]
    assert not bad, "instances failed under fill %s: %s" % (fill, "; ".join(bad))
    for i, (s, o) in enumerate(zip(specs, orc)):
        assert_instance_parity(res, i, s, o)
    assert np.array_equal(res.chain, sum(o["chain"] for o in orc)[:res.chain.shape[0]])
    assert np.array_equal(res.delay, sum(o["delay"] for o in orc)[:res.delay.shape[0]])


_EXEC_CASES = {
    "mixed": dict(seed=9, n=5, instances=20, cmds=150, window=6, cycle_pct=30),
    "dense": dict(seed=21, n=3, instances=16, cmds=200, window=24, cycle_pct=60, conflicts=(100,)),
}


@functools.lru_cache(maxsize=None)
def _planes(case):
    return fs.synth_host(fs.synth_params(**_EXEC_CASES[case]))


@pytest.mark.parametrize("fill", FILLS, ids=FILL_IDS)
@pytest.mark.parametrize("tier", [0, 1, 2, 3, 4, 5, 6, _lib.FX_TIER_WIDE, _lib.FX_TIER_WIDE_HBM])
def test_poisoned_executor_tiers(tier, fill):
    case = "dense" if tier in (_lib.FX_TIER_WIDE, _lib.FX_TIER_WIDE_HBM) else "mixed"
    planes = _planes(case)
    res = fd.run_batch(planes, tiered=False, tier=tier, before_launch=poisoner(*fill))
    assert_parity(planes, res)


@pytest.mark.parametrize("fill", FILLS, ids=FILL_IDS)
def test_poisoned_escalation_and_cut(fill):
    """The tiered driver (first launch poisoned, reruns after it) and the
    quiescent-cut driver of configs[4] on a cycle-heavy stream."""
    planes = _planes("dense")
    assert_parity(planes, fd.run_batch(planes, before_launch=poisoner(*fill)))
    huge = fs.synth_host(fs.synth_params(seed=3, n=5, instances=1, cmds=4000, window=8, cycle_pct=30,
                                         conflicts=(2,)))
    res = fd.run_batch(huge, cut=True, before_launch=poisoner(*fill))
    assert res.status == _lib.FX_OK
    assert_parity(huge, res)


@pytest.mark.parametrize("fill", FILLS, ids=FILL_IDS)
@pytest.mark.parametrize("tier", [None, _lib.FX_PRED_TIER_SMALL, _lib.FX_PRED_TIER_LDS, _lib.FX_PRED_TIER_HBM])
def test_poisoned_pred(tier, fill):
    # test_pred_gpu.py::test_random_streams' sparse shape (n = 4, 16 events, 32 keys):
    # a fixed tier may stop a stream with FX_ERR_CAPACITY; the rest must match
    streams = P.random_streams(7, 24, 4, 16, keys=32, window=4)
    planes, clo, chi, nd = P.pack_pred_streams(streams, 4)
    res = fd.run_pred(planes, clo, chi, ndeps=nd, tier=tier, before_launch=poisoner(*fill))
    o_order, o_rel, o_nexec, o_err = O.pred_batch_execute(planes, clo, chi, threads=8, ndeps=nd)
    ok = res.err == 0
    if tier is None:
        assert np.all(ok)
    assert np.all(ok | (res.err == _lib.FX_ERR_CAPACITY))
    assert np.array_equal(res.err[ok], o_err[ok]) and ok.sum() > 0
    for s in np.flatnonzero(ok):
        assert res.nexec[s] == o_nexec[s]
        rows = _lib.index(np.arange(int(o_nexec[s])), s, planes.steps)
        assert np.array_equal(res.order[rows], o_order[rows]), "order differs on stream %d" % s
        L = planes.steps if planes.lengths is None else int(planes.lengths[s])
        rr = _lib.index(np.arange(L), s, planes.steps)
        assert np.array_equal(res.release[rr], o_rel[rr]), "release differs on stream %d" % s


@pytest.mark.parametrize("fill", FILLS, ids=FILL_IDS)
def test_poisoned_pred_compiled_layout(fill):
    """The bench's shape (n = 5, dmax = 5): the SMALL tier's compiled-in layout."""
    from test_pred_gpu import synth_pred_case
    planes, clo, chi = synth_pred_case(seed=6)
    res = fd.run_pred(planes, clo, chi, tier=_lib.FX_PRED_TIER_SMALL, before_launch=poisoner(*fill))
    o_order, o_rel, o_nexec, o_err = O.pred_batch_execute(planes, clo, chi, threads=8)
    ok = res.err == 0
    assert np.all(ok | (res.err == _lib.FX_ERR_CAPACITY)) and ok.sum() > planes.S // 2
    for s in np.flatnonzero(ok):
        rows = _lib.index(np.arange(int(o_nexec[s])), s, planes.steps)
        assert res.nexec[s] == o_nexec[s] and np.array_equal(res.order[rows], o_order[rows])


@pytest.mark.parametrize("fill", FILLS, ids=FILL_IDS)
def test_poisoned_persistent_handle_first_launch(fill):
    """The register file is poisoned on the null stream right before the
    handle's first pull; the handle's stream is a blocking one, so its
    resident kernel starts after the fill (and fresh from `init`)."""
    p = fs.synth_params(seed=44, n=5, instances=1, cmds=80, window=8, cycle_pct=30, conflicts=(50,))
    st = fs.synth_host(p).stream(0)[:300]
    g = O.Graph(1, 5)
    for (dot, deps, t, _kind) in st:
        g.handle_add(dot, deps, t)
    exp = [d for d, _, _ in g.drain()]
    h = GraphExecutor(1, 0, 5, monitor=False)
    out = []
    for i, (dot, deps, t, _kind) in enumerate(st):
        h.handle_add(dot, dot, [0], deps, t)
        if i == 0:
            poisoner(*fill)(None)
        out += [d for d, _ in h.drain_dots()]
    h.close()
    assert out == exp
