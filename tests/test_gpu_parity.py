"""Parity of the HIP path (through the C-ABI) with the CPU oracle.  GPU only.

Integer/index work: everything is compared bit-exactly — the order plane
(executed arrival index + SCC-start flag, row by row), the release plane,
nexec and the per-stream status — on the same seeded inputs."""
import os
import subprocess

import numpy as np
import pytest

import kat_shapes as K
from fantoch_amd import _lib
from fantoch_amd import device as fd
from fantoch_amd import streams as fs
from fantoch_amd.executor import GraphExecutor, CHAIN_SIZE, EXECUTION_DELAY
from oracle import oracle_lib

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def valid_rows(order, nexec, S, steps):
    idx = []
    for s in range(S):
        idx.append(_lib.index(np.arange(int(nexec[s])), s, steps))
    return np.concatenate(idx) if idx else np.zeros(0, np.int64)


def release_rows(lengths, S, steps):
    idx = []
    for s in range(S):
        L = steps if lengths is None else int(lengths[s])
        idx.append(_lib.index(np.arange(L), s, steps))
    return np.concatenate(idx) if idx else np.zeros(0, np.int64)


def assert_parity(planes, res, execute_at_commit=False, init_frontier=None):
    o_order, o_rel, o_nexec, o_err = oracle_lib.batch_execute(
        planes, execute_at_commit=execute_at_commit, init_frontier=init_frontier, threads=8)
    assert np.array_equal(res.err, o_err), (np.unique(res.err), np.unique(o_err))
    assert np.array_equal(res.nexec, o_nexec)
    rows = valid_rows(res.order, res.nexec, planes.S, planes.steps)
    assert np.array_equal(res.order[rows], o_order[rows])
    rrows = release_rows(planes.lengths, planes.S, planes.steps)
    assert np.array_equal(res.release[rrows], o_rel[rrows])
    return o_order, o_rel, o_nexec


def oracle_hists(planes, order, release, nexec, nbc, nbd):
    chain = np.zeros(nbc, np.uint64)
    delay = np.zeros(nbd, np.uint64)
    t = planes.hdr & 0xFFFFFF
    for s in range(planes.S):
        k = int(nexec[s])
        if not k:
            continue
        o = order[_lib.index(np.arange(k), s, planes.steps)]
        rec = (o & 0x7FFFFFFF).astype(np.int64)
        start = (o & _lib.FX_ORDER_SCC_START) != 0
        rel = release[_lib.index(rec, s, planes.steps)].astype(np.int64)
        d = t[_lib.index(rel, s, planes.steps)].astype(np.int64) - t[_lib.index(rec, s, planes.steps)]
        np.add.at(delay, np.minimum(d, nbd - 1), 1)
        starts = np.flatnonzero(start)
        sizes = np.diff(np.append(starts, k))
        np.add.at(chain, np.minimum(sizes, nbc - 1), 1)
    return chain, delay


# ------------------------------------------------------------ synthetic
SYNTH_CASES = [
    dict(n=5, instances=40, cmds=200, window=8, cycle_pct=30),
    dict(n=3, instances=64, cmds=150, window=6, cycle_pct=50),
    dict(n=7, instances=20, cmds=120, window=8, cycle_pct=30),
    dict(n=5, instances=16, cmds=100, window=0, cycle_pct=0),
    dict(n=5, instances=16, cmds=300, window=24, cycle_pct=60),  # deep pending: tier reruns
    dict(n=2, instances=33, cmds=77, window=5, cycle_pct=40),   # ragged tile (S % 64 != 0)
]


@pytest.mark.parametrize("case", SYNTH_CASES)
def test_synthetic_parity(gpu, case):
    p = fs.synth_params(seed=11, **case)
    planes = fs.synth_host(p)
    res = fd.run_batch(planes, nbins_chain=64, nbins_delay=2048)
    o_order, o_rel, o_nexec = assert_parity(planes, res)
    assert res.status == _lib.FX_OK
    assert np.all(res.nexec == planes.steps)  # complete streams execute everything
    chain, delay = oracle_hists(planes, o_order, o_rel, o_nexec, 64, 2048)
    assert np.array_equal(res.chain, chain)
    assert np.array_equal(res.delay, delay)


@pytest.mark.parametrize("case", SYNTH_CASES)
def test_synthetic_parity_lane_reg_first(gpu, case):
    """Tier 5 (register slot table) as the first tier, reruns 5 -> 1 -> 2."""
    p = fs.synth_params(seed=12, **case)
    planes = fs.synth_host(p)
    res = fd.run_batch(planes, tier=_lib.FX_TIER_LANE_REG, nbins_chain=64, nbins_delay=2048)
    o_order, o_rel, o_nexec = assert_parity(planes, res)
    assert res.status == _lib.FX_OK
    chain, delay = oracle_hists(planes, o_order, o_rel, o_nexec, 64, 2048)
    assert np.array_equal(res.chain, chain)
    assert np.array_equal(res.delay, delay)


def test_tier_reruns_happen_and_match(gpu):
    p = fs.synth_params(seed=5, n=5, instances=10, cmds=300, window=40, cycle_pct=70,
                        conflicts=(100,))
    planes = fs.synth_host(p)
    res = fd.run_batch(planes, tier=0)
    assert res.tier_counts[0] == planes.S
    assert res.tier_counts[1] > 0, res.tier_counts  # the group tier overflowed: reruns
    assert_parity(planes, res)


def test_capacity_escalates_past_64_pending(gpu):
    """Streams that need more than 64 pending vertices (the ceiling of tiers
    0-6) escalate to the wide tiers (1024 / 16384 pending) and execute exactly
    like the oracle; nothing stops on FX_ERR_CAPACITY."""
    p = fs.synth_params(seed=5, n=5, instances=10, cmds=300, window=120, cycle_pct=70,
                        conflicts=(100, 50))
    planes = fs.synth_host(p)
    res = fd.run_batch(planes, metrics=False)
    o_order, o_rel, o_nexec, o_err, mp, _ = oracle_lib.batch_execute(planes, threads=8, stats=True)
    assert (mp > 64).any() and (mp < 64).any()
    assert np.all(res.err == 0) and np.all(o_err == 0)
    assert res.tier_counts[_lib.FX_TIER_WIDE] + res.tier_counts[_lib.FX_TIER_WIDE_HBM] >= int((mp > 64).sum())
    for s in range(planes.S):
        idx = _lib.index(np.arange(int(o_nexec[s])), s, planes.steps)
        assert res.nexec[s] == o_nexec[s]
        assert np.array_equal(res.order[idx], o_order[idx])
        ridx = _lib.index(np.arange(planes.steps), s, planes.steps)
        assert np.array_equal(res.release[ridx], o_rel[ridx])


@pytest.mark.parametrize("tier", [0, 1, 2, 3, 4, 5, 6])
def test_each_tier_standalone(gpu, tier):
    p = fs.synth_params(seed=9, n=5, instances=20, cmds=150, window=6, cycle_pct=30)
    planes = fs.synth_host(p)
    res = fd.run_batch(planes, tiered=False, tier=tier)
    assert_parity(planes, res)


@pytest.mark.parametrize("block,instances,n", [(16, 80, 5), (13, 57, 3), (1, 40, 7)])
def test_split_tier_mixed_tiles(gpu, block, instances, n):
    """FX_TIER_SPLIT over conflict-major batches (tiles of one rate, tiles
    straddling two rates, a ragged last tile): sparse tiles run on the lane
    tier, dense ones on the group tier, concurrently; bit-exact either way."""
    p = fs.synth_params(seed=31, n=n, instances=instances, cmds=120, window=8, cycle_pct=30,
                        conflicts=(0, 100, 2, 50, 10), conflict_block=block)
    planes = fs.synth_host(p)
    res = fd.run_batch(planes, tiered=False, tier=_lib.FX_TIER_SPLIT, nbins_chain=64,
                       nbins_delay=2048)
    ok = res.err == 0
    assert ok.sum() > planes.S // 2  # capacity stops are allowed, results must still match
    o_order, o_rel, o_nexec, o_err = oracle_lib.batch_execute(planes, threads=8)
    for s in np.flatnonzero(ok):
        idx = _lib.index(np.arange(int(o_nexec[s])), s, planes.steps)
        assert res.nexec[s] == o_nexec[s]
        assert np.array_equal(res.order[idx], o_order[idx])
        ridx = _lib.index(np.arange(planes.steps), s, planes.steps)
        assert np.array_equal(res.release[ridx], o_rel[ridx])
    assert np.all(res.err[~ok] == _lib.FX_ERR_CAPACITY)
    # k_metrics over a batch with errored streams: order-major for those, record-major
    # for the rest; same histograms as the host fold of the GPU's own order/release
    chain, delay = oracle_hists(planes, res.order, res.release, res.nexec, 64, 2048)
    assert np.array_equal(res.chain, chain) and np.array_equal(res.delay, delay)
    tiered = fd.run_batch(planes, tier=_lib.FX_TIER_SPLIT, nbins_chain=64, nbins_delay=2048)
    assert tiered.status == _lib.FX_OK
    assert_parity(planes, tiered)


def test_device_generator_matches_host(gpu):
    import ctypes
    p = fs.synth_params(seed=123, n=5, instances=70, cmds=64, window=8, cycle_pct=30)
    host = fs.synth_host(p)
    lib = _lib.load()
    bufs = [fd.DeviceBuffer(a.nbytes) for a in (host.dot, host.hdr, host.deps)]
    _lib.check(lib.fx_synth_generate(ctypes.byref(p), bufs[0].ptr, bufs[1].ptr, bufs[2].ptr, None))
    for b, a in zip(bufs, (host.dot, host.hdr, host.deps)):
        assert np.array_equal(b.download(np.uint32, a.size), a)


def test_execute_at_commit(gpu):
    p = fs.synth_params(seed=3, n=3, instances=8, cmds=50, window=8)
    planes = fs.synth_host(p)
    res = fd.run_batch(planes, execute_at_commit=True)
    assert_parity(planes, res, execute_at_commit=True)


def test_ragged_lengths_and_truncated_streams(gpu):
    p = fs.synth_params(seed=21, n=5, instances=30, cmds=100, window=8, cycle_pct=30)
    planes = fs.synth_host(p)
    rng = np.random.default_rng(0)
    planes.lengths = rng.integers(0, planes.steps + 1, planes.S).astype(np.uint32)
    planes.lengths[0] = 0  # empty stream
    res = fd.run_batch(planes, nbins_chain=64, nbins_delay=2048)
    o_order, o_rel, o_nexec = assert_parity(planes, res)
    chain, delay = oracle_hists(planes, o_order, o_rel, o_nexec, 64, 2048)
    assert np.array_equal(res.chain, chain) and np.array_equal(res.delay, delay)


@pytest.mark.parametrize("tier", [0, 1, 2, 3, 4, 5])
def test_chunked_resume_equals_one_shot(gpu, tier):
    import ctypes
    p = fs.synth_params(seed=8, n=5, instances=30, cmds=100, window=10, cycle_pct=30)
    planes = fs.synth_host(p)
    one = fd.run_batch(planes, tiered=False, tier=tier, metrics=False)
    lib = _lib.load()
    S, steps, pw = planes.S, planes.steps, planes.plane
    d = [fd.DeviceBuffer(a.nbytes) for a in (planes.dot, planes.hdr, planes.deps)]
    for b, a in zip(d, (planes.dot, planes.hdr, planes.deps)):
        b.upload(a)
    order, release = fd.DeviceBuffer(pw * 4), fd.DeviceBuffer(pw * 4)
    nexec, err = fd.DeviceBuffer(S * 4), fd.DeviceBuffer(S * 4)
    state = fd.DeviceBuffer(lib.fx_batch_state_bytes(tier, 5, S))
    inb = _lib.StreamBatch(d[0].ptr, d[1].ptr, d[2].ptr, None, S, steps, planes.dmax, 5)
    outb = _lib.OrderBatch(order.ptr, release.ptr, nexec.ptr, err.ptr)
    cuts = [0, 1, 7, 64, 65, 200, 333, steps]
    for a, b in zip(cuts[:-1], cuts[1:]):
        flags = _lib.FX_FLAG_SAVE_STATE | (_lib.FX_FLAG_INIT if a == 0 else 0)
        _lib.check(lib.fx_batch_execute(ctypes.byref(inb), ctypes.byref(outb), tier, None, S,
                                        state.ptr, a, b, flags, None, None))
    ne = nexec.download(np.uint32, S)
    er = err.download(np.uint32, S)
    assert np.array_equal(ne, one.nexec)
    assert np.array_equal(er, one.err)
    rows = valid_rows(None, ne, S, steps)
    assert np.array_equal(order.download(np.uint32, pw)[rows], one.order[rows])
    # release rows are defined for the arrivals a stream processed; a stream
    # that stopped at the tier-0 capacity leaves the rest undefined
    ok = np.flatnonzero(er == 0)
    assert len(ok) > S // 2
    rrows = np.concatenate([_lib.index(np.arange(steps), s, steps) for s in ok])
    assert np.array_equal(release.download(np.uint32, pw)[rrows], one.release[rrows])


# ------------------------------------------- the reference's KATs as streams
def kat_stream(args, t0=0):
    return [(dot, sorted(deps), t0 + t) for t, (dot, _keys, deps) in enumerate(args)]


def test_kat_permutations_as_one_batch(gpu):
    import itertools
    streams, n_of = [], []
    for args in K.random_cases():
        for perm in itertools.permutations(args):
            streams.append(kat_stream(list(perm)))
    for perm in itertools.permutations(K.CYCLE["args"]):
        streams.append(kat_stream(list(perm)))
    planes = fs.pack_streams(streams, 3)
    res = fd.run_batch(planes)
    assert_parity(planes, res)
    assert np.all(res.nexec == planes.lengths)


def test_sccs_found_and_missing_dep_batch(gpu):
    f = K.SCCS_MISSING
    stream = [(dot, deps, 0, _lib.FX_KIND_INDEX_ONLY) for dot, deps in f["indexed"]]
    stream.append((f["root"][0], f["root"][1], 0))
    planes = fs.pack_streams([stream], f["n"])
    front = np.zeros((1, 8), np.uint32)
    front[0, :5] = f["executed"]
    res = fd.run_batch(planes, tiered=False, tier=0, init_frontier=front)
    assert_parity(planes, res, init_frontier=front)
    order = fs.decode_orders(res.order, res.nexec, 1, planes.steps)[0]
    assert [rec for rec, _ in order] == list(range(10))  # (4,31)..(4,40)
    assert all(start for _, start in order)


# ------------------------------------- single executor (Executor trait)
class GpuExec:
    def __init__(self, n):
        self.ex = GraphExecutor(1, 0, n, monitor=True)

    def handle_add(self, dot, deps, t):
        self.ex.handle_add(dot, dot, [0], deps, t)

    def drain(self):
        return [d for d, _ in self.ex.drain_dots()]


def make_gpu(n):
    return GpuExec(n)


def test_executor_simple(gpu):
    ex = GraphExecutor(1, 0, 2)
    ex.handle_add((1, 1), (1, 1), [0], [(2, 1)], 0)
    assert ex.drain_dots() == []
    ex.handle_add((2, 1), (2, 1), [0], [(1, 1)], 0)
    assert ex.drain_dots() == [((1, 1), True), ((2, 1), False)]


def test_executor_cycle(gpu):
    K.shuffle_it(make_gpu, K.CYCLE["n"], K.CYCLE["args"])


def test_executor_regressions(gpu):
    for case in (K.REGRESSION_1, K.REGRESSION_2):
        # keys matter for regression 2: use the monitor path (per-key order)
        def run(args):
            ex = GraphExecutor(1, 0, case["n"], monitor=True)
            ids = {"A": 1, "B": 2, K.CONF: 0}
            for t, (dot, keys, deps) in enumerate(args):
                ex.handle_add(dot, dot, [ids[k] for k in (keys or [K.CONF])], sorted(deps), t)
            ex.to_clients_iter()
            return {k: ex.monitor(k) for k in (0, 1, 2)}
        assert run(case["order_a"]) != run(case["order_b"])


def test_executor_sccs_found_and_missing_dep(gpu):
    f = K.SCCS_MISSING
    ex = GraphExecutor(f["process_id"], 0, f["n"])
    ex.set_executed_frontier(f["executed"])
    for dot, deps in f["indexed"]:
        ex.index_only(dot, (1, 1), [0], deps)
    ex.handle_add(f["root"][0], (1, 1), [0], f["root"][1], 0)
    assert ex.drain_dots() == [((4, s), True) for s in range(31, 41)]
    assert ex.pending() == [(f["root"][0], f["missing"][0])]


def test_executor_metrics_and_results_match_oracle(gpu):
    p = fs.synth_params(seed=4, n=3, instances=1, cmds=200, window=8, cycle_pct=40)
    planes = fs.synth_host(p)
    stream = planes.stream(1)
    ex = GraphExecutor(2, 0, 3, monitor=True)
    g = oracle_lib.Graph(2, 3)
    for i, (dot, deps, t, _kind) in enumerate(stream):
        ex.handle_add(dot, dot, [0 if i % 3 else 1], deps, 1_700_000_000_000 + t)
        g.handle_add(dot, deps, t)
        if i % 17 == 0:  # pull results mid-stream too (resume path)
            ex.to_clients_iter()
    got = [d for d, _ in ex.drain_dots()]
    exp = [d for d, _, _ in g.drain()]
    assert got == exp
    assert ex.metrics(CHAIN_SIZE) == g.metrics(1)
    assert ex.metrics(EXECUTION_DELAY) == g.metrics(0)


def test_executor_wide_adds_match_oracle(gpu):
    """Adds with 17-31 deps (beyond the group tier's 16 lanes) must not poison
    the handle: it starts such a log one tier up (executor_host.cpp)."""
    n = 8
    ex = GraphExecutor(1, 0, n, monitor=True)
    g = oracle_lib.Graph(1, n)
    rng = np.random.default_rng(17)
    seqs = {p: 0 for p in range(1, n + 1)}
    issued = []
    for i in range(300):
        src = int(rng.integers(1, n + 1))
        seqs[src] += 1
        dot = (src, seqs[src])
        # wide Adds: up to 27 old deps (long executed: ignored by every search,
        # tarjan.rs:128-145) plus up to 4 recent ones that may still be pending
        old_pool = issued[:-40]
        recent = [d for d in issued[-40:] if d != dot]
        k = int(rng.integers(0, min(len(old_pool), 27) + 1)) if i % 5 else min(len(old_pool), 24)
        deps = [old_pool[j] for j in rng.choice(len(old_pool), size=k, replace=False)] if k else []
        r = int(rng.integers(0, min(len(recent), 4) + 1))
        deps += [recent[j] for j in rng.choice(len(recent), size=r, replace=False)] if r else []
        # a few deps on not-yet-issued dots of other sources (pending waits)
        if i % 7 == 3:
            other = 1 + src % n
            deps.append((other, seqs[other] + 1))
        deps = sorted(set(deps))
        ex.handle_add(dot, dot, [0], deps, i)
        g.handle_add(dot, deps, i)
        issued.append(dot)
        if i % 11 == 0:
            ex.to_clients_iter()
    # deliver the dots waited on but never issued, so every Add executes
    for p in range(1, n + 1):
        for q in range(seqs[p] + 1, seqs[p] + 3):
            ex.handle_add((p, q), (p, q), [0], [], 400)
            g.handle_add((p, q), [], 400)
    assert [d for d, _ in ex.drain_dots()] == [d for d, _, _ in g.drain()]
    assert ex.metrics(CHAIN_SIZE) == g.metrics(1)
    assert ex.metrics(EXECUTION_DELAY) == g.metrics(0)


def test_executor_drain_after_every_add_is_linear(gpu):
    """The simulator drains to_clients after every handle (runner.rs:406-424):
    bytes moved per drained Add must not grow with the log length."""
    p = fs.synth_params(seed=9, n=3, instances=1, cmds=10_000, window=8, cycle_pct=30)
    planes = fs.synth_host(p)
    stream = planes.stream(0)
    ex = GraphExecutor(1, 0, 3, monitor=False)
    marks = {}
    for i, (dot, deps, t, _kind) in enumerate(stream):
        ex.handle_add(dot, dot, [0], deps, t)
        ex.to_clients_iter()
        if i + 1 in (3_000, 30_000):
            marks[i + 1] = sum(ex.transfer_stats())
    assert len(stream) >= 30_000
    per_add_small = marks[3_000] / 3_000
    per_add_large = (marks[30_000] - marks[3_000]) / 27_000
    # linear: the later Adds cost no more per Add than the early ones (capacity
    # doubling re-uploads are amortised); quadratic would be ~10x here
    assert per_add_large < 2.0 * per_add_small + 64, (per_add_small, per_add_large)
    # and small: a flush moves only this stream's words of each tile (strided
    # copies), not the 64-stream tiles (~1.8 KB per Add before)
    assert per_add_large < 256, per_add_large


def test_executor_many_pending_escalates_to_hbm_tables(gpu):
    """configs[3]-shaped log (64 clients per process, 100 % conflicts): the
    pending set passes the 64 slots of tier 2, so the handle reruns its log on
    the resumable HBM tables (tier 8) and keeps resuming there; results, metrics
    and the pending set equal the oracle's at every pull."""
    p = fs.synth_params(seed=5, instances=1, n=5, cmds=640, window=320, cycle_pct=30, conflicts=(100,),
                        clients=64)
    stream = fs.synth_host(p).stream(0)
    ex = GraphExecutor(1, 0, 5, monitor=True)
    g = oracle_lib.Graph(1, 5)
    got, exp = [], []
    max_pending = 0
    for i, (dot, deps, t, _kind) in enumerate(stream):
        ex.handle_add(dot, dot, [0], deps, t)
        g.handle_add(dot, deps, t)
        if i % 97 == 0 or i == len(stream) - 1:
            got += [d for d, _ in ex.drain_dots()]
            exp += [d for d, _, _ in g.drain()]
            assert got == exp, i
            pend = ex.pending()
            max_pending = max(max_pending, len(pend))
            if i % 388 == 0:
                assert pend == sorted(g.pending(cap=20_000)), i
    assert max_pending > 64
    assert ex.metrics(CHAIN_SIZE) == g.metrics(1)
    assert ex.metrics(EXECUTION_DELAY) == g.metrics(0)
    assert max(ex.metrics(CHAIN_SIZE)) > 5


def test_executor_u32_sequences_above_the_frontier(gpu):
    """Sequences near 2^32 - 1: the handle starts from an executed frontier F
    and holds seq - F on the device; the run equals the same stream at F = 0."""
    p = fs.synth_params(seed=12, n=3, instances=1, cmds=300, window=8, cycle_pct=30)
    stream = fs.synth_host(p).stream(0)
    F = 2**32 - 1 - 2000
    runs = []
    for base in (0, F):
        ex = GraphExecutor(1, 0, 3, monitor=False)
        if base:
            ex.set_executed_frontier([base] * 3)
        shift = lambda d: (d[0], d[1] + base)
        for i, (dot, deps, t, _kind) in enumerate(stream):
            ex.handle_add(shift(dot), dot, [0], [shift(d) for d in deps] + ([(1, base)] if base else []), t)
            if i % 50 == 0:
                ex.to_clients_iter()
        runs.append([((d[0], d[1] - base), s) for d, s in ex.drain_dots()])
    assert runs[0] == runs[1] and len(runs[0]) > 0
    ex = GraphExecutor(1, 0, 3, monitor=False)
    ex.set_executed_frontier([F] * 3)
    with pytest.raises(_lib.FxError):
        ex.handle_add((1, F), (1, 1), [0], [], 0)  # at or below the frontier: executed


def test_cpp_executor_tests(gpu):
    exe = os.path.join(ROOT, "tests", "cpp", "build", "test_graph_executor")
    assert os.path.exists(exe), "build with `make`"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr


# ------------------------------------------- BASELINE configs at full size
@pytest.mark.parametrize("name,cmds,conflict", [
    # configs[4]: one instance, 10^6-command commit streams with cycles (5 executors)
    ("single_huge_instance", 200_000, 2),
    # configs[3]: dense-dependency stress, 100 % conflicts, 64 clients/region x 1k
    # commands at n=5 -> 320k commands per instance, large SCCs
    ("dense_stress", 64_000, 100),
])
def test_full_size_single_instance_matches_oracle(gpu, name, cmds, conflict):
    p = fs.synth_params(seed=2025, instances=1, n=5, cmds=cmds, window=8, cycle_pct=30,
                        conflicts=(conflict,))
    planes = fs.synth_host(p)
    res = fd.run_batch(planes, nbins_chain=64, nbins_delay=2048)
    assert res.status == _lib.FX_OK
    o_order, o_rel, o_nexec = assert_parity(planes, res)
    assert np.all(res.nexec == planes.steps)
    chain, delay = oracle_hists(planes, o_order, o_rel, o_nexec, 64, 2048)
    assert np.array_equal(res.chain, chain) and np.array_equal(res.delay, delay)
    if conflict == 100:
        # SCCs larger than one command exist (the worst-case graph of configs[3])
        assert chain[2:].sum() > 0


def _drain_run(stream, n, every, env=None, sleep_at=None):
    import os
    import time
    old = os.environ.get("FX_HANDLE_PERSIST")
    if env is not None:
        os.environ["FX_HANDLE_PERSIST"] = env
    try:
        ex = GraphExecutor(1, 0, n, monitor=True)
    finally:
        if env is not None:
            if old is None:
                del os.environ["FX_HANDLE_PERSIST"]
            else:
                os.environ["FX_HANDLE_PERSIST"] = old
    got = []
    for i, (dot, deps, t, _kind) in enumerate(stream):
        ex.handle_add(dot, dot, [0], deps, t)
        if i % every == 0:
            got += ex.drain_dots()
        if sleep_at is not None and i == sleep_at:
            time.sleep(0.6)  # the persistent kernel exits when idle; the next flush relaunches it
    got += ex.drain_dots()
    out = (got, ex.metrics(CHAIN_SIZE), ex.metrics(EXECUTION_DELAY), ex.pending())
    ex.close()
    return out


def test_executor_persistent_handles_interleaved_one_thread(gpu):
    """The simulator drives one executor per process from one thread
    (runner.rs:406-424): six persistent handles fed in turn, each drained after
    every Add.  Each handle's kernel has a hardware queue of its own; on shared
    queues a resident kernel holds back the next handle's until its idle exit
    (20 ms per switch here).  Orders equal the oracle's, and quickly."""
    import time
    streams = []
    for seed in range(6):
        p = fs.synth_params(seed=40 + seed, n=5, instances=1, cmds=120, window=8, cycle_pct=30, conflicts=(50,))
        streams.append(fs.synth_host(p).stream(0)[:500])
    exps = []
    for st in streams:
        g = oracle_lib.Graph(1, 5)
        for (dot, deps, t, _kind) in st:
            g.handle_add(dot, deps, t)
        exps.append([d for d, _, _ in g.drain()])
    hs = [GraphExecutor(1, 0, 5, monitor=False) for _ in streams]
    got = [[] for _ in streams]
    t0 = time.perf_counter()
    for i in range(max(len(st) for st in streams)):
        for h, st, out in zip(hs, streams, got):
            if i < len(st):
                dot, deps, t, _kind = st[i]
                h.handle_add(dot, dot, [0], deps, t)
                out += [d for d, _ in h.drain_dots()]
    dt = time.perf_counter() - t0
    for h, out in zip(hs, got):
        out += [d for d, _ in h.drain_dots()]
        h.close()
    assert got == exps
    assert dt < 5.0, dt


def test_executor_handles_made_one_after_another(gpu):
    """A freed handle's persistent resources (its hardware queue, mapped
    buffers, state block) go to a pool the next handle takes from: a program
    that makes a handle per case (the reference's shuffle tests,
    graph/mod.rs:1045-1113) pays for the queue once."""
    import time
    p = fs.synth_params(seed=5, n=3, instances=1, cmds=20, window=4, cycle_pct=30, conflicts=(50,))
    st = fs.synth_host(p).stream(0)[:40]
    g = oracle_lib.Graph(1, 3)
    for (dot, deps, t, _kind) in st:
        g.handle_add(dot, deps, t)
    exp = [d for d, _, _ in g.drain()]
    t0 = time.perf_counter()
    for _ in range(60):
        h = GraphExecutor(1, 0, 3, monitor=False)
        out = []
        for (dot, deps, t, _kind) in st:
            h.handle_add(dot, dot, [0], deps, t)
            out += [d for d, _ in h.drain_dots()]
        h.close()
        assert out == exp
    assert time.perf_counter() - t0 < 10.0


def test_executor_persistent_mode_equals_batch_tiers_and_oracle(gpu):
    """The handle's persistent mode (one resident wavefront running the wave
    tier over Adds published in host-mapped memory, drained after every Add as
    runner.rs:406-424 does) against the batch-tier handle (FX_HANDLE_PERSIST=0)
    and the oracle: same order, SCC starts, metrics; the kernel's idle exit and
    relaunch in the middle of the log change nothing."""
    p = fs.synth_params(seed=21, n=5, instances=1, cmds=3000, window=8, cycle_pct=30, conflicts=(50,))
    stream = fs.synth_host(p).stream(0)
    g = oracle_lib.Graph(1, 5)
    for (dot, deps, t, _kind) in stream:
        g.handle_add(dot, deps, t)
    exp = [d for d, _, _ in g.drain()]
    a = _drain_run(stream, 5, 1)
    b = _drain_run(stream, 5, 7, env="0")
    c = _drain_run(stream, 5, 3, sleep_at=len(stream) // 2)
    assert [d for d, _ in a[0]] == exp
    assert a[0] == b[0] == c[0]
    assert a[1:] == b[1:] == c[1:]
    assert a[1] == g.metrics(1) and a[2] == g.metrics(0)


def _with_env(env, fn):
    import os
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _bounded_wait_stream():
    p = fs.synth_params(seed=8, n=3, instances=1, cmds=20, window=4, cycle_pct=30, conflicts=(50,))
    st = fs.synth_host(p).stream(0)[:30]
    g = oracle_lib.Graph(1, 3)
    for (dot, deps, t, _kind) in st:
        g.handle_add(dot, deps, t)
    return st, [d for d, _, _ in g.drain()]


def test_executor_persistent_wait_is_bounded(gpu):
    """Every host wait of the persistent handle has a deadline (SURVEY §8(b):
    status codes replace panics; the reference's Executor never blocks,
    fantoch/src/executor/mod.rs:27-89).  A test hook makes the kernel skip the
    status store of its 3rd flush, so that pull's wait expires (300 ms here).
    The kernel still answers the stop request, so its stream drains: the
    handle moves the log to the batch tiers (as a capacity escalation does)
    and every pull, that one included, returns the oracle's order."""
    import time
    st, exp = _bounded_wait_stream()
    h = _with_env({"FX_HANDLE_TIMEOUT_MS": 300}, lambda: GraphExecutor(1, 0, 3, monitor=False))
    h.debug_hooks(skip_status_flush=3)
    out, slow = [], []
    for (dot, deps, t, _kind) in st:
        h.handle_add(dot, dot, [0], deps, t)
        t0 = time.perf_counter()
        out += [d for d, _ in h.drain_dots()]
        slow.append(time.perf_counter() - t0)
    h.close()
    assert out == exp
    assert 0.25 < slow[2] < 2.0, slow[:4]  # the expired wait, then the batch tiers


def test_executor_persistent_dead_kernel_is_abandoned(gpu):
    """A kernel that does not answer the stop request either (a hook holds it
    resident for 1.5 s, then it exits by itself): the pull returns
    FX_ERR_TIMEOUT within two deadlines, the error is sticky, and freeing the
    handle returns at once without touching its buffers or streams (they are
    leaked: the kernel may still use them).  A new handle then runs
    normally."""
    import time
    st, exp = _bounded_wait_stream()
    h = _with_env({"FX_HANDLE_TIMEOUT_MS": 300}, lambda: GraphExecutor(1, 0, 3, monitor=False))
    h.debug_hooks(skip_status_flush=3, hold_ms=1500)
    t0 = time.perf_counter()
    err = None
    for i, (dot, deps, t, _kind) in enumerate(st[:5]):
        h.handle_add(dot, dot, [0], deps, t)
        try:
            h.drain_dots()
        except _lib.FxError as e:
            err = (i, e.status, time.perf_counter() - t0)
            break
    assert err is not None and err[0] == 2 and err[1] == _lib.FX_ERR_TIMEOUT, err
    assert err[2] < 1.4, err
    with pytest.raises(_lib.FxError) as again:
        h.drain_dots()
    assert again.value.status == _lib.FX_ERR_TIMEOUT
    t1 = time.perf_counter()
    h.close()
    assert time.perf_counter() - t1 < 0.2
    time.sleep(1.6)  # the held kernel has exited by itself
    h2 = GraphExecutor(1, 0, 3, monitor=False)
    out = []
    for (dot, deps, t, _kind) in st:
        h2.handle_add(dot, dot, [0], deps, t)
        out += [d for d, _ in h2.drain_dots()]
    h2.close()
    assert out == exp


def test_executor_persistent_handle_beside_null_stream_work(gpu):
    """A resident handle kernel runs on a stream of its own hardware queue,
    which HIP makes a blocking stream: null-stream work (here synchronous
    copies through the library's device buffers) waits for it at most until
    its idle exit (20 ms).  A program that mixes a live handle with such work
     stays correct and pays at most that per switch."""
    import time
    p = fs.synth_params(seed=9, n=5, instances=1, cmds=40, window=8, cycle_pct=30, conflicts=(50,))
    st = fs.synth_host(p).stream(0)[:120]
    g = oracle_lib.Graph(1, 5)
    for (dot, deps, t, _kind) in st:
        g.handle_add(dot, deps, t)
    exp = [d for d, _, _ in g.drain()]
    h = GraphExecutor(1, 0, 5, monitor=False)
    out = []
    buf = fd.DeviceBuffer(4096)
    src = np.arange(1024, dtype=np.uint32)
    worst = 0.0
    for i, (dot, deps, t, _kind) in enumerate(st):
        h.handle_add(dot, dot, [0], deps, t)
        out += [d for d, _ in h.drain_dots()]
        if i % 20 == 0:
            t0 = time.perf_counter()
            buf.upload(src)  # null-stream copies while the handle's kernel is resident
            back = buf.download(np.uint32, 1024)
            worst = max(worst, time.perf_counter() - t0)
            assert np.array_equal(back, src)
    out += [d for d, _ in h.drain_dots()]
    h.close()
    buf.free()
    assert out == exp
    assert worst < 0.5, worst


def test_executor_persistent_mailbox_line_is_used(gpu):
    """One-Add flushes carry their row in the mailbox line next to the
    doorbell; the line's checksum (fx_internal.h persist_mb_mix) rejects a
    line read across two flushes, which then takes the ring path.  On an
    undisturbed drain-after-every-Add loop almost every flush takes the
    mailbox (a wrong checksum would silently fall back to the ring for all),
    and the order equals the oracle's."""
    p = fs.synth_params(seed=10, n=5, instances=1, cmds=60, window=8, cycle_pct=30, conflicts=(10,))
    st = fs.synth_host(p).stream(0)[:200]
    g = oracle_lib.Graph(1, 5)
    for (dot, deps, t, _kind) in st:
        g.handle_add(dot, deps, t)
    exp = [d for d, _, _ in g.drain()]
    h = _with_env({"FX_HANDLE_STATS": 1}, lambda: GraphExecutor(1, 0, 5, monitor=False))
    out = []
    for (dot, deps, t, _kind) in st:
        h.handle_add(dot, dot, [0], deps, t)
        out += [d for d, _ in h.drain_dots()]
    s = h.persist_stats()
    h.close()
    assert out == exp
    flushes, mailbox = s[0], s[14]
    assert flushes == len(st)
    assert mailbox >= 0.9 * flushes, (mailbox, flushes)
