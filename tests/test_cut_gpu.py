"""Quiescent-cut driver (fx_batch_run_cut) vs the CPU oracle, bit for bit:
order plane, release plane, nexec, status and both histograms.  GPU only.

The driver splits each stream at its dependency-closed prefixes and runs the
segments as one batch (graph_cut.hip); a stream it cannot split runs whole.
Either way the outputs must equal the oracle's on the unsplit stream."""
import time

import numpy as np
import pytest

from fantoch_amd import _lib
from fantoch_amd import device as fd
from fantoch_amd import streams as fs
from oracle import oracle_lib
from test_gpu_parity import assert_parity, oracle_hists

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", [
    dict(n=5, instances=8, cmds=400, window=8, cycle_pct=30, conflicts=(2, 50, 100)),
    dict(n=3, instances=16, cmds=300, window=6, cycle_pct=60, conflicts=(10, 100)),
    # long SCC chains at 100 % conflicts: most streams still split
    dict(n=7, instances=4, cmds=200, window=16, cycle_pct=60, conflicts=(100,)),
    dict(n=5, instances=8, cmds=200, window=0, cycle_pct=0, conflicts=(0, 100)),
    dict(n=2, instances=33, cmds=77, window=5, cycle_pct=40, conflicts=(50,)),
])
def test_cut_matches_oracle(case):
    case = dict(case)
    p = fs.synth_params(seed=11, **case)
    planes = fs.synth_host(p)
    res = fd.run_batch(planes, cut=True, nbins_chain=64, nbins_delay=4096)
    assert res.status == _lib.FX_OK
    o_order, o_rel, o_nexec = assert_parity(planes, res)
    chain, delay = oracle_hists(planes, o_order, o_rel, o_nexec, 64, 4096)
    assert np.array_equal(res.chain, chain) and np.array_equal(res.delay, delay)
    st = res.cut_stats
    assert st.failed_streams == 0
    assert st.whole_streams == 0 and st.segments > planes.S
    assert st.single_segments <= st.segments


def test_cut_only_single_segments():
    """Streams without dependencies: every segment is one Add long, so no
    batch runs at all (k_build writes every row); the same outputs as the
    oracle's.  One stream beside them with deps checks the mixed case."""
    n = 3
    streams = [[((1 + (k % n), 1 + k // n), [], 1) for k in range(9)] for _ in range(4)]
    planes = fs.pack_streams(streams, n)
    res = fd.run_batch(planes, cut=True, nbins_chain=64, nbins_delay=4096)
    assert res.status == _lib.FX_OK
    o_order, o_rel, o_nexec = assert_parity(planes, res)
    chain, delay = oracle_hists(planes, o_order, o_rel, o_nexec, 64, 4096)
    assert np.array_equal(res.chain, chain) and np.array_equal(res.delay, delay)
    st = res.cut_stats
    assert st.segments == 36 and st.single_segments == 36 and sum(st.tier_counts) == 0
    # a cycle (two Adds waiting on each other) among single Adds
    streams[1] = [((1, 1), [], 1), ((2, 1), [(3, 1)], 2), ((3, 1), [(2, 1)], 3), ((1, 2), [], 4)]
    planes = fs.pack_streams(streams, n)
    res = fd.run_batch(planes, cut=True)
    assert res.status == _lib.FX_OK
    assert_parity(planes, res)
    st = res.cut_stats
    assert st.segments == 3 * 9 + 3 and st.single_segments == 3 * 9 + 2


def test_cut_ragged_lengths():
    """Ragged stream lengths (an empty stream among them): a truncated stream
    whose last Adds wait on dots past its end has no final cut and runs whole."""
    p = fs.synth_params(seed=5, instances=12, n=5, cmds=120, window=8, cycle_pct=30, conflicts=(2, 50, 100))
    planes = fs.synth_host(p)
    rng = np.random.default_rng(3)
    lengths = rng.integers(0, planes.steps + 1, planes.S).astype(np.uint32)
    lengths[0] = 0
    lengths[1] = planes.steps
    planes.lengths = lengths
    res = fd.run_batch(planes, cut=True)
    assert res.status == _lib.FX_OK
    assert_parity(planes, res)


def test_cut_unsplittable_and_errors():
    """A dep that never arrives (no final cut: the stream runs whole) and a
    double index (runs whole, FX_ERR_DOUBLE_INDEX as with the tiered driver)."""
    n = 3
    streams = [
        [((1, 1), [], 1), ((2, 1), [(3, 9)], 2), ((1, 2), [(2, 1)], 3), ((3, 1), [], 4)],  # (3, 9) never arrives
        [((1, 1), [(3, 5)], 1), ((2, 1), [(1, 1)], 2), ((1, 1), [], 3)],  # double index of a pending dot
        [((1, 1), [(2, 1)], 1), ((2, 1), [(1, 1)], 2), ((3, 1), [(1, 1), (2, 1)], 3)],  # a 2-cycle, then a cut
        [],
    ]
    planes = fs.pack_streams(streams, n)
    res = fd.run_batch(planes, cut=True)
    ref = fd.run_batch(planes)
    assert np.array_equal(res.err, ref.err) and np.array_equal(res.nexec, ref.nexec)
    assert res.err[1] == _lib.FX_ERR_DOUBLE_INDEX and res.err[0] == _lib.FX_OK
    assert res.cut_stats.whole_streams == 2
    assert_parity(planes, res)


def _segment_stream(lengths, n, seq0=None):
    """One commit stream made of dependency-closed segments of the given
    lengths: a segment of L > 1 Adds is a cycle (Add j waits on Add j + 1 mod
    L, dots spread over the n sources), a segment of 1 Add has no deps."""
    seq = dict(seq0 or {}) or {q: 0 for q in range(1, n + 1)}
    out, t = [], 1
    for L in lengths:
        dots = []
        for j in range(L):
            src = 1 + (len(out) + j) % n
            seq[src] += 1
            dots.append((src, seq[src]))
        for j in range(L):
            deps = [dots[(j + 1) % L]] if L > 1 else []
            out.append((dots[j], deps, t))
            t += 1
    return out


@pytest.mark.parametrize("many_long", [False, True])
def test_cut_segment_length_classes(many_long):
    """Segments of every length class (1 to 130 Adds, cycles) in a few
    streams: the batch ordered longest class first, ranks by k_rank_slots
    (the longer segments hold few Adds) or by k_rank over every Add; the
    outputs equal the oracle's."""
    n = 5
    rng = np.random.default_rng(17 if many_long else 16)
    streams = []
    for s in range(3):
        longs = [2, 3, 4, 5, 8, 9, 16, 17, 32, 33, 64, 65, 130]
        lengths = longs * (6 if many_long else 1) + [1] * (100 if many_long else 6000)
        rng.shuffle(lengths)
        streams.append(_segment_stream(lengths, n))
    planes = fs.pack_streams(streams, n)
    res = fd.run_batch(planes, cut=True, nbins_chain=256, nbins_delay=4096)
    assert res.status == _lib.FX_OK
    o_order, o_rel, o_nexec = assert_parity(planes, res)
    assert np.all(res.nexec == planes.lengths)
    chain, delay = oracle_hists(planes, o_order, o_rel, o_nexec, 256, 4096)
    assert np.array_equal(res.chain, chain) and np.array_equal(res.delay, delay)
    st = res.cut_stats
    assert st.whole_streams == 0 and st.failed_streams == 0
    assert st.segments == 3 * len(lengths)
    assert st.single_segments == 3 * lengths.count(1)
    assert st.max_segment == 130


def test_config4_single_huge_instance_cut():
    """BASELINE configs[4]: one instance, five executors each fed a
    10^6-Add commit stream with cycles; bit-exact with the oracle and timed
    against it."""
    p = fs.synth_params(seed=2025, instances=1, n=5, cmds=200_000, window=8, cycle_pct=30, conflicts=(2,))
    planes = fs.synth_host(p)
    fd.run_batch(planes, cut=True, metrics=False)  # warm-up (module load, allocations)
    t0 = time.time()
    res = fd.run_batch(planes, cut=True, nbins_chain=64, nbins_delay=2048)
    t_gpu = time.time() - t0
    assert res.status == _lib.FX_OK and res.cut_stats.whole_streams == 0
    t0 = time.time()
    o_order, o_rel, o_nexec = assert_parity(planes, res)
    t_cpu = time.time() - t0
    assert np.all(res.nexec == planes.steps)
    chain, delay = oracle_hists(planes, o_order, o_rel, o_nexec, 64, 2048)
    assert np.array_equal(res.chain, chain) and np.array_equal(res.delay, delay)
    st = res.cut_stats
    print("configs[4]: GPU cut driver %.3f s (incl. host<->device copies), oracle+compare %.3f s, "
          "%d segments (%d of one Add), longest %d" % (t_gpu, t_cpu, st.segments, st.single_segments,
                                                       st.max_segment))
    assert 0 < st.single_segments < st.segments


def test_config4_s5_single_huge_instance_cut():
    """BASELINE configs[4] on the stream SURVEY §8(d) specifies (S5): one
    instance, five executors of 10^6 Adds each, per-key chains over 1,000 keys
    plus cycles, mean deps ~3 (bench.py --mode huge's default shape);
    bit-exact with the oracle, histograms included."""
    p = fs.synth_params(seed=2026, instances=1, n=5, cmds=200_000, window=8, cycle_pct=30, horizon=640,
                        key_pool=1000)
    planes = fs.synth_host(p)
    nd = ((planes.hdr >> 24) & 31).astype(np.int64).sum() / (planes.S * planes.steps)
    assert 2.8 < nd < 3.2, nd
    res = fd.run_batch(planes, cut=True, nbins_chain=64, nbins_delay=2048)
    assert res.status == _lib.FX_OK
    o_order, o_rel, o_nexec = assert_parity(planes, res)
    assert np.all(res.nexec == planes.steps)
    chain, delay = oracle_hists(planes, o_order, o_rel, o_nexec, 64, 2048)
    assert np.array_equal(res.chain, chain) and np.array_equal(res.delay, delay)
    st = res.cut_stats
    print("S5: %d segments (%d of one Add), longest %d, whole streams %d" % (
        st.segments, st.single_segments, st.max_segment, st.whole_streams))
    assert st.failed_streams == 0


@pytest.mark.parametrize("rate", [50, 100])
def test_high_conflict_single_instance_cut(rate):
    """One instance at high conflict rates (every command on the shared key at
    100 %, 30 % concurrent cycles): cuts become rare, and segments longer than
    the driver's limit (or a stream without a final cut) run whole; either way
    bit-exact with the oracle."""
    p = fs.synth_params(seed=2027, instances=1, n=5, cmds=20_000, window=8, cycle_pct=30, conflicts=(rate,))
    planes = fs.synth_host(p)
    res = fd.run_batch(planes, cut=True, nbins_chain=256, nbins_delay=2048)
    assert res.status == _lib.FX_OK
    o_order, o_rel, o_nexec = assert_parity(planes, res)
    assert np.all(res.nexec == planes.steps)
    chain, delay = oracle_hists(planes, o_order, o_rel, o_nexec, 256, 2048)
    assert np.array_equal(res.chain, chain) and np.array_equal(res.delay, delay)
    st = res.cut_stats
    print("%d %%: %d segments, longest %d, whole streams %d" % (rate, st.segments, st.max_segment,
                                                               st.whole_streams))
    assert st.failed_streams == 0


def test_cut_every_stream_empty():
    """All lengths 0: no segment at all; every stream still gets nexec = 0 and
    FX_OK (the outputs start as a sentinel, device.run_batch)."""
    p = fs.synth_params(seed=8, instances=4, n=3, cmds=20, window=4, cycle_pct=20, conflicts=(50,))
    planes = fs.synth_host(p)
    planes.lengths = np.zeros(planes.S, np.uint32)
    res = fd.run_batch(planes, cut=True)
    assert res.status == _lib.FX_OK
    assert np.all(res.nexec == 0) and np.all(res.err == _lib.FX_OK)


def test_cut_empty_stream_beside_unsplittable_only():
    """One empty stream next to streams that all run whole (a dep that never
    arrives): the empty one is still written."""
    n = 3
    streams = [
        [((1, 1), [], 1), ((2, 1), [(3, 9)], 2)],  # (3, 9) never arrives: runs whole
        [],
        [((2, 1), [(1, 7)], 1), ((1, 1), [], 2)],  # (1, 7) never arrives
    ]
    planes = fs.pack_streams(streams, n)
    res = fd.run_batch(planes, cut=True)
    ref = fd.run_batch(planes)
    assert res.status == _lib.FX_OK
    assert np.array_equal(res.err, ref.err) and np.array_equal(res.nexec, ref.nexec)
    assert res.nexec[1] == 0 and res.err[1] == _lib.FX_OK
    assert res.cut_stats.whole_streams == 2
    assert_parity(planes, res)
