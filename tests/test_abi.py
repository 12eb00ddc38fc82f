"""C-ABI checks that need no GPU: the library loads, exports every symbol the
header declares, refuses compute without a device (no CPU fallback), and its
host-side pieces (Histogram statistics, synthetic streams) are correct."""
import ctypes
import math
import os
import random
import re

import numpy as np
import pytest

from fantoch_amd import _lib
from fantoch_amd import streams as fs
from oracle import histogram as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fantoch_amd.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b(fx_[a-z0-9_]+)\s*\(", text))
    # static inline helpers and macros are not exported
    return sorted(n for n in names if n not in ("fx_plane_words", "fx_index"))


def test_every_declared_symbol_is_exported_and_bound(lib):
    bound = {name for name, _, _ in _lib.SIGNATURES}
    for name in declared_symbols():
        assert hasattr(lib, name), name
        assert name in bound, "ctypes binding missing for " + name


def test_version(lib):
    assert b"gfx950" in lib.fx_version()


def test_tier_query(lib):
    ti = _lib.TierInfo()
    assert lib.fx_tier_query(0, 5, ctypes.byref(ti)) == 0
    assert ti.pending_cap >= 8 and ti.window_bits >= 32 and ti.max_sources >= 5
    caps = []
    # the escalation order of fx_batch_run_tiered: 0 -> 1 -> 2 -> 7 (wide, LDS) -> 8 (wide, HBM)
    for t in (0, 1, 2, _lib.FX_TIER_WIDE, _lib.FX_TIER_WIDE_HBM):
        assert lib.fx_tier_query(t, 7, ctypes.byref(ti)) == 0
        caps.append((ti.pending_cap, ti.window_bits))
    assert caps == sorted(caps)
    assert lib.fx_tier_query(3, 7, ctypes.byref(ti)) == 0
    assert lib.fx_tier_query(1, 9, ctypes.byref(ti)) != 0
    assert lib.fx_tier_query(_lib.FX_NUM_TIERS, 5, ctypes.byref(ti)) != 0


def test_no_device_fails_loudly(lib):
    if lib.fx_device_count() > 0:
        pytest.skip("a GPU is visible")
    p = fs.synth_params(instances=1, n=3, cmds=4)
    S, steps, dmax = fs.synth_shape(p)
    planes = fs.synth_host(p)
    inb = _lib.StreamBatch(planes.dot.ctypes.data, planes.hdr.ctypes.data, planes.deps.ctypes.data,
                           None, S, steps, dmax, 3)
    o = np.zeros(planes.plane, np.uint32)
    r = np.zeros(planes.plane, np.uint32)
    ne = np.zeros(S, np.uint32)
    er = np.zeros(S, np.uint32)
    outb = _lib.OrderBatch(o.ctypes.data, r.ctypes.data, ne.ctypes.data, er.ctypes.data)
    st = lib.fx_batch_execute(ctypes.byref(inb), ctypes.byref(outb), 0, None, S, None, 0, steps,
                              _lib.FX_FLAG_INIT, None, None)
    assert st == _lib.FX_ERR_NO_DEVICE
    assert lib.fx_batch_run_tiered(ctypes.byref(inb), ctypes.byref(outb), 0, None, None) == \
        _lib.FX_ERR_NO_DEVICE
    cfg = _lib.Config(3, 1, 1, 0, 1)
    assert not lib.fx_graph_executor_new(1, 0, ctypes.byref(cfg))
    from fantoch_amd.executor import GraphExecutor
    with pytest.raises(_lib.FxError):
        GraphExecutor(1, 0, 3)


def test_bad_args_rejected(lib):
    ti = _lib.TierInfo()
    assert lib.fx_tier_query(0, 5, None) == _lib.FX_ERR_INVALID_ARG
    assert lib.fx_batch_execute(None, None, 0, None, 0, None, 0, 0, 0, None, None) == \
        _lib.FX_ERR_INVALID_ARG
    cfg = _lib.Config(3, 1, 2, 0, 0)  # shard_count > 1: partial replication is out of scope
    assert not lib.fx_graph_executor_new(1, 0, ctypes.byref(cfg))
    del ti


# ------------------------------------------- Histogram (product host code)
def product_stats(values):
    h = H.Histogram(values)
    items = h.items()
    v = (ctypes.c_uint64 * len(items))(*[x for x, _ in items])
    c = (ctypes.c_uint64 * len(items))(*[y for _, y in items])
    st = _lib.HistStats()
    assert _lib.load().fx_hist_stats_compute(v, c, len(items), ctypes.byref(st)) == 0
    return st, v, c, len(items)


def test_product_histogram_matches_reference_kats():  # histogram.rs:390-463
    st, *_ = product_stats([10, 20, 30])
    assert (st.mean, st.cov, st.min, st.max) == (20.0, 0.5, 10.0, 30.0)
    st, *_ = product_stats([10, 20])
    assert (st.mean, st.mdtm) == (15.0, 5.0)
    st, *_ = product_stats([10, 20, 40, 10])
    assert (H.round1(st.mean), H.round1(st.cov), H.round1(st.mdtm)) == ("20.0", "0.7", "10.0")
    data = [43, 54, 56, 61, 62, 66, 68, 69, 69, 70, 71, 72, 77, 78, 79, 85, 87, 88, 89, 93, 95,
            96, 98, 99, 99]
    _, v, c, n = product_stats(data)
    out = ctypes.c_double()
    for p, expect in ((0.9, 98.0), (0.5, 77.0), (0.2, 64.0)):
        assert _lib.load().fx_hist_percentile(v, c, n, p, ctypes.byref(out)) == 0
        assert out.value == expect


def test_product_histogram_matches_oracle_random():
    rng = random.Random(3)
    for _ in range(100):
        vals = [rng.randrange(0, 300) for _ in range(rng.randrange(2, 60))]
        st, v, c, n = product_stats(vals)
        h = H.Histogram(vals)
        for a, b in ((st.mean, h.mean()), (st.stddev, h.stddev()), (st.cov, h.cov()),
                     (st.mdtm, h.mdtm()), (st.min, h.min()), (st.max, h.max())):
            assert a == b or (math.isnan(a) and math.isnan(b)), (a, b)
        out = ctypes.c_double()
        for p in (0.0, 0.1, 0.25, 0.5, 0.75, 0.95, 0.99, 1.0):
            rc = _lib.load().fx_hist_percentile(v, c, n, p, ctypes.byref(out))
            try:
                expect = h.percentile(p)
            except (IndexError, TypeError):
                assert rc != 0
                continue
            assert rc == 0 and out.value == expect


# ------------------------------------------------- plane layout helpers
def test_index_matches_header_formula():
    steps = 37
    for s in (0, 1, 63, 64, 130):
        for i in (0, 1, 3, 4, 36):
            expect = ((s // 64) * ((steps + 3) // 4) + i // 4) * 256 + (s % 64) * 4 + i % 4
            assert int(_lib.index(i, s, steps)) == expect
    assert _lib.plane_words(65, 5) == 128 * 8


def test_pack_streams_roundtrip():
    streams = [[((1, 1), [(2, 1)], 5), ((2, 1), [(1, 1), (1, 1)], 7)],
               [((2, 1), [], 0)]]
    p = fs.pack_streams(streams, 2)
    assert p.stream(0) == [((1, 1), [(2, 1)], 5, 0), ((2, 1), [(1, 1)], 7, 0)]
    assert p.stream(1) == [((2, 1), [], 0, 0)]


def test_dense_stats_match_the_histogram_oracle():
    from fantoch_amd import metrics
    rng = np.random.default_rng(3)
    counts = np.zeros(64, np.uint64)
    for v in rng.integers(0, 40, 500):
        counts[v] += 1
    h = H.Histogram()
    for v, c in enumerate(counts):
        for _ in range(int(c)):
            h.increment(v)
    st = metrics.dense_stats(counts)
    assert st["count"] == 500 and st["clamped"] == 0
    assert math.isclose(st["mean"], h.mean(), rel_tol=1e-12)
    assert math.isclose(st["p99"], h.percentile(0.99), rel_tol=1e-12)
    assert metrics.dense_stats(np.zeros(8)) == {"count": 0, "clamped": 0}


def test_quorum_sizes_kats():
    # config.rs atlas_parameters / epaxos_parameters tests
    A, E = _lib.FX_PROTOCOL_ATLAS, _lib.FX_PROTOCOL_EPAXOS
    assert [_lib.quorum_sizes(A, 7, f) for f in (1, 2, 3)] == [(4, 2), (5, 3), (6, 4)]
    assert [_lib.quorum_sizes(E, n) for n in (3, 5, 7, 9, 11, 13, 15, 17)] == \
        [(2, 2), (3, 3), (5, 4), (6, 5), (8, 6), (9, 7), (11, 8), (12, 9)]
    assert _lib.quorum_sizes(A, 3, 1) == (2, 2)  # BASELINE configs[0]: d <= 2
    with pytest.raises(_lib.FxError):
        _lib.quorum_sizes(7, 5, 1)


def test_product_planet_matches_the_oracle_parser():
    """fx_planet_load (product, host C++) and the oracle's Planet parser read the
    same latency_gcp/*.dat files into the same matrix and distance order."""
    from fantoch_amd import sim as S
    from oracle import oracle_lib as O
    pl = S.Planet()
    assert pl.regions == O.planet_regions()
    lat, srt = O.planet_matrix()
    R = pl.R
    assert np.array_equal(pl.ping[:R, :R].astype(np.int64), lat)
    for a in range(R):  # rank[a][b] = position of b in sorted(a)
        assert [int(b) for b in np.argsort(pl.rank[a, :R])] == [int(x) for x in srt[a]]


def test_sim_plan_sizes():
    from fantoch_amd import sim as S
    import ctypes
    pl = S.Planet()
    lib = _lib.load()
    regs = pl.ids(S.GCP5[:5])
    s = S.spec(S.EPAXOS, 5, 2, regs, regs)
    b = ctypes.c_uint32()
    assert lib.fx_sim_plan(ctypes.byref(s), 32, 8, ctypes.byref(b)) == 0
    small = b.value
    assert 4 * 1024 < small < 64 * 1024
    # default pools (0 = 16 n messages per client region, min(64, 8 C) dots) need more LDS than 32 / 8
    assert lib.fx_sim_plan(ctypes.byref(s), 0, 0, ctypes.byref(b)) == 0
    assert small < b.value < 64 * 1024
    assert lib.fx_sim_plan(ctypes.byref(s), 0, 257, ctypes.byref(b)) == _lib.FX_ERR_UNSUPPORTED
    s9 = S.spec(S.EPAXOS, 5, 2, regs, regs, clients_per_region=40)  # 200 clients: too many links
    assert lib.fx_sim_plan(ctypes.byref(s9), 32, 8, ctypes.byref(b)) == _lib.FX_ERR_UNSUPPORTED


def test_sim_default_geometry_occupancy():
    """The default tables keep the benchmarked geometries at their measured
    occupancy: configs[1] (EPaxos n = 5, one client per region) fits 20
    instances per CU (the 5-wave kernel, <= 8,192 B of LDS), configs[2]'s n = 7
    Atlas placements use 32 live dots and >= 192 messages (13 per CU: the
    ChainSize and client-latency samples are counted in lanes, not LDS)."""
    from fantoch_amd import sim as S
    import ctypes
    pl = S.Planet()
    lib = _lib.load()
    b = ctypes.c_uint32()
    r5 = pl.ids(S.GCP5[:5])
    s5 = S.spec(S.EPAXOS, 5, 2, r5, r5, commands_per_client=1000)
    assert lib.fx_sim_plan(ctypes.byref(s5), 0, 0, ctypes.byref(b)) == 0
    assert b.value <= 160 * 1024 // 20, b.value
    r7 = pl.ids(sorted(pl.names)[:7]) if hasattr(pl, "names") else pl.ids(S.GCP5[:5] + ["us-east1", "us-west1"])
    s7 = S.spec(S.ATLAS, 7, 1, r7, r7, commands_per_client=100)
    assert lib.fx_sim_plan(ctypes.byref(s7), 0, 0, ctypes.byref(b)) == 0
    d7 = b.value
    assert lib.fx_sim_plan(ctypes.byref(s7), 192, 32, ctypes.byref(b)) == 0
    assert d7 == b.value and 160 * 1024 // d7 == 13, d7
