"""bench_sim.hist_parity: the headline bench's histogram check on its sample
(client latency per region, ChainSize, ExecutionDelay; runner.rs:619-634,
histogram.rs:55-59, graph/mod.rs:492-518).  CPU only: synthetic arrays."""
import numpy as np

import bench_sim


def _case(rng):
    R, LB = 4, 32
    per = [{"latency": rng.integers(0, 5, (R, LB)).astype(np.uint64),
            "chain": rng.integers(0, 5, 16).astype(np.uint64),
            "delay": rng.integers(0, 5, 24).astype(np.uint64)} for _ in range(3)]
    sample = (sum(p["latency"] for p in per).astype(np.int64), sum(p["chain"] for p in per).astype(np.int64),
              sum(p["delay"] for p in per).astype(np.int64))
    rest = (rng.integers(0, 9, (R, LB)), rng.integers(0, 9, 16), rng.integers(0, 9, 24))
    timed = tuple(s + r for s, r in zip(sample, rest))
    return timed, sample, rest, per


def test_hist_parity_accepts_consistent_histograms():
    timed, sample, rest, per = _case(np.random.default_rng(1))
    ok, detail = bench_sim.hist_parity(timed, sample, rest, per)
    assert ok
    assert all(d["sample_equals_oracle"] and d["timed_equals_sample_plus_rest"] for d in detail.values())


def test_hist_parity_rejects_a_wrong_bin_anywhere():
    for which in range(3):
        for part in ("timed", "sample"):
            timed, sample, rest, per = _case(np.random.default_rng(2 + which))
            t = [x.copy() for x in timed]
            s = [x.copy() for x in sample]
            (t if part == "timed" else s)[which].flat[3] += 1
            ok, detail = bench_sim.hist_parity(tuple(t), tuple(s), rest, per)
            assert not ok, (which, part)


def test_hist_parity_oracle_bins_wider_than_gpu():
    """The oracle's bins may be wider than the GPU's arrays: the overlap is compared."""
    timed, sample, rest, per = _case(np.random.default_rng(7))
    wide = [dict(p, delay=np.concatenate([p["delay"], np.zeros(8, np.uint64)])) for p in per]
    ok, _ = bench_sim.hist_parity(timed, sample, rest, wide)
    assert ok
