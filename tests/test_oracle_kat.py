"""Pins the CPU oracle (oracle/graph_oracle.cpp, oracle/histogram.py) to the
reference's own known-answer tests before it is trusted as the checker of the
HIP path.  CPU only."""
import math
import random

import pytest

import kat_shapes as K
from oracle import histogram as H
from oracle import oracle_lib


class OracleExec:
    """Adapter: the oracle DependencyGraph behind the check_termination driver."""

    def __init__(self, n, process_id=1):
        self.g = oracle_lib.Graph(process_id, n)

    def handle_add(self, dot, deps, t):
        self.g.handle_add(dot, sorted(deps), t)

    def drain(self):
        return [d for d, _, _ in self.g.drain()]


def make(n):
    return OracleExec(n)


# ----------------------------------------------------- graph/mod.rs tests
def test_simple():  # mod.rs:714-752
    g = oracle_lib.Graph(1, K.SIMPLE["n"])
    for (dot, deps), expect in zip(K.SIMPLE["adds"], K.SIMPLE["ready_after"]):
        g.handle_add(dot, deps)
        assert [d for d, _, _ in g.drain()] == expect


def test_cycle():  # mod.rs:896-917
    K.shuffle_it(make, K.CYCLE["n"], K.CYCLE["args"])


def test_add_random():  # mod.rs:919-930 (seeded)
    for args in K.random_cases():
        K.shuffle_it(make, 2, args)


def test_transitive_conflicts_assumption_regression_1():  # mod.rs:788-824
    a = K.check_termination(make, K.REGRESSION_1["n"], K.REGRESSION_1["order_a"])
    b = K.check_termination(make, K.REGRESSION_1["n"], K.REGRESSION_1["order_b"])
    assert a != b


def test_transitive_conflicts_assumption_regression_2():  # mod.rs:855-894
    a = K.check_termination(make, K.REGRESSION_2["n"], K.REGRESSION_2["order_a"])
    b = K.check_termination(make, K.REGRESSION_2["n"], K.REGRESSION_2["order_b"])
    assert a != b


def test_sccs_found_and_missing_dep():  # mod.rs:1115-1348
    f = K.SCCS_MISSING
    g = oracle_lib.Graph(f["process_id"], f["n"])
    root, root_deps = f["root"]
    g.index_only(root, root_deps)
    for dot, deps in f["indexed"]:
        g.index_only(dot, deps)
    for p, fr in enumerate(f["executed"], start=1):
        g.set_executed(p, fr)
    kind, missing, ready, ndots = g.find_scc(root, first_find=True)
    assert kind == 1  # FinderInfo::MissingDependencies
    assert missing == f["missing"]
    assert ready == ndots  # ready_commands == to_be_executed.len()
    # with canonical C1 order the SCCs are found on the first try (the
    # reference loops until hash order visits (4, 40) before (5, 61))
    assert ndots == 10
    executed = g.drain()
    assert [d for d, _, _ in executed] == [(4, s) for s in range(31, 41)]
    assert all(start for _, _, start in executed)


def test_executed_clock_exceptions():
    # AEClock semantics (threshold 0.9.1): out-of-order adds are kept above the
    # frontier and compacted when the gap closes.  (2,3) depends on (2,1)
    # which arrives last; (2,2) has no deps and executes first.
    g = oracle_lib.Graph(1, 2)
    g.handle_add((2, 2), [])
    g.handle_add((2, 3), [(2, 1), (2, 2)])
    assert [d for d, _, _ in g.drain()] == [(2, 2)]
    g.handle_add((2, 1), [])
    assert [d for d, _, _ in g.drain()] == [(2, 1), (2, 3)]


def test_double_index_is_an_error():  # mod.rs:233-237 panics
    g = oracle_lib.Graph(1, 2)
    g.handle_add((1, 1), [(2, 1)])
    with pytest.raises(RuntimeError):
        g.handle_add((1, 1), [(2, 1)])


# ------------------------------------------------- histogram.rs tests
def approx(a, b):
    return a == b or (math.isnan(a) and math.isnan(b))


def test_histogram_stats():  # histogram.rs:390-410
    s = H.Histogram([1, 1, 1])
    assert s.mean() == 1.0 and s.cov() == 0.0 and s.mdtm() == 0.0
    assert s.min() == 1.0 and s.max() == 1.0
    s = H.Histogram([10, 20, 30])
    assert s.mean() == 20.0 and s.cov() == 0.5 and s.min() == 10.0 and s.max() == 30.0
    s = H.Histogram([10, 20])
    assert s.mean() == 15.0 and s.mdtm() == 5.0 and s.min() == 10.0 and s.max() == 20.0


def test_histogram_stats_show():  # histogram.rs:412-433
    cases = [([1, 1, 1], "1.0", "0.0", "0.0"), ([10, 20, 30], "20.0", "0.5", "6.7"),
             ([10, 20], "15.0", "0.5", "5.0"), ([10, 20, 40, 10], "20.0", "0.7", "10.0")]
    for vals, mean, cov, mdtm in cases:
        s = H.Histogram(vals)
        assert (H.round1(s.mean()), H.round1(s.cov()), H.round1(s.mdtm())) == (mean, cov, mdtm)


def test_histogram_stats_improv():  # histogram.rs:435-448
    a, b = H.Histogram([1, 1, 1]), H.Histogram([10, 20])
    assert a.mean() - b.mean() == -14.0
    assert a.mdtm() - b.mdtm() == -5.0
    assert H.Histogram([1, 1, 1]).cov() - H.Histogram([10, 20, 30]).cov() == -0.5


def test_histogram_percentile():  # histogram.rs:450-463
    data = [43, 54, 56, 61, 62, 66, 68, 69, 69, 70, 71, 72, 77, 78, 79, 85, 87, 88, 89, 93, 95,
            96, 98, 99, 99]
    s = H.Histogram(data)
    assert s.min() == 43.0 and s.max() == 99.0
    assert s.percentile(0.9) == 98.0
    assert s.percentile(0.5) == 77.0
    assert s.percentile(0.2) == 64.0


def test_histogram_merge_check():  # histogram.rs:354-383 (quickcheck -> seeded random)
    rng = random.Random(7)
    for _ in range(200):
        a = [(rng.randrange(50), rng.randrange(1, 5)) for _ in range(rng.randrange(20))]
        b = [(rng.randrange(50), rng.randrange(1, 5)) for _ in range(rng.randrange(20))]
        ha, hb = H.Histogram.from_pairs(a), H.Histogram.from_pairs(b)
        ha.merge(hb)
        ref = {}
        for v, c in a + b:
            ref[v] = ref.get(v, 0) + c
        assert ha.values == ref
