"""The simulator oracle (oracle/sim_oracle.cpp) pinned by the reference's own
known-answer tests.  CPU only.

Each test names the reference test it restates.  The reference's randomness
(rand::thread_rng) and hash orders are replaced by the canonical C3-C12 of
SURVEY.md §8(a) row a16; the assertions the reference makes are order- and
seed-independent, so they hold verbatim."""
import numpy as np
import pytest

from oracle import oracle_lib as O

REGIONS = O.planet_regions()
IDX = {r: i for i, r in enumerate(REGIONS)}
BASIC, ATLAS, EPAXOS = 2, 0, 1


def hist_mean(h):
    v = np.arange(h.shape[0], dtype=np.float64)
    c = h.astype(np.float64)
    return (v * c).sum() / c.sum()


def hist_cov(h):  # histogram.rs:74-90: stddev (n - 1) / mean
    v = np.arange(h.shape[0], dtype=np.float64)
    c = h.astype(np.float64)
    n = c.sum()
    m = (v * c).sum() / n
    return np.sqrt((c * (v - m) ** 2).sum() / (n - 1)) / m


# ------------------------------------------------------------------ planet
def test_planet_has_the_20_gcp_regions():
    assert len(REGIONS) == 20 and REGIONS == sorted(REGIONS)


def test_dat_latencies_europe_west3():  # planet/dat.rs:124-154
    lat, _ = O.planet_matrix()
    expected = {
        "europe-west3": 0, "europe-west4": 7, "europe-west6": 7, "europe-west1": 8,
        "europe-west2": 13, "europe-north1": 31, "us-east4": 86, "northamerica-northeast1": 87,
        "us-east1": 98, "us-central1": 105, "us-west1": 136, "us-west2": 139,
        "southamerica-east1": 214, "asia-northeast1": 224, "asia-northeast2": 233,
        "asia-east1": 258, "asia-east2": 268, "australia-southeast1": 276,
        "asia-southeast1": 289, "asia-south1": 352,
    }
    a = IDX["europe-west3"]
    assert {REGIONS[b]: int(lat[a, b]) for b in range(20)} == expected


def test_planet_latency_symmetry():  # planet/mod.rs:190-210
    lat, _ = O.planet_matrix()
    sym = lambda a, b: lat[IDX[a], IDX[b]] == lat[IDX[b], IDX[a]]
    assert sym("europe-west3", "us-central1")
    assert not sym("us-east1", "europe-west3")
    assert not sym("us-east4", "us-west1")
    assert not sym("us-west1", "europe-west3")


def test_planet_sorted_europe_west3():  # planet/mod.rs:212-254
    _, srt = O.planet_matrix()
    expected = ["europe-west3", "europe-west4", "europe-west6", "europe-west1", "europe-west2",
                "europe-north1", "us-east4", "northamerica-northeast1", "us-east1", "us-central1",
                "us-west1", "us-west2", "southamerica-east1", "asia-northeast1", "asia-northeast2",
                "asia-east1", "asia-east2", "australia-southeast1", "asia-southeast1", "asia-south1"]
    assert [REGIONS[i] for i in srt[IDX["europe-west3"]]] == expected


SEVENTEEN = ["asia-east1", "asia-northeast1", "asia-south1", "asia-southeast1",
             "australia-southeast1", "europe-north1", "europe-west1", "europe-west2",
             "europe-west3", "europe-west4", "northamerica-northeast1", "southamerica-east1",
             "us-central1", "us-east1", "us-east4", "us-west1", "us-west2"]


def test_sort_processes_by_distance():  # util.rs:222-266
    procs = [(i, IDX[r]) for i, r in enumerate(SEVENTEEN)]
    got = O.sort_processes(IDX["europe-west3"], procs)
    assert got == [8, 9, 6, 7, 5, 14, 10, 13, 12, 15, 16, 11, 1, 0, 4, 3, 2]


def test_discover_quorums():  # protocol/base.rs:268-347 (n=17, f=3, fq=6, wq=4)
    procs = [(i, IDX[r]) for i, r in enumerate(SEVENTEEN)]
    s = O.sort_processes(IDX["europe-west3"], procs)
    assert set(s[:6]) == {8, 9, 6, 7, 5, 14}
    assert set(s[:4]) == {8, 9, 6, 7}


def test_discover_same_region():  # protocol/base.rs:349-409 (fq=3, wq=4)
    regs = ["asia-east1", "asia-east1", "europe-north1", "europe-north1", "europe-west1"]
    s = O.sort_processes(IDX["europe-north1"], [(i, IDX[r]) for i, r in enumerate(regs)])
    assert set(s[:3]) == {2, 3, 4}
    assert set(s[:4]) == {2, 3, 4, 0}


def test_client_discover_closest():  # client/mod.rs:196-232 (shard 0 part)
    regs = ["asia-east1", "australia-southeast1", "europe-west1"]
    s = O.sort_processes(IDX["europe-west2"], [(i, IDX[r]) for i, r in enumerate(regs)])
    assert s[0] == 2


# ---------------------------------------------------------------- building blocks
def d(s, q):
    return (s, q)


def test_quorum_deps_all():  # quorum.rs:119-133
    deps = {d(1, 1), d(1, 2)}
    assert not O.quorum_deps(3, [deps, deps], 1)[1]
    assert O.quorum_deps(3, [deps, deps, deps], 1)[1]


def test_quorum_deps_check_threshold():  # quorum.rs:135-228
    d12, d123, d1 = {d(1, 1), d(1, 2)}, {d(1, 1), d(1, 2), d(1, 3)}, {d(1, 1)}
    for t, ok in ((1, True), (2, True), (3, True), (4, False)):
        u, _, th, _ = O.quorum_deps(3, [d12, d12, d12], t)
        assert u == d12 and th == ok
    for t, ok in ((1, True), (2, False), (3, False), (4, False)):
        u, _, th, _ = O.quorum_deps(3, [d123, d12, d12], t)
        assert u == d123 and th == ok
        u, _, th, _ = O.quorum_deps(3, [d123, d12, d1], t)
        assert u == d123 and th == ok


def test_quorum_deps_check_equal():  # quorum.rs:230-308
    d1, d12 = {d(1, 1)}, {d(1, 1), d(1, 2)}
    d13, d23, d123 = {d(1, 1), d(1, 3)}, {d(1, 2), d(1, 3)}, {d(1, 1), d(1, 2), d(1, 3)}
    cases = [(2, [set(), set()], set(), True), (3, [set(), set(), d1], d1, False),
             (3, [d1, d1, d1], d1, True), (2, [d12, d12], d12, True), (2, [d12, set()], d12, False),
             (3, [d12, d13, d23], d123, False),
             (3, [d1, {d(1, 2)}, d12], d12, False)]  # check_equal_regression_test
    for fq, reps, u, eq in cases:
        got = O.quorum_deps(fq, reps, 1)
        assert got[0] == u and got[3] == eq, (fq, reps)


def test_key_deps_flow():  # deps/keys/mod.rs:149-381 (A=1, B=2, C=3)
    A, B, C = 1, 2, 3
    q = lambda keys: ("deps", keys, False)
    queries = [q([A]), q([B]), q([A, B]), q([C]), ("noop_deps",)]
    script, expect = [], []

    def step(op, exp):
        script.append(op)
        script.extend(queries)
        expect.append(exp)

    D = lambda *xs: {(1, x) for x in xs}
    script.extend(queries)
    expect0 = [set(), set(), set(), set(), set()]
    step(("add", (1, 1), [A], False), [D(1), set(), D(1), set(), D(1)])
    step(("noop", (1, 2)), [D(1, 2), D(2), D(1, 2), D(2), D(1, 2)])
    step(("add", (1, 3), [B], False), [D(1, 2), D(2, 3), D(1, 2, 3), D(2), D(1, 2, 3)])
    step(("add", (1, 4), [B], False), [D(1, 2), D(2, 4), D(1, 2, 4), D(2), D(1, 2, 4)])
    step(("add", (1, 5), [A, B], False), [D(2, 5), D(2, 5), D(2, 5), D(2), D(2, 5)])
    step(("add", (1, 6), [A], False), [D(2, 6), D(2, 5), D(2, 5, 6), D(2), D(2, 5, 6)])
    step(("add", (1, 7), [C], False), [D(2, 6), D(2, 5), D(2, 5, 6), D(2, 7), D(2, 5, 6, 7)])
    step(("noop", (1, 8)), [D(8, 6), D(8, 5), D(8, 5, 6), D(8, 7), D(8, 5, 6, 7)])
    step(("add", (1, 9), [B], False), [D(8, 6), D(8, 9), D(8, 6, 9), D(8, 7), D(8, 6, 7, 9)])
    res = O.key_deps_script(script)
    assert res[:5] == expect0
    pos = 5
    for exp in expect:
        pos += 1  # the mutating op itself
        assert res[pos:pos + 5] == exp
        pos += 5


@pytest.mark.parametrize("nfr", [False, True])
def test_key_deps_read_deps(nfr):  # deps/keys/mod.rs:383-485
    A = 1
    rd, wr = ("deps", [A], True), ("deps", [A], False)
    D = lambda *xs: {(1, x) for x in xs}
    script = [rd, wr,
              ("add", (1, 1), [A], True), rd, wr,
              ("add", (1, 2), [A], True), rd, wr,
              ("add", (1, 3), [A], False), rd, wr,
              ("add", (1, 4), [A], False), rd, wr,
              ("add", (1, 5), [A], True), rd, wr]
    r = O.key_deps_script(script, nfr=nfr)
    assert r[0] == set() and r[1] == set()
    assert r[3] == set() and r[4] == (set() if nfr else D(1))
    assert r[6] == set() and r[7] == (set() if nfr else D(2))
    assert r[9] == D(3) and r[10] == (D(3) if nfr else D(2, 3))
    assert r[12] == D(4) and r[13] == (D(4) if nfr else D(2, 4))
    assert r[15] == D(4) and r[16] == (D(4) if nfr else D(4, 5))


def test_gc_flow():  # protocol/gc/clock.rs:187-251 (n=2)
    ops = [("stable",),
           ("add", (1, 2)), ("stable",),
           ("add", (1, 1)), ("stable",),
           ("update", 2, [0, 0]), ("stable",),
           ("update", 2, [1, 0]), ("stable",), ("stable",),  # gc2 committed 11 and 13
           ("add", (1, 3)), ("update", 2, [3, 0]), ("stable",), ("stable",)]
    r = O.gc_script(2, ops)
    assert r[0] == ([], [0, 0])
    assert r[2] == ([], [0, 0])
    assert r[4] == ([], [2, 0])
    assert r[6] == ([], [2, 0])
    assert r[8] == ([(1, 1, 1)], [2, 0])  # dot11 stable
    assert r[9] == ([], [2, 0])
    assert r[12] == ([(1, 2, 3)], [3, 0])  # dot12, dot13
    assert r[13] == ([], [3, 0])


def conflict_spec(rate, keys=1, pool=1, client=1):
    return O.make_spec(ATLAS, 3, 1, [0, 1, 2], [0], keys_per_command=keys, conflict_rate=rate,
                       pool_size=pool, seed=11)


def test_workload_gen_cmd_key():  # client/workload.rs:223-275 (C7 ids)
    k, _ = O.workload_keys(conflict_spec(100), 1, 1)
    assert k.tolist() == [[0]]            # "CONFLICT0"
    k, _ = O.workload_keys(conflict_spec(0), 1, 1)
    assert k.tolist() == [[1 + 1]]        # "1" -> pool_size + client id


@pytest.mark.parametrize("rate", [1, 2, 10, 50])
def test_workload_conflict_rate(rate):  # client/workload.rs:350-398 (1M commands)
    k, _ = O.workload_keys(conflict_spec(rate), 1, 1_000_000)
    pct = (k[:, 0] == 0).sum() * 100.0 / k.shape[0]
    assert round(pct) == rate


def test_workload_two_keys_are_distinct():  # workload.rs:188-197 with pool 1
    k, _ = O.workload_keys(conflict_spec(50, keys=2), 3, 1000)
    assert (k[:, 0] != k[:, 1]).all() and set(k.ravel().tolist()) == {0, 1 + 3}


# ------------------------------------------------------------------ runner
def runner_run(f, clients_per_process):  # sim/runner.rs:730-816
    s = O.make_spec(BASIC, 3, f, [IDX["asia-east1"], IDX["us-central1"], IDX["us-west1"]],
                    [IDX["us-west1"], IDX["us-west2"]], clients_per_region=clients_per_process,
                    commands_per_client=1000, conflict_rate=100, pool_size=1,
                    gc_interval_ms=100, executed_notification_ms=50, extra_sim_time_ms=1000)
    r = O.sim_run(s)
    expected = 1000 * clients_per_process
    assert r["issued"][IDX["us-west1"]] == expected and r["issued"][IDX["us-west2"]] == expected
    assert (r["stable"] == 2 * expected).all()  # every command GC-ed at every process
    return r["latency"][IDX["us-west1"]], r["latency"][IDX["us-west2"]]


def test_runner_single_client_per_process():  # sim/runner.rs:818-843
    w1, w2 = runner_run(0, 1)
    assert hist_mean(w1) == 0.0 and hist_mean(w2) == 24.0
    w1, w2 = runner_run(1, 1)
    assert hist_mean(w1) == 34.0 and hist_mean(w2) == 58.0


def test_runner_multiple_clients_per_process():  # sim/runner.rs:845-864
    a1, a2 = runner_run(1, 1)
    b1, b2 = runner_run(1, 10)
    assert hist_mean(a1) == hist_mean(b1) and hist_cov(a1) == hist_cov(b1)
    assert hist_mean(a2) == hist_mean(b2) and hist_cov(a2) == hist_cov(b2)


# ------------------------------------------------- protocol simulations
def sim_test(protocol, n, f, read_only=0, keys=2, nfr=False, seed=3):
    """fantoch_ps/src/protocol/mod.rs:702-768: 10 clients per process x 100
    commands, conflict 50 % over a pool of 1, message reordering, 10 s of
    extra time; regions = the planet's first n (planet.regions() is HashMap
    order in the reference; name order here, C12)."""
    s = O.make_spec(protocol, n, f, list(range(n)), list(range(n)), clients_per_region=10,
                    commands_per_client=100, keys_per_command=keys, conflict_rate=50,
                    pool_size=1, read_only_pct=read_only, gc_interval_ms=100,
                    executed_notification_ms=100, extra_sim_time_ms=10_000, reorder=True,
                    nfr=nfr, seed=seed)
    r = O.sim_run(s)
    # check_monitors (mod.rs:787-801): every process executed every key in the same order
    assert len(set(r["monitor_hash"].tolist())) == 1
    # check_metrics (mod.rs:878-942)
    total = 100 * 10 * n
    assert r["fast"].sum() + r["slow"].sum() == total
    assert r["stable"].sum() == n * total
    assert all(len(e) == total for e in r["executed"])
    return r


def test_sim_atlas_3_1():  # protocol/mod.rs:331-341
    assert sim_test(ATLAS, 3, 1)["slow"].sum() == 0


def test_sim_atlas_5_2():  # protocol/mod.rs:355-365
    assert sim_test(ATLAS, 5, 2)["slow"].sum() > 0


def test_sim_atlas_5_1():  # protocol/mod.rs:343-353 (the reference builds config!(3, 1) here)
    assert sim_test(ATLAS, 3, 1, seed=4)["slow"].sum() == 0


@pytest.mark.parametrize("seed", [3, 4])
def test_sim_atlas_5_2_nfr(seed):  # protocol/mod.rs:367-383 (20 % single-key reads, NFR)
    r = sim_test(ATLAS, 5, 2, read_only=20, keys=1, nfr=True, seed=seed)
    assert r["slow"].sum() > 0
    assert r["slow_reads"].sum() == 0 and r["fast_reads"].sum() > 0  # slow_paths_reads() == 0


def test_sim_epaxos_3_1():  # protocol/mod.rs:454-464
    assert sim_test(EPAXOS, 3, 1)["slow"].sum() == 0


def test_sim_epaxos_5_2():  # protocol/mod.rs:466-476
    assert sim_test(EPAXOS, 5, 2)["slow"].sum() > 0


@pytest.mark.parametrize("seed", [3, 4])
def test_sim_epaxos_7_3_nfr(seed):  # protocol/mod.rs:478-493 (100 % single-key reads, NFR)
    r = sim_test(EPAXOS, 7, 3, read_only=100, keys=1, nfr=True, seed=seed)
    assert r["slow"].sum() == 0
    assert r["slow_reads"].sum() == 0 and r["fast_reads"].sum() > 0  # slow_paths_reads() == 0


def test_sim_is_deterministic_and_seeded():
    a = sim_test(ATLAS, 3, 1, seed=5)
    b = sim_test(ATLAS, 3, 1, seed=5)
    c = sim_test(ATLAS, 3, 1, seed=6)
    assert a["trace"] == b["trace"] and all((x == y).all() for x, y in zip(a["executed"], b["executed"]))
    assert a["trace"] != c["trace"]


def test_batch_equals_single_runs():
    specs = [O.make_spec(EPAXOS, 5, 2, list(range(5)), list(range(5)), commands_per_client=50,
                         conflict_rate=c, seed=9, instance=i) for i, c in enumerate((0, 2, 10, 50, 100))]
    many = O.sim_batch(specs, threads=4)
    for s, m in zip(specs, many):
        one = O.sim_run(s)
        assert one["trace"] == m["trace"] and (one["latency"] == m["latency"]).all()
