"""The large-instance GPU simulator (sim_big.hip, FX_SIM_FLAG_LARGE or any
batch the all-on-chip kernel cannot hold) vs the simulator oracle, bit for
bit: per-process execution order, client latencies (every latency
histogram), fast / slow / stable / read counters, the action trace and where
the run stopped.

* BASELINE configs[3]: Atlas n=5 f=1 and EPaxos n=5 f=2, 64 clients per region
  (320 per instance), 100 % conflicts, SCCs of hundreds of commands.
* The reference's own protocol simulations (fantoch_ps/src/protocol/mod.rs:
  702-768 sim_test: 10 clients per process, 2 keys, conflict 50 % over a pool
  of 1, message reordering, GC and executed notifications every 100 ms,
  10 s of extra time), with check_monitors / check_metrics
  (mod.rs:787-801, 878-942) asserted on the GPU's own output.
* Instances of the all-on-chip kernel's shapes run on both kernels: identical
  outputs (the large kernel simulates the GC traffic the small one evaluates).
GPU only; instances sized for the oracle to finish in seconds."""
import numpy as np
import pytest

from fantoch_amd import _lib
from fantoch_amd import sim as S
from oracle import oracle_lib as O

pytestmark = pytest.mark.gpu

PLANET = None


def planet():
    global PLANET
    if PLANET is None:
        PLANET = S.Planet()
    return PLANET


def client_regions(s):
    out = []
    for r in range(s.num_client_regions):
        out += [s.client_regions[r]] * s.clients_per_region
    return out


def mix64(x):
    M = (1 << 64) - 1
    x = (x + 0x9E3779B97F4A7C15) & M
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M
    return x ^ (x >> 31)


def monitor_hash(mon):
    """The oracle's ExecutionOrderMonitor hash (sim_oracle.cpp fill)."""
    h = 0x1234567
    for key in sorted(mon):
        h = mix64(h ^ (key << 32))
        for c, q in mon[key]:
            h = mix64(h ^ (c << 40) ^ q)
    return h


def assert_instance_parity(res, i, s, o):
    g_exec = res.executed(i)
    for p in range(s.n):
        assert np.array_equal(g_exec[p], o["executed"][p]), "process %d order differs" % (p + 1)
    assert int(res.err[i]) == 0
    for name in ("fast", "slow", "stable", "fast_reads", "slow_reads"):
        assert [int(x) for x in getattr(res, name)(i)] == [int(x) for x in o[name]], name
    assert res.end_ms(i) == o["end_ms"]
    assert res.events(i) == o["events"]
    assert res.trace(i) == o["trace"]
    lat = res.latencies(i)
    hist = np.zeros_like(o["latency"])
    for c, r in enumerate(client_regions(s)):
        np.add.at(hist[r], np.minimum(lat[c, :s.commands_per_client], hist.shape[1] - 1), 1)
    assert np.array_equal(hist, o["latency"])
    # the GPU's monitors, rebuilt from its own outputs, hash as the oracle's
    mons = res.monitors(i)
    assert [monitor_hash(m) for m in mons] == [int(x) for x in o["monitor_hash"]]
    return mons


def run_and_compare(specs, **kw):
    res = S.run(specs, planet(), **kw)
    bad = [(i, int(e)) for i, e in enumerate(res.err) if e]
    assert not bad, "instances failed: %s" % bad[:8]
    orc = O.sim_batch([O.spec_from(s) for s in specs], threads=8)
    mons = []
    for i, (s, o) in enumerate(zip(specs, orc)):
        assert o["status"] == 0
        mons.append(assert_instance_parity(res, i, s, o))
    lat = sum(o["latency"] for o in orc)
    assert np.array_equal(res.latency_hist[:, :lat.shape[1]], lat[:, :res.latency_hist.shape[1]])
    assert np.array_equal(res.chain, sum(o["chain"] for o in orc)[:res.chain.shape[0]])
    assert np.array_equal(res.delay, sum(o["delay"] for o in orc)[:res.delay.shape[0]])
    return res, orc, mons


@pytest.mark.parametrize("protocol,f", [(S.ATLAS, 1), (S.EPAXOS, 2)])
def test_config3_64_clients_per_region_full_conflict(protocol, f):
    """BASELINE configs[3]: n = 5, 64 clients per region (320 per instance),
    100 % conflicts (pool of 1): every command conflicts with every other."""
    pl = planet()
    regs = sorted(pl.ids(S.GCP5))
    specs = [S.spec(protocol, 5, f, regs, regs, clients_per_region=64, commands_per_client=30,
                    conflict_rate=100, seed=11, instance=i) for i in range(2)]
    res, orc, _ = run_and_compare(specs)
    # large SCCs: the chain-size histogram reaches far past singletons
    assert int(np.nonzero(res.chain)[0].max()) >= 64
    assert all(len(e) >= 9000 for e in res.executed(0))


def sim_test_specs(protocol, n, f, read_only=0, keys=2, nfr=False, seeds=(3,)):
    """protocol/mod.rs:702-768 sim_test at the reference's parameters."""
    return [S.spec(protocol, n, f, list(range(n)), list(range(n)), clients_per_region=10,
                   commands_per_client=100, keys_per_command=keys, conflict_rate=50, pool_size=1,
                   read_only_pct=read_only, gc_interval_ms=100, executed_notification_ms=100,
                   extra_sim_time_ms=10_000, reorder=True, nfr=nfr, seed=sd) for sd in seeds]


def check_sim_test(res, i, mons):
    """check_monitors + check_metrics (mod.rs:787-801, 878-942) on GPU output."""
    s = res.specs[i]
    assert all(m == mons[0] for m in mons[1:]), "processes executed some key in different orders"
    total = s.commands_per_client * s.clients_per_region * s.n
    assert int(res.fast(i).sum() + res.slow(i).sum()) == total
    assert int(res.stable(i).sum()) == s.n * total
    assert all(len(e) == total for e in res.executed(i))


@pytest.mark.parametrize("name,protocol,n,f,ro,keys,nfr,slow", [
    ("sim_atlas_3_1", S.ATLAS, 3, 1, 0, 2, False, "zero"),          # mod.rs:331-341
    ("sim_atlas_5_2", S.ATLAS, 5, 2, 0, 2, False, "some"),          # mod.rs:355-365
    ("sim_atlas_5_2_nfr", S.ATLAS, 5, 2, 20, 1, True, "some"),      # mod.rs:367-383
    ("sim_epaxos_3_1", S.EPAXOS, 3, 1, 0, 2, False, "zero"),        # mod.rs:454-464
    ("sim_epaxos_5_2", S.EPAXOS, 5, 2, 0, 2, False, "some"),        # mod.rs:466-476
    ("sim_epaxos_7_3_nfr", S.EPAXOS, 7, 3, 100, 1, True, "zero"),   # mod.rs:478-493
])
def test_reference_protocol_simulations(name, protocol, n, f, ro, keys, nfr, slow):
    specs = sim_test_specs(protocol, n, f, ro, keys, nfr, seeds=(3, 4))
    res, orc, mons = run_and_compare(specs)
    for i in range(len(specs)):
        check_sim_test(res, i, mons[i])
        if slow == "zero":
            assert int(res.slow(i).sum()) == 0
        else:
            assert int(res.slow(i).sum()) > 0
        if nfr:  # assert_eq!(metrics.slow_paths_reads(), 0) (mod.rs:381, 492)
            assert int(res.slow_reads(i).sum()) == 0 and int(res.fast_reads(i).sum()) > 0


def test_small_shapes_equal_on_both_kernels():
    """configs[1]'s shape (EPaxos n=5 f=2, 1 client per region, GC every 10 ms)
    and configs[2]'s (Atlas n=7): the large kernel simulates every GC action
    the all-on-chip kernel evaluates in closed form; every output is equal."""
    pl = planet()
    regs = pl.ids(S.GCP5[:5])
    specs = [S.spec(S.EPAXOS, 5, 2, regs, regs, commands_per_client=100, conflict_rate=c,
                    seed=77, instance=i) for i, c in enumerate([0, 2, 10, 50, 100])]
    a = S.run(specs, pl)
    b = S.run(specs, pl, large=True)
    for i in range(len(specs)):
        assert int(a.err[i]) == 0 and int(b.err[i]) == 0
        for p in range(5):
            assert np.array_equal(a.executed(i)[p], b.executed(i)[p])
        assert np.array_equal(a.latencies(i), b.latencies(i))
        for name in ("fast", "slow", "stable"):
            assert np.array_equal(getattr(a, name)(i), getattr(b, name)(i)), name
        assert a.trace(i) == b.trace(i) and a.end_ms(i) == b.end_ms(i) and a.events(i) == b.events(i)
        # both kernels record every dot's rifl (dot_client): equal monitors
        assert a.rifls(i) == b.rifls(i) and a.monitors(i) == b.monitors(i)
    assert np.array_equal(a.chain, b.chain) and np.array_equal(a.delay, b.delay)
    assert np.array_equal(a.latency_hist, b.latency_hist)


def test_extra_time_and_client_regions_apart_large():
    pl = planet()
    p = pl.ids(["asia-east1", "us-central1", "us-west1"])
    c = pl.ids(["us-west1", "us-west2", "europe-west3"])
    specs = [S.spec(S.ATLAS, 3, 1, p, c, clients_per_region=20, commands_per_client=40, conflict_rate=100,
                    gc_interval_ms=100, executed_notification_ms=50, extra_sim_time_ms=1000,
                    reorder=bool(i % 2), seed=2, instance=i) for i in range(4)]
    run_and_compare(specs)


def test_large_capacity_escalation_is_exact():
    """Tiny tables: the first launch stops instances with FX_ERR_SIM_CAPACITY;
    fx_sim_run_tiered reruns them twice larger and removes their partial
    histogram samples, so every output still equals the oracle's."""
    specs = sim_test_specs(S.ATLAS, 3, 1, seeds=(5, 6, 7))
    res, _, _ = run_and_compare(specs, ring_entries=128, dot_slots=48)
    assert res.reruns > 0


def test_large_arena_plan():
    lib = _lib.load()
    import ctypes
    pl = planet()
    regs = sorted(pl.ids(S.GCP5))
    s = S.spec(S.ATLAS, 5, 1, regs, regs, clients_per_region=64, commands_per_client=30, conflict_rate=100)
    b = ctypes.c_uint64()
    assert lib.fx_sim_plan_large(ctypes.byref(s), 0, 0, ctypes.byref(b)) == 0
    assert 0 < b.value < 8 << 20
