"""GPU simulator (fx_sim_run) vs the simulator oracle, bit for bit: per-process
execution order, per-command client latencies (so every latency histogram),
fast/slow/stable counters, the action trace and where the run stopped.  GPU
only; instances are small enough for the oracle to finish in seconds."""
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


def to_oracle(s):
    o = O.SimSpec()
    for name, _ in _lib.SimSpec._fields_:
        v = getattr(s, name)
        if name in ("process_regions", "client_regions"):
            arr = getattr(o, name)
            for i in range(len(v)):
                arr[i] = v[i]
        else:
            setattr(o, name, v)
    return o


def client_regions(s):
    out = []
    for r in range(s.num_client_regions):
        out += [s.client_regions[r]] * s.clients_per_region
    return out


def assert_instance_parity(res, i, s, o):
    g_exec = res.executed(i)
    for p in range(s.n):
        assert np.array_equal(g_exec[p], o["executed"][p]), "process %d order differs" % (p + 1)
    assert int(res.err[i]) == 0
    assert [int(x) for x in res.fast(i)] == [int(x) for x in o["fast"]]
    assert [int(x) for x in res.slow(i)] == [int(x) for x in o["slow"]]
    assert [int(x) for x in res.stable(i)] == [int(x) for x in o["stable"]]
    assert res.end_ms(i) == o["end_ms"]
    assert res.events(i) == o["events"]
    assert res.trace(i) == o["trace"]
    # client latency histograms per region (clients_latencies, runner.rs:619-634)
    lat = res.latencies(i)
    regs = client_regions(s)
    hist = np.zeros_like(o["latency"])
    for c, r in enumerate(regs):
        np.add.at(hist[r], np.minimum(lat[c, :s.commands_per_client], hist.shape[1] - 1), 1)
    assert np.array_equal(hist, o["latency"])
    # per-instance latency sum (FX_SIM_STAT_LAT_SUM, the per-placement mean of configs[2])
    lat_sum = int(sum(ms * int(c) for h in o["latency"] for ms, c in enumerate(h) if c))
    assert int(res.stats[i, _lib.FX_SIM_STAT_LAT_SUM]) == lat_sum


def run_and_compare(specs, **kw):
    res = S.run(specs, planet(), **kw)
    bad = [(i, int(e)) for i, e in enumerate(res.err) if e]
    assert not bad, "instances failed: %s" % bad[:8]
    orc = O.sim_batch([to_oracle(s) for s in specs], threads=8)
    for i, (s, o) in enumerate(zip(specs, orc)):
        assert o["status"] == 0
        assert_instance_parity(res, i, s, o)
    # batch histograms = sums of the oracle's
    lat = sum(o["latency"] for o in orc)
    assert np.array_equal(res.latency_hist[:, :lat.shape[1]], lat[:, :res.latency_hist.shape[1]])
    assert np.array_equal(res.chain, sum(o["chain"] for o in orc)[:res.chain.shape[0]])
    assert np.array_equal(res.delay, sum(o["delay"] for o in orc)[:res.delay.shape[0]])
    return res, orc


def test_config0_atlas_n3_gcp_reference_order():
    """BASELINE configs[0]: Atlas n=3 f=1, GCP planet (simulation.rs gcp_planet
    regions), 1 client per region, 2 % conflicts, 1000 commands per client."""
    pl = planet()
    regs = pl.ids(S.GCP5[:3])
    s = S.spec(S.ATLAS, 3, 1, regs, regs, commands_per_client=1000, conflict_rate=2, seed=1)
    res, orc = run_and_compare([s])
    assert all(len(e) >= 2990 for e in res.executed(0))


@pytest.mark.parametrize("protocol,n,f", [(S.EPAXOS, 5, 2), (S.ATLAS, 5, 1), (S.ATLAS, 5, 2)])
def test_conflict_sweep_n5(protocol, n, f):
    """configs[1] shape: seeds x conflict {0,2,10,50,100} %, n = 5 (100 commands)."""
    pl = planet()
    regs = pl.ids(S.GCP5[:n])
    specs = [S.spec(protocol, n, f, regs, regs, commands_per_client=100, conflict_rate=c,
                    seed=77, instance=i) for i, c in enumerate([0, 2, 10, 50, 100] * 4)]
    run_and_compare(specs)


def test_config1_full_size_bench_instances():
    """BASELINE configs[1] at the bench's full size: EPaxos n=5 f=2, GCP regions,
    1 client per region, 1,000 commands per client, two instances per conflict
    rate {100,50,10,2,0} % taken from the bench's own rate-major enumeration
    (bench_sim.global_spec: seed 20250213, instance = global index, 4,096 seeds
    per rate), bit-exact vs the oracle like every other instance."""
    pl = planet()
    regs = pl.ids(S.GCP5[:5])
    specs = []
    for k, c in enumerate([100, 50, 10, 2, 0]):
        for g in (k * 4096, k * 4096 + 4095):
            specs.append(S.spec(S.EPAXOS, 5, 2, regs, regs, commands_per_client=1000, conflict_rate=c,
                                seed=20250213, instance=g))
    res, orc = run_and_compare(specs)
    # the run stops when the last client is done: a far process may still
    # hold a few committed commands (the bench executes 24,996 of 25,000)
    assert all(4900 <= len(e) <= 5000 for i in range(len(specs)) for e in res.executed(i))


def test_region_subsets_n7():
    """configs[2] shape: Atlas n=7 f=1/2 over region subsets of the 20 GCP regions."""
    import itertools
    pl = planet()
    subsets = list(itertools.combinations(range(pl.R), 7))[::9973][:12]
    specs = [S.spec(S.ATLAS, 7, 1 + (i % 2), list(sub), list(sub), commands_per_client=60,
                    conflict_rate=10, seed=5, instance=i) for i, sub in enumerate(subsets)]
    run_and_compare(specs)


def test_two_clients_per_region_two_keys():
    pl = planet()
    regs = pl.ids(S.GCP5[:5])
    specs = [S.spec(S.EPAXOS, 5, 2, regs, regs, clients_per_region=2, commands_per_client=60,
                    keys_per_command=2, conflict_rate=c, seed=3, instance=i)
             for i, c in enumerate([10, 50, 90])]
    run_and_compare(specs)


def test_extra_time_and_client_regions_apart():
    """Clients in regions without a process, extra simulated time after the
    clients finish (runner.rs:285-311) and executed notifications simulated."""
    pl = planet()
    p = pl.ids(["asia-east1", "us-central1", "us-west1"])
    c = pl.ids(["us-west1", "us-west2", "europe-west3"])
    specs = [S.spec(S.ATLAS, 3, 1, p, c, commands_per_client=80, conflict_rate=100,
                    gc_interval_ms=100, executed_notification_ms=50, extra_sim_time_ms=1000,
                    seed=2, instance=i) for i in range(3)]
    run_and_compare(specs, flags=_lib.FX_SIM_FLAG_EXEC_NOTIFICATIONS)
    run_and_compare(specs)


def test_no_gc():
    pl = planet()
    regs = pl.ids(S.GCP5[:5])
    specs = [S.spec(S.EPAXOS, 5, 2, regs, regs, commands_per_client=80, conflict_rate=50,
                    gc_interval_ms=0, seed=4, instance=i) for i in range(4)]
    run_and_compare(specs)


def test_capacity_escalation_is_exact():
    """configs[2]-style placements where a far replica lags: with small tables
    the first launch stops some instances with FX_ERR_SIM_CAPACITY;
    fx_sim_run_tiered reruns them with larger tables and removes their partial
    histogram samples, so every output still equals the oracle's."""
    pl = planet()
    subs = [["asia-east1", "europe-west1", "europe-west2", "europe-west4", "us-east4"],
            ["asia-east2", "europe-west1", "europe-west3", "europe-west6", "us-west1"],
            ["asia-northeast2", "europe-north1", "europe-west2", "europe-west3", "europe-west4"],
            ["asia-south1", "europe-north1", "southamerica-east1", "australia-southeast1", "europe-west1"]]
    specs = [S.spec(S.ATLAS, 5, 1, pl.ids(sorted(r)), pl.ids(sorted(r)), commands_per_client=80, conflict_rate=c,
                    seed=9, instance=i) for i, (r, c) in enumerate((r, c) for r in subs for c in (2, 50))]
    # 24 messages / 16 dots in flight: the lagging placements outgrow them
    res, _ = run_and_compare(specs, ring_entries=24, dot_slots=16)
    assert res.reruns > 0


def test_config2_bench_placements_full_size():
    """BASELINE configs[2] at the bench's size: placements taken from
    bench_placements' own global enumeration (every (n, f) group, spread over
    the 186,048-placement sweep), Atlas, one client per process region, 100
    commands per client, 2 % conflicts, seed 20250213, instance = placement
    id, exactly as `bench.py --mode placements` builds them; bit-exact vs the
    oracle, one launch per geometry."""
    import bench_placements as BP
    pl = planet()
    allp = BP.enumerate_placements(pl.R)
    assert len(allp) == 186048
    for n in (5, 7):
        ids = []
        for f in (1, 2):  # 6 placements spread over each (n, f) group
            grp = [g for g, (n2, f2, _) in enumerate(allp) if (n2, f2) == (n, f)]
            ids += [grp[k * (len(grp) - 1) // 5] for k in range(6)]
        specs = [S.spec(S.ATLAS, n, allp[g][1], list(allp[g][2]), list(allp[g][2]), commands_per_client=100,
                        conflict_rate=2, seed=20250213, instance=g) for g in ids]
        run_and_compare(specs)


def basic_runner_specs(f, clients_per_process):
    """sim/runner.rs:730-816 run(f, clients_per_process): Basic, n = 3 in
    asia-east1 / us-central1 / us-west1, clients in us-west1 and us-west2,
    100 % conflicts on a pool of 1, 1,000 commands per client, GC every 100 ms,
    one extra simulated second."""
    pl = planet()
    return [S.spec(S.BASIC, 3, f, pl.ids(["asia-east1", "us-central1", "us-west1"]),
                   pl.ids(["us-west1", "us-west2"]), clients_per_region=clients_per_process,
                   commands_per_client=1000, conflict_rate=100, pool_size=1, gc_interval_ms=100,
                   executed_notification_ms=50, extra_sim_time_ms=1000)]


def region_hist(res, s, region):
    """The client latency histogram of one region, from the GPU's latency log."""
    lat = res.latencies(0)
    regs = client_regions(s)
    h = np.zeros(int(lat.max()) + 1, np.int64)
    for c, r in enumerate(regs):
        if r == region:
            np.add.at(h, lat[c, :s.commands_per_client], 1)
    return h


def test_runner_basic_reference_means_on_gpu():
    """The reference's only numeric simulator KAT (runner.rs:818-843,
    runner_single_client_per_process) asserted on GPU output: us-west1 /
    us-west2 mean latency 0 / 24 ms at f = 0 and 34 / 58 ms at f = 1, every
    command stable at every process (runner.rs:800-812); bit-exact vs the
    oracle besides."""
    from test_sim_oracle import hist_mean
    pl = planet()
    w1, w2 = pl.index["us-west1"], pl.index["us-west2"]
    for f, means in ((0, (0.0, 24.0)), (1, (34.0, 58.0))):
        specs = basic_runner_specs(f, 1)
        # f = 0: the us-west1 client's commands commit at its own process in
        # 0 ms, so all 1,000 are issued at t = 0 and wait for the far
        # replicas: ~1,000 live dots and ~4,000 messages in flight, the
        # large-instance kernel's tables
        kw = dict(large=True, ring_entries=8192, dot_slots=4096) if f == 0 else {}
        res, _ = run_and_compare(specs, **kw)
        assert (hist_mean(region_hist(res, specs[0], w1)), hist_mean(region_hist(res, specs[0], w2))) == means
        assert [int(x) for x in res.stable(0)] == [2000] * 3


def test_runner_basic_multiple_clients_on_gpu():
    """runner.rs:845-864 runner_multiple_clients_per_process on GPU output: 1 and
    10 clients per region give the same mean and cov in both regions."""
    from test_sim_oracle import hist_cov, hist_mean
    pl = planet()
    out = []
    for cpp in (1, 10):
        specs = basic_runner_specs(1, cpp)
        res, _ = run_and_compare(specs)
        assert [int(x) for x in res.stable(0)] == [2000 * cpp] * 3
        out.append([region_hist(res, specs[0], pl.index[r]) for r in ("us-west1", "us-west2")])
    for one, ten in zip(out[0], out[1]):
        assert hist_mean(one) == hist_mean(ten) and hist_cov(one) == hist_cov(ten)
