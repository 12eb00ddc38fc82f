"""bench.py --mode sim: BASELINE configs[1] on the GPU simulator (fx_sim_run).

Workload per GPU (weak scaling): EPaxos n=5 f=2 (Config::new(5, 2)) on the GCP
planet with fantoch_ps/src/bin/simulation.rs's regions (gcp_planet, first n),
1 client per region, pool 1, 1 key per command, GC and executed
notifications every 10 ms (the binary's config! macro), Runner::run(None);
`--seeds` seeds x conflict {0,2,10,50,100}% instances, `--cmds` commands per
client (default 1000).

bench.py --mode dense-sim: BASELINE configs[3] on the same entry point (the
large-instance kernel, sim_big.hip): Atlas n=5 f=1 and EPaxos n=5 f=2
(`--protocol both`, alternating instances), 64 clients per region (320 per
instance), 100 % conflicts over a pool of 1, `--cmds` commands per client
(default 50).  Rank r simulates global instances
[r P, (r + 1) P), P = seeds x rates, each with its own C6 RNG stream, the
heaviest conflict rate first.  One step = every instance simulated from
Runner::new to the end of Runner::run in one kernel launch (inputs resident
in HBM); outputs = per-process execution orders, client latency histograms,
protocol counters.

value = commands executed by every process's GraphExecutor, summed over the
instances of every rank, / the max-over-ranks time of the timed steps.
"""
import ctypes
import json
import os
import time

import numpy as np

METRIC = "executed cmds/sec (node) for batched Atlas/EPaxos sims; % of HBM roofline"
HBM_PEAK_GBPS = 8000.0


def protocol_of(S, args, g):
    """(protocol, f) of global instance g: --protocol both alternates Atlas
    n f=1 and EPaxos (f = n / 2), the two configs of BASELINE configs[3]."""
    if args.protocol == "both":
        return (S.ATLAS, 1) if g % 2 == 0 else (S.EPAXOS, args.n // 2)
    return (S.EPAXOS if args.protocol == "epaxos" else S.ATLAS), args.f


def rate_list(args):
    """Conflict rates, heaviest first (the instances of a rank are rate-major)."""
    return sorted((int(c) for c in args.conflicts.split(",")), reverse=True)


def global_spec(S, args, g, regs):
    """Global instance g: rank g // P's instance g % P, P = seeds x rates,
    rate-major (heaviest first), with its own C6 RNG stream (instance = g)."""
    conflicts = rate_list(args)
    per = args.seeds * len(conflicts)
    c = conflicts[(g % per) // args.seeds]
    proto, f = protocol_of(S, args, g)
    return S.spec(proto, args.n, f, regs, regs, clients_per_region=args.clients_per_region,
                  commands_per_client=args.cmds, conflict_rate=c, seed=args.seed, instance=g), c


def local_specs(S, args, rank, planet):
    """Rank r's instances: the contiguous global range [r P, (r + 1) P)."""
    conflicts = rate_list(args)
    regs = planet.ids(S.GCP5[:args.n])
    per = args.seeds * len(conflicts)
    specs, rates = [], []
    for g in range(rank * per, (rank + 1) * per):
        sp, c = global_spec(S, args, g, regs)
        specs.append(sp)
        rates.append(c)
    return specs, rates, conflicts


ROW_FIELDS = ["instance", "conflict_pct", "executed", "fast_paths", "slow_paths", "status"]


def instance_rows(torch, gid0, rates, executed_len, stats, err, n):
    """[instances, 6] int64 rows (ROW_FIELDS) of one rank's batch: executed
    summed over the n processes, Fast / Slow paths summed, the FX_* status."""
    from fantoch_amd import _lib
    N = len(rates)
    dev = executed_len.device
    st = stats.view(N, _lib.FX_SIM_STATS)
    gid = torch.arange(N, dtype=torch.int64, device=dev) + gid0
    return torch.stack([gid, torch.tensor(rates, dtype=torch.int64, device=dev),
                        executed_len.view(N, n).to(torch.int64).sum(1),
                        st[:, _lib.FX_SIM_STAT_FAST:_lib.FX_SIM_STAT_FAST + n].sum(1),
                        st[:, _lib.FX_SIM_STAT_SLOW:_lib.FX_SIM_STAT_SLOW + n].sum(1),
                        err.to(torch.int64)], 1)


def allreduce_hists(dist, world, hists):
    """The step's output: histograms summed over every rank's instances
    (exact integers, so identical for any number of ranks; RCCL on GPUs)."""
    if world > 1:
        for h in hists:
            dist.all_reduce(h)


def gather_rows(dist, world, rows):
    """One all_gather of the equal-sized per-rank row blocks -> global order."""
    import torch
    if world <= 1:
        return rows
    parts = [torch.empty_like(rows) for _ in range(world)]
    dist.all_gather(parts, rows.contiguous())
    return torch.cat(parts)


def main_sim(args):
    import torch
    import torch.distributed as dist

    from bench import host_cpus, measured_copy_gbps
    from fantoch_amd import _lib
    from fantoch_amd import metrics as fm
    from fantoch_amd import sim as S

    dense = args.mode == "dense-sim"
    if dense:  # BASELINE configs[3]
        args.clients_per_region = 64 if args.clients_per_region is None else args.clients_per_region
        # (seeds, conflicts, protocol: bench.MODE_DEFAULTS["dense-sim"])
        if args.cmds is None:
            args.cmds = 50
    if args.clients_per_region is None:
        args.clients_per_region = 1
    if args.cmds is None:
        args.cmds = 1000  # 1 client per region, 1k commands
    if args.cpu_baseline_seconds is None:
        args.cpu_baseline_seconds = 15.0
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == args.gpus
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    lib = _lib.load()
    if lib.fx_device_count() <= 0:
        raise SystemExit("no GPU visible to libfantoch_amd")

    planet = S.Planet()
    specs, rates, conflicts = local_specs(S, args, rank, planet)
    N = len(specs)
    n = args.n
    C = n * args.clients_per_region  # clients in the process regions
    exec_cap = C * args.cmds + 8
    LAT_BINS, CHAIN_BINS, DELAY_BINS = 8192, 256, 8192
    host = (_lib.SimSpec * N)(*specs)
    stream = torch.cuda.current_stream(dev)
    hs = ctypes.c_void_p(stream.cuda_stream)

    spec_dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(dev)
    ping = torch.from_numpy(planet.ping.astype(np.int16).view(np.int16)).to(dev)
    rank_m = torch.from_numpy(planet.rank).to(dev)
    executed = torch.empty(N * n * exec_cap, dtype=torch.int32, device=dev)
    executed_len = torch.zeros(N * n, dtype=torch.int32, device=dev)
    lat_hist = torch.zeros(planet.R * LAT_BINS, dtype=torch.int64, device=dev)
    chain = torch.zeros(CHAIN_BINS, dtype=torch.int64, device=dev)
    delay = torch.zeros(DELAY_BINS, dtype=torch.int64, device=dev)
    stats = torch.zeros(N * _lib.FX_SIM_STATS, dtype=torch.int64, device=dev)
    err = torch.zeros(N, dtype=torch.int32, device=dev)
    sim_flags = _lib.FX_SIM_FLAG_GENERIC if getattr(args, "generic", False) else 0
    batch = _lib.SimBatch(spec_dev.data_ptr(), ctypes.addressof(host), N, sim_flags, ping.data_ptr(),
                          rank_m.data_ptr(), planet.R, S.Planet.STRIDE, exec_cap, 0, 0,
                          args.ring_entries, args.dot_slots, 0)
    out = _lib.SimOutput(executed.data_ptr(), executed_len.data_ptr(), None, lat_hist.data_ptr(),
                         chain.data_ptr(), delay.data_ptr(), stats.data_ptr(), err.data_ptr(),
                         LAT_BINS, CHAIN_BINS, DELAY_BINS, 0, None)
    plan = ctypes.c_uint32()
    large = lib.fx_sim_plan(ctypes.byref(specs[0]), args.ring_entries, args.dot_slots, ctypes.byref(plan)) != 0 \
        or args.clients_per_region * n > 32
    arena = ctypes.c_uint64()
    if large:
        _lib.check(lib.fx_sim_plan_large(ctypes.byref(specs[0]), args.ring_entries, args.dot_slots,
                                         ctypes.byref(arena)), "fx_sim_plan_large")
    kernel_name = "k_simx" if large else "k_sim"

    def step():
        lat_hist.zero_()
        chain.zero_()
        delay.zero_()
        _lib.check(lib.fx_sim_run_tiered(ctypes.byref(batch), ctypes.byref(out), hs, None), "fx_sim_run_tiered")

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize(dev)
    bad = int((err != 0).sum().item())
    if bad:
        raise SystemExit("%d simulated instances failed: %s" % (bad, torch.unique(err).tolist()))

    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kernel_ms = []
    reruns = ctypes.c_uint32()  # instances rerun at larger tables (FX_ERR_SIM_CAPACITY) in the last step
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        lat_hist.zero_()
        chain.zero_()
        delay.zero_()
        ev0.record(stream)
        _lib.check(lib.fx_sim_run_tiered(ctypes.byref(batch), ctypes.byref(out), hs, ctypes.byref(reruns)),
                   "fx_sim_run_tiered")
        ev1.record(stream)
        allreduce_hists(dist, world, (lat_hist, chain, delay))
        ev1.synchronize()
        kernel_ms.append(ev0.elapsed_time(ev1))
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    st = stats.view(N, _lib.FX_SIM_STATS)
    executed_local = int(executed_len.to(torch.int64).sum().item())
    events_local = int(st[:, _lib.FX_SIM_STAT_EVENTS].sum().item())
    deps_local = int(st[:, _lib.FX_SIM_STAT_DEPS].sum().item())
    client_cmds_local = N * C * args.cmds
    tot = torch.tensor([elapsed, executed_local, events_local, deps_local, client_cmds_local],
                       dtype=torch.float64, device=dev)
    if world > 1:
        mx = tot[:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tot[1:].clone()
        dist.all_reduce(sm)
        elapsed = float(mx.item())
        executed_all, events_all, deps_all, client_all = [float(x) for x in sm.tolist()]
    else:
        executed_all, events_all, deps_all, client_all = (float(executed_local), float(events_local),
                                                          float(deps_local), float(client_cmds_local))

    # per-instance rows (global id, conflict %, executed, fast, slow, status), one all_gather
    rows = gather_rows(dist, world, instance_rows(torch, rank * N, rates, executed_len, stats, err, n))
    summary = {"fields": ROW_FIELDS,
               "instances": int(rows.shape[0]), "all_ok": bool((rows[:, 5] == 0).all().item()),
               "executed_matches": int(rows[:, 2].sum().item()) == int(executed_all)}
    fast_all, slow_all = int(rows[:, 3].sum().item()), int(rows[:, 4].sum().item())

    value = executed_all * args.steps / elapsed
    result = None
    if rank == 0:
        kavg = sum(kernel_ms) / len(kernel_ms)
        dbar = deps_all / executed_all if executed_all else 0.0
        # 32 + 4k + 8d bytes per executed command (k = 1)
        alg_bytes = (36.0 + 8.0 * dbar) * executed_local
        achieved = alg_bytes / (kavg * 1e-3) / 1e9
        traffic = None
        issue = None
        tj_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "sim_traffic_latest.json")
        if os.path.exists(tj_path):
            try:
                tj = json.load(open(tj_path))
                if tj.get("workload_key") == sim_key(args):
                    traffic = tj.get("hbm_bytes_per_launch")
                    issue = tj.get("issue")
            except Exception:
                traffic = None
        copy = measured_copy_gbps(torch, dev)
        roof = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 6), "traffic": traffic, "kernel": kernel_name,
                "kernel_ms_avg": round(kavg, 3), "alg_bytes_per_launch": int(alg_bytes),
                "alg_bytes_per_cmd": round(36.0 + 8.0 * dbar, 3),
                "alg_bytes_definition": "SURVEY.md 8(d): 32 + 4k + 8d per executed command, k = 1, "
                                        "d = mean deps of the executor Adds",
                "measured_copy_gbps": copy,
                "note": "the simulator has no HBM-bound phase: it is bound by instruction issue (the "
                        "scalar unit), see 'issue'"}
        if issue:
            # the bound that holds: SALU instructions per CU cycle against the
            # scalar unit's one per cycle (PMC passes of the same workload)
            roof["issue"] = dict(issue, bound="salu-issue", frac=issue.get("salu_per_cu_cycle"),
                                 source="profiles/sim_traffic_latest.json (rocprofv3 --pmc SQ_INSTS_*, GRBM_GUI_ACTIVE)")
        # the per-mode counter record of this exact workload (tools/mode_pmc.sh), when there is one
        import bench_pmc
        pm = bench_pmc.load(args.mode, args)
        if pm:
            bench_pmc.attach(roof, pm, alg_bytes)
            if dense:
                roof["note"] = ("k_simx walks its per-instance HBM arena with dependent round trips: "
                                "latency-bound, see issue.wait_any_frac_of_wave_cycles")
            elif roof.get("issue"):
                roof["issue"].update(bound="salu-issue", frac=roof["issue"].get("salu_per_cu_cycle"))
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            def run_subset(idx):
                return _subset_hists(torch, lib, _lib, [specs[i] for i in idx], planet, ping, rank_m, dev, hs,
                                     sim_flags, exec_cap, args, (LAT_BINS, CHAIN_BINS, DELAY_BINS), n)
            timed = (lat_hist.view(planet.R, LAT_BINS).cpu().numpy(), chain.cpu().numpy(), delay.cpu().numpy())
            cpu = cpu_baseline_sim(args, specs, rates, executed, executed_len, st, timed, n, exec_cap,
                                   planet, run_subset)
        lat = lat_hist.view(planet.R, LAT_BINS).cpu().numpy()
        regions = S.GCP5[:n]
        hist_stats = {"client_latency_ms": {r: fm.dense_stats(lat[planet.index[r]]) for r in regions},
                      "chain_size": fm.dense_stats(chain.cpu().numpy()),
                      "execution_delay_ms": fm.dense_stats(delay.cpu().numpy())}
        result = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "cmds/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: seeded closed-loop clients (canonical C6 RNG), GCP latency matrix",
            "config": {
                "workload": ("%s n=%d, %d seeds x conflict {%s}%% per GPU, %d clients/region, "
                             "%d cmds/client, GCP regions %s (BASELINE configs[%d])"
                             % ("Atlas f=1 + EPaxos f=%d (alternating)" % (n // 2) if args.protocol == "both"
                                else "%s f=%d" % (args.protocol.capitalize(), args.f),
                                n, args.seeds, args.conflicts, args.clients_per_region, args.cmds,
                                ",".join(S.GCP5[:n]), 3 if dense else 1)),
                "instances_per_gpu": N, "client_cmds_per_gpu": client_cmds_local,
                "parallelism": "instances sharded over %d GPU(s) (weak), one wavefront per "
                               "simulated instance" % world,
                "kernel": kernel_name,
                "arena_bytes_per_instance": int(arena.value) if large else 0,
                "effective_args": {k: getattr(args, k) for k in ("seeds", "conflicts", "protocol", "f", "cmds",
                                                                  "clients_per_region", "seed")},
            },
            "executed_per_step": int(executed_all),
            "client_cmds_per_s": round(client_all * args.steps / elapsed, 1),
            "sim_events_per_s": round(events_all * args.steps / elapsed, 1),
            "reruns_at_larger_tables_rank0": int(reruns.value),
            # graph edges = deps of every executor Add, per second
            "edges_per_s": round(deps_all * args.steps / elapsed, 1),
            "fast_paths": fast_all, "slow_paths": slow_all,
            "roofline": roof,
            "cpu_baseline": cpu,
            "instance_summary": summary,
            "histograms": hist_stats,
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


def sim_key(args):
    return "sim_%s_n%d_f%d_s%d_c%s_m%d_seed%d%s" % (
        args.protocol, args.n, args.f, args.seeds, args.conflicts.replace(",", "-"), args.cmds, args.seed,
        "" if (args.clients_per_region or 1) == 1 else "_k%d" % args.clients_per_region)


def _subset_hists(torch, lib, _lib, sub, planet, ping, rank_m, dev, hs, sim_flags, exec_cap, args, bins, n):
    """Histograms (client latency [R, bins], ChainSize, ExecutionDelay) of a
    GPU run over a subset of the bench's instances (same specs, so the same
    C6 RNG streams): the kernel is deterministic per instance, so the sample's
    run and the rest's run add up to the timed batch's histograms exactly."""
    import ctypes as ct
    LAT_BINS, CHAIN_BINS, DELAY_BINS = bins
    N = len(sub)
    if N == 0:
        return (np.zeros((planet.R, LAT_BINS), np.int64), np.zeros(CHAIN_BINS, np.int64),
                np.zeros(DELAY_BINS, np.int64))
    host = (_lib.SimSpec * N)(*sub)
    spec_dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(dev)
    executed = torch.empty(N * n * exec_cap, dtype=torch.int32, device=dev)
    executed_len = torch.zeros(N * n, dtype=torch.int32, device=dev)
    lat = torch.zeros(planet.R * LAT_BINS, dtype=torch.int64, device=dev)
    chain = torch.zeros(CHAIN_BINS, dtype=torch.int64, device=dev)
    delay = torch.zeros(DELAY_BINS, dtype=torch.int64, device=dev)
    stats = torch.zeros(N * _lib.FX_SIM_STATS, dtype=torch.int64, device=dev)
    err = torch.zeros(N, dtype=torch.int32, device=dev)
    batch = _lib.SimBatch(spec_dev.data_ptr(), ct.addressof(host), N, sim_flags, ping.data_ptr(),
                          rank_m.data_ptr(), planet.R, planet.STRIDE, exec_cap, 0, 0,
                          args.ring_entries, args.dot_slots, 0)
    out = _lib.SimOutput(executed.data_ptr(), executed_len.data_ptr(), None, lat.data_ptr(),
                         chain.data_ptr(), delay.data_ptr(), stats.data_ptr(), err.data_ptr(),
                         LAT_BINS, CHAIN_BINS, DELAY_BINS, 0, None)
    _lib.check(lib.fx_sim_run_tiered(ct.byref(batch), ct.byref(out), hs, None), "fx_sim_run_tiered (subset)")
    torch.cuda.synchronize(dev)
    if int((err != 0).sum().item()):
        raise SystemExit("subset rerun: simulated instances failed")
    return (lat.view(planet.R, LAT_BINS).cpu().numpy(), chain.cpu().numpy(), delay.cpu().numpy())


def hist_parity(timed, gpu_sample, gpu_rest, oracle_res):
    """(ok, detail) of the histogram check on the bench's sample:
    the GPU's sample histograms (client latency per region, ChainSize,
    ExecutionDelay) equal the oracle's summed over the sample, and the timed
    batch's histograms equal the sample's plus the rest's, bin for bin
    (runner.rs:619-634 clients_latencies, histogram.rs:55-59 increment;
    graph/mod.rs:492-518 ChainSize / ExecutionDelay)."""
    names = ("client_latency", "chain_size", "execution_delay")
    keys = ("latency", "chain", "delay")
    detail = {}
    ok = True
    for nm, k, t, s, r in zip(names, keys, timed, gpu_sample, gpu_rest):
        o = np.zeros(s.shape, np.int64)
        for res in oracle_res:
            a = res[k].astype(np.int64)
            o[tuple(slice(0, m) for m in a.shape)] += a[tuple(slice(0, m) for m in o.shape)]
        same_oracle = bool(np.array_equal(s, o))
        adds_up = bool(np.array_equal(t, s + r))
        detail[nm] = {"sample_equals_oracle": same_oracle, "timed_equals_sample_plus_rest": adds_up,
                      "sample_samples": int(o.sum())}
        ok = ok and same_oracle and adds_up
    return ok, detail


def cpu_baseline_sim(args, specs, rates, executed, executed_len, st, timed_hists, n, exec_cap, planet,
                     run_subset=None):
    """The simulator oracle (oracle/sim_oracle.cpp, the C++ restatement of the
    reference simulator) on a bounded sample of the same instances, one
    instance per std::thread task like the reference binary's rayon par_iter,
    on every usable host core; the GPU's outputs for the sample are checked
    against it bit for bit: execution orders, fast / slow / stable counters,
    action trace and end time per instance, and the three histograms
    (client latency per region, ChainSize, ExecutionDelay) through
    `hist_parity` — the timed batch's histograms = the sample's GPU rerun + the
    rest's GPU rerun, and the sample's = the oracle's sum over the sample."""
    import torch
    from bench import host_cpus
    from oracle import oracle_lib as O
    from fantoch_amd import _lib

    host = host_cpus()
    threads = host["usable"]
    to_o = lambda s: _to_oracle(_lib, O, s)
    # calibrate: one instance of every rate, single-threaded
    t0 = time.perf_counter()
    firsts = {}
    for i, r in enumerate(rates):
        firsts.setdefault(r, i)
    O.sim_batch([to_o(specs[i]) for i in firsts.values()], threads=1)
    per_inst = (time.perf_counter() - t0) / len(firsts)
    budget = max(len(firsts), int(args.cpu_baseline_seconds * threads / max(per_inst, 1e-4)))
    k = min(len(specs), budget)
    pick = np.unique(np.linspace(0, len(specs) - 1, k).round().astype(np.int64))
    t0 = time.perf_counter()
    res = O.sim_batch([to_o(specs[i]) for i in pick], threads=threads)
    dt = time.perf_counter() - t0
    executed_cpu = sum(int(sum(len(e) for e in r["executed"])) for r in res)
    # parity on the sample
    el = executed_len.view(len(specs), n).cpu().numpy()
    stc = st.cpu().numpy().view(np.uint64)
    ok = True
    for j, i in enumerate(pick):
        r = res[j]
        ex = executed[i * n * exec_cap:(i + 1) * n * exec_cap].view(n, exec_cap).cpu().numpy().view(np.uint32)
        for p in range(n):
            if not np.array_equal(ex[p, :el[i, p]], r["executed"][p]):
                ok = False
        if [int(x) for x in stc[i, 0:n]] != [int(x) for x in r["fast"]] or \
           [int(x) for x in stc[i, 8:8 + n]] != [int(x) for x in r["slow"]] or \
           [int(x) for x in stc[i, 16:16 + n]] != [int(x) for x in r["stable"]] or \
           int(stc[i, 26]) != r["trace"] or int(stc[i, 25]) != r["end_ms"]:
            ok = False
        if not ok:
            break
    orders_ok = ok
    hist_detail = None
    if run_subset is not None:
        rest = np.setdiff1d(np.arange(len(specs)), pick)
        hok, hist_detail = hist_parity(timed_hists, run_subset(pick), run_subset(rest), res)
        ok = ok and hok
    else:
        ok = False  # histograms unchecked: no parity claim
    return {"value": round(executed_cpu / dt, 1), "unit": "cmds/s", "cores": threads, "kind": "port",
            "host": host,
            "sample": "%d of %d instances spread over every conflict rate, simulated end to end by the "
                      "C++ simulator oracle in %.2f s on %d threads (%d executed commands); GPU output "
                      "on the sample %s the oracle bit-for-bit (execution orders, fast/slow/stable "
                      "counters, action trace, end time, and the client-latency / ChainSize / "
                      "ExecutionDelay histograms: the sample's GPU histograms equal the oracle's, and the "
                      "timed batch's equal the sample's plus the other instances' GPU rerun)"
                      % (len(pick), len(specs), dt, threads, executed_cpu,
                         "matches" if ok else "DIFFERS FROM"),
            "sample_parity": ok, "sample_orders_counters_parity": orders_ok,
            "sample_histogram_parity": hist_detail}


def _to_oracle(_lib, O, s):
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
