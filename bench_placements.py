"""bench.py --mode placements: BASELINE configs[2] on the GPU simulator.

Atlas with n = 5 and n = 7, f = 1 and f = 2, over every 5- and 7-region subset
of the 20 GCP regions: C(20,5) x 2 + C(20,7) x 2 = 186,048 placements.  Each
placement is one instance of fantoch_ps/src/bin/simulation.rs's run
(Runner::new + Runner::run): processes in the subset's regions (name order,
canonical C12), one client per process region, `--cmds` commands per client,
`--placement-conflict` % conflicts, GC and executed notifications every 10 ms.

The placements are enumerated (n, f) group by group, subsets in
lexicographic order, and sharded by contiguous global range over the ranks
(rank r: [r P / N, (r + 1) P / N)); a rank launches one fx_sim_run per
geometry (n).  Per-placement rows (id, n, f, executed, mean client latency,
fast/slow paths, status) travel in one all_gather after the timed region, and
rank 0 reports the best placement of every (n, f) by mean client latency.
`--placement-limit K` runs the first K placements of the enumeration (tests).

value = commands executed by all executors of all placements / max-over-ranks
time of the sweep."""
import ctypes
import itertools
import json
import os
import time

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)

import numpy as np

from bench_sim import METRIC, _to_oracle

GROUPS = [(5, 1), (5, 2), (7, 1), (7, 2)]


def enumerate_placements(R, limit=None):
    """[(n, f, subset)] in the global order (canonical C12: regions by name)."""
    out = []
    for n, f in GROUPS:
        for sub in itertools.combinations(range(R), n):
            out.append((n, f, sub))
            if limit is not None and len(out) >= limit:
                return out
    return out


def rank_range(P, rank, world):
    """Rank r's contiguous share [r P / N, (r + 1) P / N) of the placements."""
    return rank * P // world, (rank + 1) * P // world


ROW_FIELDS = ["placement", "n", "f", "executed", "latency_sum", "client_cmds", "fast_paths", "slow_paths",
              "status"]


def placement_rows(torch, ids, allp, n, cmds, executed_len, stats, err):
    """[len(ids), 9] int64 rows (ROW_FIELDS) of one launch (geometry n)."""
    from fantoch_amd import _lib
    N = len(ids)
    dev = executed_len.device
    st = stats.view(N, _lib.FX_SIM_STATS)
    t = torch.tensor(ids, dtype=torch.int64, device=dev)
    fs_ = torch.tensor([allp[g][1] for g in ids], dtype=torch.int64, device=dev)
    return torch.stack([t, torch.full_like(t, n), fs_, executed_len.view(N, n).to(torch.int64).sum(1),
                        st[:, _lib.FX_SIM_STAT_LAT_SUM], torch.full_like(t, n * cmds),
                        st[:, _lib.FX_SIM_STAT_FAST:_lib.FX_SIM_STAT_FAST + n].sum(1),
                        st[:, _lib.FX_SIM_STAT_SLOW:_lib.FX_SIM_STAT_SLOW + n].sum(1),
                        err.to(torch.int64)], 1)


def gather_rows(dist, world, rows):
    """all_gather of per-rank row blocks of different sizes (padded to the
    largest) -> every rank's rows, sorted by placement id."""
    import torch
    if world > 1:
        dev = rows.device
        cnt = torch.tensor([rows.shape[0]], dtype=torch.int64, device=dev)
        counts = [torch.zeros_like(cnt) for _ in range(world)]
        dist.all_gather(counts, cnt)
        mx = int(max(c.item() for c in counts))
        pad = torch.full((mx, rows.shape[1]), -1, dtype=torch.int64, device=dev)
        pad[:rows.shape[0]] = rows
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad)
        rows = torch.cat([p[:int(c.item())] for p, c in zip(parts, counts)])
    return rows[torch.argsort(rows[:, 0])] if rows.shape[0] else rows


def main_placements(args):
    import torch
    import torch.distributed as dist

    from bench import host_cpus
    from fantoch_amd import _lib
    from fantoch_amd import sim as S

    cmds = args.cmds if args.cmds is not None else 1000
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
    allp = enumerate_placements(planet.R, args.placement_limit)
    P = len(allp)
    lo, hi = rank_range(P, rank, world)
    mine = list(range(lo, hi))
    stream = torch.cuda.current_stream(dev)
    hs = ctypes.c_void_p(stream.cuda_stream)
    ping = torch.from_numpy(planet.ping.astype(np.int16).view(np.int16)).to(dev)
    rank_m = torch.from_numpy(planet.rank).to(dev)
    LAT_BINS, CHAIN_BINS, DELAY_BINS = 8192, 256, 8192
    lat_hist = torch.zeros(planet.R * LAT_BINS, dtype=torch.int64, device=dev)
    chain = torch.zeros(CHAIN_BINS, dtype=torch.int64, device=dev)
    delay = torch.zeros(DELAY_BINS, dtype=torch.int64, device=dev)

    # one launch per geometry (n); instances heaviest (n = 7) first
    launches = []
    for n in (7, 5):
        ids = [g for g in mine if allp[g][0] == n]
        if not ids:
            continue
        specs = [S.spec(S.ATLAS, n, allp[g][1], list(allp[g][2]), list(allp[g][2]), commands_per_client=cmds,
                        conflict_rate=args.placement_conflict, seed=args.seed, instance=g) for g in ids]
        N = len(specs)
        host = (_lib.SimSpec * N)(*specs)
        spec_dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(dev)
        executed_len = torch.zeros(N * n, dtype=torch.int32, device=dev)
        stats = torch.zeros(N * _lib.FX_SIM_STATS, dtype=torch.int64, device=dev)
        err = torch.zeros(N, dtype=torch.int32, device=dev)
        sim_flags = _lib.FX_SIM_FLAG_GENERIC if getattr(args, "generic", False) else 0
        batch = _lib.SimBatch(spec_dev.data_ptr(), ctypes.addressof(host), N, sim_flags, ping.data_ptr(),
                              rank_m.data_ptr(),
                              planet.R, S.Planet.STRIDE, 0, 0, 0, args.ring_entries, args.dot_slots, 0)
        out = _lib.SimOutput(None, executed_len.data_ptr(), None, lat_hist.data_ptr(), chain.data_ptr(),
                             delay.data_ptr(), stats.data_ptr(), err.data_ptr(), LAT_BINS, CHAIN_BINS, DELAY_BINS, 0)
        launches.append(dict(n=n, ids=ids, specs=specs, host=host, spec_dev=spec_dev, executed_len=executed_len,
                             stats=stats, err=err, batch=batch, out=out))

    reruns = ctypes.c_uint32()

    def sweep():
        lat_hist.zero_()
        chain.zero_()
        delay.zero_()
        for L in launches:
            _lib.check(lib.fx_sim_run_tiered(ctypes.byref(L["batch"]), ctypes.byref(L["out"]), hs, reruns),
                       "fx_sim_run_tiered")
            L["reruns"] = int(reruns.value)

    for _ in range(args.warmup):
        sweep()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # each launch (one geometry: n = 7, then n = 5) timed by HIP events on the
    # stream it runs on (fx_sim_run_tiered: the kernel, plus any capacity reruns)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in launches]
    launch_ms = [[] for _ in launches]
    t0 = time.perf_counter()
    for _ in range(args.steps):
        lat_hist.zero_()
        chain.zero_()
        delay.zero_()
        for i, L in enumerate(launches):
            evs[i][0].record(stream)
            _lib.check(lib.fx_sim_run_tiered(ctypes.byref(L["batch"]), ctypes.byref(L["out"]), hs, reruns),
                       "fx_sim_run_tiered")
            evs[i][1].record(stream)
            L["reruns"] = int(reruns.value)
        for i in range(len(launches)):
            evs[i][1].synchronize()
            launch_ms[i].append(evs[i][0].elapsed_time(evs[i][1]))
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    # per-placement rows: id, n, f, executed, latency sum, client commands, fast, slow, status
    rows = [placement_rows(torch, L["ids"], allp, L["n"], cmds, L["executed_len"], L["stats"], L["err"])
            for L in launches]
    rows = torch.cat(rows) if rows else torch.zeros((0, len(ROW_FIELDS)), dtype=torch.int64, device=dev)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        for h in (lat_hist, chain, delay):
            dist.all_reduce(h)
    rows = gather_rows(dist, world, rows)
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return None
    R = rows.cpu().numpy()
    executed_all = int(R[:, 3].sum())
    value = executed_all * args.steps / elapsed
    best = {}
    for n, f in GROUPS:
        sel = R[(R[:, 1] == n) & (R[:, 2] == f) & (R[:, 8] == 0)]
        if len(sel):
            mean = sel[:, 4] / sel[:, 5]
            j = int(np.argmin(mean))
            best["n%d_f%d" % (n, f)] = {"placement": [planet.regions[r] for r in allp[int(sel[j, 0])][2]],
                                        "mean_latency_ms": round(float(mean[j]), 3),
                                        "placements": int(len(sel))}
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = _cpu_baseline(args, launches, cmds)
    # roofline of rank 0's launches: SURVEY.md 8(d) bytes (32 + 4k + 8 d per
    # executed command, d = mean deps of the executor Adds, from the kernel's
    # per-instance counters) over the launches' own time (HIP events)
    import bench_pmc
    per = []
    alg_total, ms_total = 0.0, 0.0
    for i, L in enumerate(launches):
        st = L["stats"].view(len(L["ids"]), _lib.FX_SIM_STATS)
        ex = int(L["executed_len"].to(torch.int64).sum().item())
        dsum = int(st[:, _lib.FX_SIM_STAT_DEPS].sum().item())
        alg = 36.0 * ex + 8.0 * dsum
        ms = sum(launch_ms[i]) / len(launch_ms[i])
        per.append({"n": L["n"], "instances": len(L["ids"]), "kernel_ms_avg": round(ms, 3),
                    "executed": ex, "alg_bytes": int(alg)})
        alg_total += alg
        ms_total += ms
    roof = None
    if per:
        ach = alg_total / (ms_total * 1e-3) / 1e9
        dom = max(per, key=lambda x: x["kernel_ms_avg"])
        roof = {"bound": "hbm", "achieved": round(ach, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBPS, 6), "kernel": "k_sim (n = %d launch dominant)" % dom["n"],
                "kernel_ms_avg": round(ms_total, 3), "per_launch": per, "alg_bytes_per_launch": int(alg_total),
                "alg_bytes_definition": "SURVEY.md 8(d): 32 + 4k + 8d per executed command, k = 1",
                "note": "the simulator is bound by scalar issue, not bytes (see issue)"}
        bench_pmc.attach(roof, bench_pmc.load("placements", args), alg_total)
        if roof.get("issue"):
            roof["issue"].update(bound="salu-issue", frac=roof["issue"].get("salu_per_cu_cycle"))
    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "cmds/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic: seeded closed-loop clients (canonical C6 RNG), GCP latency matrix",
        "config": {"workload": "Atlas n=5/7 f=1/2 over every 5-/7-region subset of the %d GCP regions, 1 "
                               "client/region, %d cmds/client, %d%% conflicts (BASELINE configs[2])"
                               % (planet.R, cmds, args.placement_conflict),
                   "placements": P, "parallelism": "placements sharded by contiguous range over %d GPU(s)"
                                                   % world},
        "executed_per_step": executed_all,
        "all_ok": bool((R[:, 8] == 0).all()),
        "failed_placements": int((R[:, 8] != 0).sum()),
        "reruns_at_larger_tables_rank0": int(sum(L.get("reruns", 0) for L in launches)),
        "best_placement_by_mean_latency": best,
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return line


def _cpu_baseline(args, launches, cmds):
    """The simulator oracle on a bounded, evenly spread sample of the
    placements (every usable host core), checked against the GPU bit for bit
    on executed counts, counters and latency sums."""
    from bench import host_cpus
    from fantoch_amd import _lib
    from oracle import oracle_lib as O

    host = host_cpus()
    threads = host["usable"]
    picks = []
    # ~cpu_baseline_seconds (default 10) of oracle work at ~0.15 M executed
    # commands per second per thread, split over the launches
    budget = (args.cpu_baseline_seconds or 10) * 0.15e6 * threads / max(1, len(launches))
    for L in launches:
        N, n = len(L["ids"]), L["n"]
        k = max(1, min(N, int(budget / (n * n * cmds))))
        for i in np.unique(np.linspace(0, N - 1, k).round().astype(np.int64)):
            picks.append((L, int(i)))
    t0 = time.perf_counter()
    res = O.sim_batch([_to_oracle(_lib, O, L["specs"][i]) for L, i in picks], threads=threads)
    dt = time.perf_counter() - t0
    executed_cpu = sum(int(sum(len(e) for e in r["executed"])) for r in res)
    ok = True
    for (L, i), r in zip(picks, res):
        n = L["n"]
        st = L["stats"].view(len(L["ids"]), _lib.FX_SIM_STATS)[i].cpu().numpy().view(np.uint64)
        el = L["executed_len"].view(len(L["ids"]), n)[i].cpu().numpy()
        lat_sum = int(sum(int(ms) * int(c) for h in r["latency"] for ms, c in enumerate(h)))
        if [int(x) for x in el] != [len(e) for e in r["executed"]] or \
           [int(x) for x in st[0:n]] != [int(x) for x in r["fast"]] or \
           [int(x) for x in st[16:16 + n]] != [int(x) for x in r["stable"]] or \
           int(st[_lib.FX_SIM_STAT_LAT_SUM]) != lat_sum or int(st[26]) != r["trace"]:
            ok = False
            break
    return {"value": round(executed_cpu / dt, 1), "unit": "cmds/s", "cores": threads, "kind": "port",
            "host": host,
            "sample": "%d placements spread over the sweep, simulated by the C++ simulator oracle in %.2f s on "
                      "%d threads; GPU output on the sample %s (executed counts, fast/stable counters, latency "
                      "sums, action trace)" % (len(picks), dt, threads, "identical" if ok else "DIFFERS"),
            "sample_parity": ok}
