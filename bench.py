#!/usr/bin/env python3
"""bench.py — executed commands/s of batched Atlas/EPaxos simulations (BASELINE.json).

--mode sim (default, bench_sim.py): BASELINE configs[1], the batched simulator
itself — EPaxos n=5 f=2 on the GCP planet, 4096 seeds x conflict {0,2,10,50,100}%
per GPU, every instance simulated end to end on the GPU (fx_sim_run).

--mode executor: the GraphExecutor alone over synthetic commit streams.
Workload (per GPU; weak scaling): EPaxos n=5, 4096 seeds x conflict rates
{0,2,10,50,100}% = 20,480 instances, 1 client per process x 1,000 commands
-> 5 commit streams of 5,000 Adds per instance (102,400 streams, 512M Adds).
Streams are seeded synthetic Atlas/EPaxos commit streams generated on the GPU
(fantoch_amd/csrc/fx_synth.h) before the timed region.

One step = one pass of the hot path over the resident batch:
  fx_batch_execute (GraphExecutor::handle over every Add of every stream)
  + fx_batch_metrics (ChainSize / ExecutionDelay histograms)
  + all-reduce of the histograms over ranks (RCCL) when N > 1.

Launch: python bench.py --gpus N --steps K --warmup W   (N > 1 via torch.distributed.run)
Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "executed cmds/sec (node) for batched Atlas/EPaxos sims; % of HBM roofline"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
KERNEL_NAMES = {0: "k_graph_group", 1: "k_graph_exec<Tier1>", 2: "k_graph_exec<Tier2>",
                3: "k_graph_exec<TierLane>", 4: "k_graph_wave", 5: "k_graph_lane",
                6: "k_graph_group||k_graph_lane"}
LAYOUT = {0: "16 lanes per stream", 1: "one lane per stream", 2: "one lane per stream",
          3: "one lane per stream", 4: "one wavefront per stream",
          5: "one lane per stream (register slot table, independent lane progress)",
          6: "per 64-stream tile: 16 lanes per stream for dense tiles, one lane per stream "
             "for sparse ones, both kernels concurrent"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["sim", "dense-sim", "executor", "huge", "dense", "placements", "pred",
                                       "handle"],
                    default="sim",
                    help="sim: the batched simulator (BASELINE configs[1], the headline); "
                         "dense-sim: the simulator on BASELINE configs[3] (64 clients/region, 100%% "
                         "conflicts); executor: the GraphExecutor alone over synthetic commit streams")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    # --seeds / --conflicts / --protocol / --f: None = the mode's default
    # (MODE_DEFAULTS); an explicit value is always honoured
    ap.add_argument("--seeds", type=int, default=None)
    ap.add_argument("--conflicts", type=str, default=None)
    ap.add_argument("--n", type=int, default=5)
    ap.add_argument("--cmds", type=int, default=None,
                    help="commands per client (sim default 1000, SURVEY.md §8(a) C2; "
                         "executor default 1000)")
    ap.add_argument("--protocol", choices=["epaxos", "atlas", "both"], default=None)
    ap.add_argument("--clients-per-region", type=int, default=None,
                    help="sim: clients per region (default 1; dense-sim 64)")
    ap.add_argument("--f", type=int, default=None)
    ap.add_argument("--window", type=int, default=8)
    ap.add_argument("--cycle-pct", type=int, default=30)
    ap.add_argument("--huge-shape", choices=["s5", "conflict2", "conflict100"], default="s5",
                    help="--mode huge: SURVEY §8(d)'s S5 stream (per-key chains over --key-pool keys plus "
                         "cycles), or the conflict-key streams at 2 %% / 100 %% conflicts")
    ap.add_argument("--key-pool", type=int, default=1000, help="--mode huge s5: keys in the pool")
    ap.add_argument("--horizon", type=int, default=None,
                    help="--mode huge: rounds searched back for a command's deps (s5 default 640: mean deps ~ 3)")
    ap.add_argument("--seed", type=int, default=20250213)
    ap.add_argument("--conflict-block", type=int, default=-1,
                    help="instances per conflict rate block (-1 = --seeds: conflict-major "
                         "enumeration, so a wavefront's streams share a rate; 0 = seed-major)")
    ap.add_argument("--tier", type=int, default=-1, help="executor tier (-1 = FX_TIER_DEFAULT)")
    ap.add_argument("--ring-entries", type=int, default=0,
                    help="sim: messages in flight per instance (pool shared by the links; 0 = 16 n x clients per region)")
    ap.add_argument("--dot-slots", type=int, default=0,
                    help="sim: live dots per instance (pool shared by the coordinators; 0 = min(64, 8 clients))")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=None,
                    help="CPU work budget of the cpu_baseline sample (sim default 15, executor 5)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--generic", action="store_true",
                    help="simulator: the run-time-geometry kernel build even for a compiled-in geometry (A/B)")
    ap.add_argument("--placement-conflict", type=int, default=2,
                    help="placements mode (BASELINE configs[2]): conflict rate of every placement")
    ap.add_argument("--placement-limit", type=int, default=None,
                    help="placements mode: run only the first K placements of the enumeration")
    args = ap.parse_args(argv)
    for k, v in MODE_DEFAULTS.get(args.mode, MODE_DEFAULTS["sim"]).items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    import bench_pmc
    args.pmc_key = bench_pmc.workload_key(args)  # before a mode fills in its own defaults
    return args


# per-mode defaults of the workload arguments (filled in only when the command
# line leaves them unset, and reported in the bench line's config)
MODE_DEFAULTS = {
    "sim": dict(seeds=4096, conflicts="0,2,10,50,100", protocol="epaxos", f=2),
    # BASELINE configs[3] on the simulator: one resident wavefront per
    # instance; k_simx's configs[3] build runs 5 waves per SIMD, two
    # instances per workgroup: 20 per CU x 256 CUs = 5,120, one round (3 waves
    # per SIMD and 3,072 instances: 117 M; 4 and 4,096: 139 M; 5 and 5,120:
    # 144 M, profiles/archive/calls/r5_occ2.sh, profiles/archive/calls/r5_x5.sh)
    "dense-sim": dict(seeds=5120, conflicts="100", protocol="both", f=2),
    # configs[3] on the batched executor: 3,072 instances = 15,360 streams,
    # one wavefront each, 5 per CU (LDS tables): 12 rounds, so the last
    # round's tail weighs less than at 768 instances (68.3 M; 1,536: 73.2 M;
    # 3,072: 77.2 M; 6,144: 79.5 M, tools/dense_scale.sh)
    "dense": dict(seeds=3072, conflicts="100", protocol="epaxos", f=2),
}


def measured_copy_gbps(torch, dev, nbytes=2 << 30, reps=10):
    """Achievable HBM bandwidth on this box: a device-to-device copy of nbytes,
    counted as read + write (SURVEY.md §8(d) asks for it next to the 8 TB/s peak)."""
    a = torch.empty(nbytes // 4, dtype=torch.int32, device=dev)
    b = torch.empty_like(a)
    a.fill_(1)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize(dev)
    gbps = 2.0 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    return round(gbps, 1)


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) without a torch.distributed launcher: start
    N fresh ranks through torch.distributed.run as a child process BEFORE this
    process touches the GPU, and exit with its status."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args))
    if args.mode in ("sim", "dense-sim"):
        from bench_sim import main_sim
        return main_sim(args)
    if args.mode == "huge":
        from bench_huge import main_huge
        return main_huge(args)
    if args.mode == "dense":
        from bench_huge import main_dense
        return main_dense(args)
    if args.mode == "handle":
        from bench_handle import main_handle
        return main_handle(args)
    if args.mode == "pred":
        from bench_pred import main_pred
        return main_pred(args)
    if args.mode == "placements":
        from bench_placements import main_placements
        return main_placements(args)
    if args.cmds is None:
        args.cmds = 1000
    if args.cpu_baseline_seconds is None:
        args.cpu_baseline_seconds = 5.0
    import numpy as np
    import torch
    import torch.distributed as dist

    from fantoch_amd import _lib
    from fantoch_amd import sharding
    from fantoch_amd import streams as fs

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

    conflicts = [int(c) for c in args.conflicts.split(",")]
    instances = args.seeds * len(conflicts)
    cblock = args.seeds if args.conflict_block < 0 else args.conflict_block
    p = sharding.rank_params(rank, args.seeds, conflicts, args.n, args.cmds, args.window,
                             args.cycle_pct, args.seed, args.conflict_block)
    S, steps, dmax = fs.synth_shape(p)
    pw = _lib.plane_words(S, steps)
    stream = torch.cuda.current_stream(dev)
    hs = ctypes.c_void_p(stream.cuda_stream)

    def buf(words):
        return torch.empty(words, dtype=torch.int32, device=dev)

    dot, hdr, deps = buf(pw), buf(pw), buf(pw * dmax)
    order, release = buf(pw), buf(pw)
    nexec, err = buf(S), buf(S)
    NBC, NBD = 64, 4096
    chain = torch.zeros(NBC, dtype=torch.int64, device=dev)
    delay = torch.zeros(NBD, dtype=torch.int64, device=dev)

    t0 = time.time()
    _lib.check(lib.fx_synth_generate(ctypes.byref(p), dot.data_ptr(), hdr.data_ptr(),
                                     deps.data_ptr(), hs), "fx_synth_generate")
    torch.cuda.synchronize(dev)
    gen_s = time.time() - t0
    inb = _lib.StreamBatch(dot.data_ptr(), hdr.data_ptr(), deps.data_ptr(), None, S, steps, dmax,
                           args.n)
    outb = _lib.OrderBatch(order.data_ptr(), release.data_ptr(), nexec.data_ptr(), err.data_ptr())
    hb = _lib.HistBatch(chain.data_ptr(), NBC, delay.data_ptr(), NBD)

    # algorithmic bytes of one executor launch, SURVEY.md §8(d): a packed input
    # record of 20 + 4k + 8d bytes (header, seq, rifl, t, k key ids, d deps as
    # (source, seq) pairs) plus a 12-byte output (dot + release step) per
    # command = 32 + 4k + 8d, with k = 1 key per command and d read from the
    # stream.  The packed planes this build actually streams (dot + hdr + 4 B per
    # dep in, order + release out = 16 + 4d) are reported beside it.
    nd_total = int(((hdr >> 24) & 31).sum(dtype=torch.int64).item())
    n_adds = S * steps
    KEYS_PER_CMD = 1
    alg_bytes = (32 + 4 * KEYS_PER_CMD) * n_adds + 8 * nd_total
    plane_bytes = 16 * n_adds + 4 * nd_total

    tier = _lib.FX_TIER_DEFAULT if args.tier < 0 else args.tier
    tiered = [False]
    tier_counts = (ctypes.c_uint32 * _lib.FX_NUM_TIERS)()
    scratch = None
    if tier in (2, _lib.FX_TIER_SPLIT):  # working memory of the HBM tier / split scratch
        scratch = buf((lib.fx_batch_state_bytes(tier, args.n, S) + 3) // 4)

    def step():
        chain.zero_()
        delay.zero_()
        if tiered[0]:
            st = lib.fx_batch_run_tiered(ctypes.byref(inb), ctypes.byref(outb),
                                         _lib.first_tier_flag(tier), hs, tier_counts)
        else:
            st = lib.fx_batch_execute(ctypes.byref(inb), ctypes.byref(outb), tier, None, S,
                                      scratch.data_ptr() if scratch is not None else None, 0,
                                      steps, _lib.FX_FLAG_INIT, None, hs)
        _lib.check(st, "executor")
        _lib.check(lib.fx_batch_metrics(ctypes.byref(inb), ctypes.byref(outb), ctypes.byref(hb), hs),
                   "metrics")
        if world > 1:
            sharding.allreduce_histograms(dist, chain, delay)

    # warmup (+ decide whether any stream needs a tier rerun)
    for w in range(max(args.warmup, 1)):
        step()
        torch.cuda.synchronize(dev)
        if w == 0:
            bad = int((err != 0).sum().item())
            if bad:
                tiered[0] = True
                step()
                torch.cuda.synchronize(dev)
    if int((err != 0).sum().item()) != 0:
        raise SystemExit("streams failed: %s" % torch.unique(err).tolist())
    executed_local = int(nexec.sum(dtype=torch.int64).item())

    lib.fx_profile_enable(1)
    kernel_ms = []
    kern_ms = {1: [], 2: []}  # split tier: group kernel, lane kernel (own-stream events)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        if not tiered[0]:
            ms = ctypes.c_float()
            # events were recorded on `hs` around the executor kernel; reading
            # them after the step keeps the next launch queued behind this one
            if lib.fx_profile_last_exec_ms(ctypes.byref(ms)) == 0:
                kernel_ms.append(ms.value)
            for which in (1, 2):
                if lib.fx_profile_last_kernel_ms(which, ctypes.byref(ms)) == 0:
                    kern_ms[which].append(ms.value)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    lib.fx_profile_enable(0)

    stats = torch.tensor([elapsed, executed_local, nd_total, n_adds], dtype=torch.float64, device=dev)
    if world > 1:
        mx = stats[:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = stats[1:].clone()
        dist.all_reduce(sm)
        elapsed = float(mx.item())
        executed_total, nd_all, adds_all = [float(x) for x in sm.tolist()]
    else:
        executed_total, nd_all, adds_all = float(executed_local), float(nd_total), float(n_adds)

    # per-placement results: one all_gather of fixed-size per-instance rows after the
    # timed region, checked against the executed total
    rows = sharding.gather_summaries(dist, sharding.instance_summaries(nexec, err, p), world)
    summary = {"fields": list(sharding.SUMMARY_FIELDS), "instances": int(rows.shape[0]),
               "all_ok": bool((rows[:, 3] == 0).all().item()),
               "executed_matches": int(rows[:, 2].sum().item()) == int(executed_total)}

    value = executed_total * args.steps / elapsed
    edges = nd_all * args.steps / elapsed
    kavg = sum(kernel_ms) / len(kernel_ms) if kernel_ms else None

    result = None
    if rank == 0:
        roof = None
        if kavg:
            # dominant kernel: the longest-running kernel of the launch, timed by
            # HIP events on the stream it was launched on (the split tier runs
            # the group kernel on the caller's stream and the lane kernel on an
            # auxiliary one, concurrently); other tiers are one kernel
            kname, dom_ms = KERNEL_NAMES.get(tier, "tier%d" % tier), kavg
            per_kernel = {}
            for which, nm in ((1, "k_graph_group"), (2, "k_graph_lane")):
                if kern_ms[which]:
                    per_kernel[nm] = round(sum(kern_ms[which]) / len(kern_ms[which]), 4)
            if per_kernel:
                kname = max(per_kernel, key=per_kernel.get)
                dom_ms = per_kernel[kname]
            achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
            # the counters come from this exact workload's PMC record
            # (tools/mode_pmc.sh executor k_graph_lane -> profiles/pmc_executor.json)
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                    "traffic": None, "kernel": kname,
                    "kernel_ms_avg": round(dom_ms, 4), "per_kernel_ms_avg": per_kernel,
                    "launch_ms_avg": round(kavg, 4),
                    "alg_bytes_per_launch": alg_bytes,
                    "alg_bytes_per_cmd": round(alg_bytes / n_adds, 3),
                    "alg_bytes_definition": "SURVEY.md 8(d): 32 + 4k + 8d per command, k = 1",
                    "plane_bytes_per_launch": plane_bytes,
                    "plane_bytes_per_cmd": round(plane_bytes / n_adds, 3),
                    "plane_frac_of_launch": round(plane_bytes / (kavg * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}
            import bench_pmc
            pm = bench_pmc.load("executor", args)
            bench_pmc.attach(roof, pm, alg_bytes)
            if pm and pm.get("kernel_pattern") and pm["kernel_pattern"] not in kname:
                roof["traffic_note"] = ("counters of %s, the dominant kernel by rocprofv3 time; the HIP-event "
                                        "dominant kernel here is %s" % (pm["kernel_pattern"], kname))
            copy = measured_copy_gbps(torch, dev)
            roof["measured_copy_gbps"] = copy
            roof["frac_of_measured_copy"] = round(achieved / copy, 4)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args, lib, dot, hdr, deps, order, release, nexec, S, steps, dmax, pw)
        from fantoch_amd import metrics as fm
        # statistics of the all-reduced histograms of the last step (Histogram stats,
        # histogram.rs:61-235, over the exact integer bins)
        hist_stats = {"chain_size": fm.dense_stats(chain.cpu().numpy()),
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
            "data": "synthetic commit streams shaped like EPaxos n=5 (seeded, generated on device; "
                    "deps = latest same-key command of every process within a horizon, not an "
                    "EPaxos fast-quorum union)",
            "config": {
                "workload": "synthetic EPaxos-shaped commit streams, n=%d, %d seeds x conflict {%s}%%, "
                            "%d cmds/process, 1 client/region (BASELINE configs[1] shape)"
                            % (args.n, args.seeds, args.conflicts, args.cmds),
                "instances_per_gpu": instances, "streams_per_gpu": S, "adds_per_stream": steps,
                "window": args.window, "cycle_pct": args.cycle_pct, "seed": args.seed,
                "instance_order": "conflict-major (%d instances per rate)" % cblock if cblock
                                  else "seed-major",
                "parallelism": "instances sharded over %d GPU(s), %s" % (world, LAYOUT.get(tier, "")),
                "tier": tier,
            },
            "edges_per_s": round(edges, 1),
            "executed_per_step": int(executed_total),
            "tier_reruns": bool(tiered[0]),
            "gen_seconds": round(gen_s, 3),
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


def host_cpus():
    """Host cores for the CPU baseline: every core this process may run on
    (nproc = os.cpu_count(); the scheduler affinity and the cgroup CPU quota
    can be lower on a shared GPU box, and threads beyond them only time-slice)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except Exception:
        quota = None
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    usable = min(nproc, aff, quota) if quota else min(nproc, aff)
    return {"nproc": nproc, "affinity": aff, "cgroup_quota_cpus": quota, "usable": usable,
            "model": model}


def workload_key(args):
    return "n%d_s%d_c%s_m%d_w%d_y%d_seed%d_b%d_t%d" % (
        args.n, args.seeds, args.conflicts.replace(",", "-"), args.cmds, args.window,
        args.cycle_pct, args.seed, args.conflict_block, args.tier)


def cpu_baseline(args, lib, dot, hdr, deps, order, release, nexec, S, steps, dmax, pw):
    """Times the CPU oracle (C++ restatement of the reference GraphExecutor) on a
    bounded sample of the same batch, with std::threads over streams like the
    reference's rayon par_iter, and checks the sample against the GPU output.
    The sample is whole 64-stream tiles spread evenly over the batch, so every
    conflict rate is represented in its batch proportion."""
    import numpy as np
    import torch
    from fantoch_amd import streams as fs
    from oracle import oracle_lib

    host = host_cpus()
    threads = host["usable"]
    full_tiles = S // 64
    if full_tiles == 0:
        return None
    # calibrate: ~3.5M Adds/s per thread over the mixed batch (measured) -> whole tiles
    budget_adds = args.cpu_baseline_seconds * 3.5e6 * min(threads, 64)
    tiles = int(max(1, min(full_tiles, budget_adds // (64 * steps))))
    pick = np.unique(np.linspace(0, full_tiles - 1, tiles).round().astype(np.int64))
    tiles = len(pick)
    Ss = tiles * 64
    steps4 = (steps + 3) // 4
    tw = steps4 * 256  # words per tile and plane
    idx = torch.from_numpy((pick[:, None] * tw + np.arange(tw)[None, :]).reshape(-1)).to(dot.device)
    gather = lambda t, base: t[base + idx].cpu().numpy().view(np.uint32)
    planes = fs.Planes(Ss, steps, dmax, args.n)
    planes.dot[:] = gather(dot, 0)[:planes.plane]
    planes.hdr[:] = gather(hdr, 0)[:planes.plane]
    for j in range(dmax):
        planes.deps[j * planes.plane:(j + 1) * planes.plane] = gather(deps, j * pw)[:planes.plane]
    t0 = time.perf_counter()
    o_order, o_rel, o_nexec, o_err = oracle_lib.batch_execute(planes, threads=threads)
    dt = time.perf_counter() - t0
    executed = int(o_nexec.sum())
    g_order = gather(order, 0)
    g_rel = gather(release, 0)
    sidx = torch.from_numpy((pick[:, None] * 64 + np.arange(64)[None, :]).reshape(-1)).to(dot.device)
    g_nexec = nexec[sidx].cpu().numpy().view(np.uint32)
    parity = bool(np.array_equal(g_nexec, o_nexec))
    if parity:
        for s in range(Ss):
            ix = fs.index(np.arange(int(o_nexec[s])), s, steps)
            if not np.array_equal(g_order[ix], o_order[ix]):
                parity = False
                break
        ridx = np.concatenate([fs.index(np.arange(steps), s, steps) for s in range(Ss)])
        parity = parity and bool(np.array_equal(g_rel[ridx], o_rel[ridx]))
    return {"value": round(executed / dt, 1), "unit": "cmds/s", "cores": threads, "kind": "port",
            "host": host,
            "sample": "%d of %d 64-stream tiles spread evenly over the batch (%d streams, %d Adds, "
                      "every conflict rate in proportion), %.2f s wall on %d threads; GPU output "
                      "on the sample %s the oracle bit-for-bit"
                      % (tiles, full_tiles, Ss, Ss * steps, dt, threads,
                         "matches" if parity else "DIFFERS FROM"),
            "sample_parity": parity}


if __name__ == "__main__":
    main()
