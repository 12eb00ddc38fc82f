"""bench.py --mode huge: BASELINE configs[4], one simulated instance whose five
executors each see a 10^6-Add commit stream with cycles (synthetic Atlas
commit streams, n = 5, 2 % conflicts, 30 % cross-coordinator cycles), executed
by the quiescent-cut driver (fx_batch_run_cut, graph_cut.hip).

One step = fx_batch_run_cut over the 5 x 10^6 Adds + fx_batch_metrics.  The
instance does not shard: with --gpus N every rank runs its
own replica and `value` counts the Adds of all replicas.  cpu_baseline: the
C++ oracle (oracle/graph_oracle.cpp, one std::thread per stream) on the same
five streams, whose outputs are also compared with the GPU's bit for bit."""
import ctypes
import json
import os
import time

HBM_PEAK_GBPS = 8000.0


def main_huge(args):
    import numpy as np
    import torch
    import torch.distributed as dist

    from fantoch_amd import _lib
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
    cmds = args.cmds if args.cmds is not None else 200_000  # n x cmds = 10^6 Adds per executor
    shape = getattr(args, "huge_shape", "conflict2")
    if shape == "s5":  # per-key chains over a key pool plus cycles
        horizon = args.horizon if args.horizon is not None else 640
        p = fs.synth_params(seed=args.seed, instances=1, n=5, cmds=cmds, window=args.window,
                            cycle_pct=args.cycle_pct, horizon=horizon, key_pool=args.key_pool)
        shape_desc = "per-key chains over %d keys, %d %%%% concurrent pairs cycling, horizon %d" % (
            args.key_pool, args.cycle_pct, horizon)
    else:
        rate = 2 if shape == "conflict2" else 100
        horizon = args.horizon if args.horizon is not None else 64
        p = fs.synth_params(seed=args.seed, instances=1, n=5, cmds=cmds, window=args.window,
                            cycle_pct=args.cycle_pct, horizon=horizon, conflicts=(rate,))
        shape_desc = "%d %%%% conflicts, %d %%%% cycles" % (rate, args.cycle_pct)
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
    _lib.check(lib.fx_synth_generate(ctypes.byref(p), dot.data_ptr(), hdr.data_ptr(), deps.data_ptr(), hs),
               "fx_synth_generate")
    torch.cuda.synchronize(dev)
    inb = _lib.StreamBatch(dot.data_ptr(), hdr.data_ptr(), deps.data_ptr(), None, S, steps, dmax, 5)
    outb = _lib.OrderBatch(order.data_ptr(), release.data_ptr(), nexec.data_ptr(), err.data_ptr())
    hb = _lib.HistBatch(chain.data_ptr(), NBC, delay.data_ptr(), NBD)
    nd_total = int(((hdr >> 24) & 31).sum(dtype=torch.int64).item())
    n_adds = S * steps
    stats = _lib.CutStats()
    # the segment batch's first executor tier (--tier; default FX_TIER_DEFAULT)
    cut_flags = _lib.first_tier_flag(args.tier) if args.tier >= 0 else 0

    def step():
        chain.zero_()
        delay.zero_()
        st = lib.fx_batch_run_cut(ctypes.byref(inb), ctypes.byref(outb), cut_flags, hs, ctypes.byref(stats))
        _lib.check(st, "fx_batch_run_cut")
        _lib.check(lib.fx_batch_metrics(ctypes.byref(inb), ctypes.byref(outb), ctypes.byref(hb), hs),
                   "fx_batch_metrics")

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.time()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.time() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    executed = int(nexec.sum(dtype=torch.int64).item())
    assert executed == n_adds and int((err != 0).sum().item()) == 0, "configs[4] run incomplete"
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    value = executed * world * args.steps / elapsed
    alg_bytes = (36.0 * n_adds + 8.0 * nd_total)
    achieved = alg_bytes / (elapsed / args.steps) / 1e9
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        from oracle import oracle_lib
        host = fs.Planes(S, steps, dmax, 5, dot=dot.cpu().numpy().view(np.uint32),
                         hdr=hdr.cpu().numpy().view(np.uint32), deps=deps.cpu().numpy().view(np.uint32))
        t1 = time.time()
        o_order, o_rel, o_nexec, o_err = oracle_lib.batch_execute(host, threads=S)
        cpu_s = time.time() - t1
        g_order = order.cpu().numpy().view(np.uint32)
        g_rel = release.cpu().numpy().view(np.uint32)
        same = bool(np.array_equal(o_nexec, nexec.cpu().numpy().view(np.uint32)))
        for s in range(S):
            idx = _lib.index(np.arange(steps), s, steps)
            same = same and np.array_equal(g_order[idx], o_order[idx]) and np.array_equal(g_rel[idx], o_rel[idx])
        cpu = {"value": round(n_adds / cpu_s, 1), "unit": "cmds/s", "cores": S, "kind": "port",
               "sample": "the whole configs[4] instance (5 x %d Adds) through the C++ oracle, one thread per "
                         "executor stream (the reference's executors of one instance run on their own "
                         "tasks), %.3f s; GPU output identical: %s" % (steps, cpu_s, same),
               "sample_parity": same}
    huge_roof = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                 "frac": round(achieved / HBM_PEAK_GBPS, 6), "traffic": None,
                 "kernel": "fx_batch_run_cut (cut analysis + segment executor + scatter)",
                 "alg_bytes_per_launch": int(alg_bytes), "alg_bytes_per_cmd": round(alg_bytes / n_adds, 3)}
    # HBM traffic of the whole step (every kernel of the cut driver summed):
    # tools/mode_pmc.sh huge -> profiles/pmc_huge.json, when it was measured on this workload
    import bench_pmc
    bench_pmc.attach(huge_roof, bench_pmc.load("huge", args), alg_bytes)
    line = {
        "metric": "executed cmds/sec (node) for batched Atlas/EPaxos sims; % of HBM roofline",
        "value": round(value, 1), "unit": "cmds/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": ("synthetic Atlas commit streams (fx_synth: " + shape_desc + ", window %d)") % args.window,
        "config": {"workload": "single huge instance: 5 executors x %d Adds with cycles (BASELINE configs[4]), "
                               "shape %s" % (steps, shape), "mean_deps": round(nd_total / n_adds, 3),
                   "parallelism": "quiescent-cut decomposition on one GPU; replicas only across GPUs"},
        "segments": int(stats.segments), "single_segments": int(stats.single_segments),
        "max_segment": int(stats.max_segment),
        "whole_streams": int(stats.whole_streams),
        "roofline": huge_roof,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_dense(args):
    """bench.py --mode dense: BASELINE configs[3], the dense-dependency stress:
    EPaxos-shaped commit streams of n = 5 processes with 64 closed-loop clients
    each, 100 % conflicts, 30 % concurrent cycles (SCCs of whole rounds of 320
    commands, ~480 pending vertices), `--seeds` instances per GPU, executed by
    fx_batch_run_tiered starting at the wide tier (`--tier`, default 7)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from bench import host_cpus
    from fantoch_amd import _lib
    from fantoch_amd import streams as fs

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    lib = _lib.load()
    if lib.fx_device_count() <= 0:
        raise SystemExit("no GPU visible to libfantoch_amd")
    clients = 64
    cmds = args.cmds if args.cmds is not None else 20  # per client
    instances = args.seeds  # default 768 (bench.MODE_DEFAULTS["dense"]): 3,840 streams
    p = fs.synth_params(seed=args.seed, instances=instances, instance_base=rank * instances, n=5,
                        cmds=clients * cmds, window=5 * clients, cycle_pct=30, conflicts=(100,), clients=clients)
    S, steps, dmax = fs.synth_shape(p)
    pw = _lib.plane_words(S, steps)
    stream = torch.cuda.current_stream(dev)
    hs = ctypes.c_void_p(stream.cuda_stream)

    def buf(words):
        return torch.empty(words, dtype=torch.int32, device=dev)

    dot, hdr, deps = buf(pw), buf(pw), buf(pw * dmax)
    order, release = buf(pw), buf(pw)
    nexec, err = buf(S), buf(S)
    NBC, NBD = 1024, 8192
    chain = torch.zeros(NBC, dtype=torch.int64, device=dev)
    delay = torch.zeros(NBD, dtype=torch.int64, device=dev)
    _lib.check(lib.fx_synth_generate(ctypes.byref(p), dot.data_ptr(), hdr.data_ptr(), deps.data_ptr(), hs),
               "fx_synth_generate")
    torch.cuda.synchronize(dev)
    inb = _lib.StreamBatch(dot.data_ptr(), hdr.data_ptr(), deps.data_ptr(), None, S, steps, dmax, 5)
    outb = _lib.OrderBatch(order.data_ptr(), release.data_ptr(), nexec.data_ptr(), err.data_ptr())
    hb = _lib.HistBatch(chain.data_ptr(), NBC, delay.data_ptr(), NBD)
    tier = _lib.FX_TIER_WIDE if args.tier < 0 else args.tier
    tier_counts = (ctypes.c_uint32 * _lib.FX_NUM_TIERS)()

    def step():
        chain.zero_()
        delay.zero_()
        _lib.check(lib.fx_batch_run_tiered(ctypes.byref(inb), ctypes.byref(outb), _lib.first_tier_flag(tier), hs,
                                           tier_counts), "fx_batch_run_tiered")
        _lib.check(lib.fx_batch_metrics(ctypes.byref(inb), ctypes.byref(outb), ctypes.byref(hb), hs),
                   "fx_batch_metrics")

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    # the dominant kernel (the first tier's launch over every stream) and the
    # rerun tier, each timed by HIP events on the stream it runs on
    lib.fx_profile_enable(1)
    tier_ms = {tier: [], _lib.FX_TIER_WIDE_HBM: []}
    t0 = time.time()
    for _ in range(args.steps):
        step()
        for tt in tier_ms:
            ms = ctypes.c_float()
            if lib.fx_profile_slot_ms(tt, ctypes.byref(ms)) == 0:
                tier_ms[tt].append(ms.value)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.time() - t0
    lib.fx_profile_enable(0)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        for h in (chain, delay):
            dist.all_reduce(h)
    n_adds = S * steps
    executed = int(nexec.sum(dtype=torch.int64).item())
    assert executed == n_adds and int((err != 0).sum().item()) == 0, "configs[3] run incomplete"
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    ch = chain.cpu().numpy()
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        from oracle import oracle_lib
        host = host_cpus()
        k = max(1, min(instances, int((args.cpu_baseline_seconds or 10) * host["usable"] / 1.5)))
        sub = fs.synth_params(seed=args.seed, instances=k, n=5, cmds=clients * cmds, window=5 * clients,
                              cycle_pct=30, conflicts=(100,), clients=clients)
        hp = fs.synth_host(sub)
        t1 = time.time()
        o_order, o_rel, o_nexec, o_err = oracle_lib.batch_execute(hp, threads=host["usable"])
        cpu_s = time.time() - t1
        g_order = order.cpu().numpy().view(np.uint32)
        g_rel = release.cpu().numpy().view(np.uint32)
        same = True
        for s in range(hp.S):  # the sample is the first k instances of the GPU batch (rank 0)
            a = _lib.index(np.arange(steps), s, steps)
            b = _lib.index(np.arange(steps), s, hp.steps)
            same = same and np.array_equal(g_order[a], o_order[b]) and np.array_equal(g_rel[a], o_rel[b])
        cpu = {"value": round(hp.S * hp.steps / cpu_s, 1), "unit": "cmds/s", "cores": host["usable"],
               "kind": "port", "host": host,
               "sample": "%d of %d instances (5 executors x %d Adds each) through the C++ oracle on %d threads, "
                         "%.2f s; GPU output identical: %s" % (k, instances, steps, host["usable"], cpu_s, same),
               "sample_parity": same}
    alg_bytes = 36.0 * n_adds + 8.0 * int(((hdr >> 24) & 31).sum(dtype=torch.int64).item())
    kms = {tt: (sum(v) / len(v) if v else None) for tt, v in tier_ms.items()}
    k_main = kms.get(tier)
    import bench_pmc
    roof = {"bound": "hbm", "peak": HBM_PEAK_GBPS, "unit": "GB/s", "kernel": "k_graph_wide<false> (tier %d)" % tier,
            "alg_bytes_per_cmd": round(alg_bytes / n_adds, 3), "alg_bytes_per_launch": int(alg_bytes),
            "alg_bytes_definition": "SURVEY.md 8(d): 32 + 4k + 8d per command, k = 1",
            "kernel_ms_avg": round(k_main, 3) if k_main else None,
            "rerun_tier_ms_avg": round(kms[_lib.FX_TIER_WIDE_HBM], 3) if kms.get(_lib.FX_TIER_WIDE_HBM) else None,
            "step_ms": round(elapsed / args.steps * 1e3, 3)}
    # achieved = algorithmic bytes over the dominant kernel's own time (HIP events)
    secs = (k_main * 1e-3) if k_main else elapsed / args.steps
    roof["achieved"] = round(alg_bytes / secs / 1e9, 3)
    roof["frac"] = round(alg_bytes / secs / 1e9 / HBM_PEAK_GBPS, 6)
    bench_pmc.attach(roof, bench_pmc.load("dense", args), alg_bytes)
    if roof.get("issue"):
        roof["note"] = ("one wavefront per stream walking the pending graph: latency-bound "
                        "(issue.wait_any_frac_of_wave_cycles, issue.mean_waves_per_cu)")
    line = {
        "metric": "executed cmds/sec (node) for batched Atlas/EPaxos sims; % of HBM roofline",
        "value": round(executed * world * args.steps / elapsed, 1), "unit": "cmds/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic EPaxos-shaped commit streams (fx_synth, 64 clients per process, 100 %% conflicts, "
                "30 %% concurrent cycles, window %d)" % (5 * clients),
        "config": {"workload": "dense-dependency stress: %d instances x 5 executors x %d Adds, 64 clients/region "
                               "(BASELINE configs[3])" % (instances, steps),
                   "parallelism": "instances sharded over %d GPU(s); first tier %d" % (world, tier)},
        "tier_counts": list(tier_counts),
        "chain_size_max": int(np.nonzero(ch)[0].max()) if ch.any() else 0,
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
