"""bench.py --mode pred: Caesar's PredecessorsExecutor
over batched commit streams of configs[1]'s shape.

Streams: fx_synth's EPaxos-shaped commit streams (n = 5, `--seeds` instances x
`--conflicts`, `--cmds` commands per process, window / cycles as the executor
bench), each Add given the Caesar clock (seq, process id) of its dot, packed as
(seq << 8) | id.  A dep with a lower clock is a predecessor the command waits
to execute (phase two); the cycle edges point at higher clocks and only wait
for the commit (phase one).  One step = fx_pred_run over every stream (table
tiers SMALL -> LDS -> HBM).  value = Adds executed / step time.

cpu_baseline: the predecessors oracle (oracle/pred_oracle.cpp) on the first
tiles of the batch, every usable host core, checked against the GPU's order,
release and nexec for those streams."""
import ctypes
import json
import os
import time
import types

import numpy as np

HBM_PEAK_GBPS = 8000.0


def main_pred(args):
    import torch

    from bench import host_cpus
    from fantoch_amd import _lib
    from fantoch_amd import streams as fs

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    import torch.distributed as dist
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    lib = _lib.load()
    if lib.fx_device_count() <= 0:
        raise SystemExit("no GPU visible to libfantoch_amd")
    cmds = args.cmds if args.cmds is not None else 1000
    seeds = args.seeds
    conflicts = tuple(int(c) for c in args.conflicts.split(","))
    p = fs.synth_params(seed=args.seed, instances=seeds * len(conflicts), instance_base=rank * seeds * len(conflicts),
                        n=args.n, cmds=cmds, window=args.window, cycle_pct=args.cycle_pct, conflicts=conflicts,
                        conflict_block=seeds)
    S, steps, dmax = fs.synth_shape(p)
    pw = _lib.plane_words(S, steps)
    stream = torch.cuda.current_stream(dev)
    hs = ctypes.c_void_p(stream.cuda_stream)

    def buf(words):
        return torch.empty(words, dtype=torch.int32, device=dev)

    dot, hdr, deps = buf(pw), buf(pw), buf(pw * dmax)
    order, release, nexec, err = buf(pw), buf(pw), buf(S), buf(S)
    _lib.check(lib.fx_synth_generate(ctypes.byref(p), dot.data_ptr(), hdr.data_ptr(), deps.data_ptr(), hs),
               "fx_synth_generate")
    # Caesar clock of each Add: (seq, process id) of its dot
    clo = (((dot & 0xFFFFFF) << 8) | ((dot >> 24) & 0xFF)).contiguous()
    chi = torch.zeros_like(clo)
    torch.cuda.synchronize(dev)
    base = _lib.StreamBatch(dot.data_ptr(), hdr.data_ptr(), deps.data_ptr(), None, S, steps, dmax, args.n)
    inb = _lib.PredBatch(base, clo.data_ptr(), chi.data_ptr(), None)
    outb = _lib.OrderBatch(order.data_ptr(), release.data_ptr(), nexec.data_ptr(), err.data_ptr())
    reruns = ctypes.c_uint32()

    def step():
        _lib.check(lib.fx_pred_run(ctypes.byref(inb), ctypes.byref(outb), 0, hs, ctypes.byref(reruns)),
                   "fx_pred_run")

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    # the dominant kernel: the SMALL tier's launch over every stream (HIP
    # events on the stream it runs on); the capacity reruns beside it
    lib.fx_profile_enable(1)
    slot_ms = {t: [] for t in (_lib.FX_PRED_TIER_SMALL, _lib.FX_PRED_TIER_LDS, _lib.FX_PRED_TIER_HBM)}
    t0 = time.time()
    for _ in range(args.steps):
        step()
        for t in slot_ms:
            ms = ctypes.c_float()
            if lib.fx_profile_slot_ms(_lib.FX_PROFILE_SLOT_PRED + t, ctypes.byref(ms)) == 0:
                slot_ms[t].append(ms.value)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.time() - t0
    lib.fx_profile_enable(0)
    executed = int(nexec.to(torch.int64).sum().item())
    nd_total = int(((hdr.to(torch.int64) >> 24) & 31).sum().item())
    n_adds = S * steps
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return None
    import bench_pmc
    value = executed * world * args.steps / elapsed
    # §8(d) record bytes (k = 1) plus the 8-byte clock
    alg_bytes = 44.0 * n_adds + 8.0 * nd_total
    kms = {t: (sum(v) / len(v) if v else None) for t, v in slot_ms.items()}
    k_main = kms[_lib.FX_PRED_TIER_SMALL]
    achieved = alg_bytes / ((k_main * 1e-3) if k_main else elapsed / args.steps) / 1e9
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = _cpu_baseline(args, S, steps, dmax, pw, dot, hdr, deps, clo, chi, order, release, nexec)
    line = {
        "metric": "executed cmds/sec (node), Caesar PredecessorsExecutor over batched commit streams",
        "value": round(value, 1), "unit": "cmds/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic commit streams (fx_synth, EPaxos-shaped) with Caesar clocks (seq, process id)",
        "config": {"workload": "PredecessorsExecutor, n=%d, %d seeds x conflict %s %%, %d cmds/process"
                               % (args.n, seeds, list(conflicts), cmds),
                   "streams_per_gpu": S, "adds_per_stream": steps,
                   "parallelism": "one wavefront per stream; instances sharded over %d GPU(s)" % world},
        "executed_per_step": executed, "reruns": int(reruns.value),
        "roofline": bench_pmc.attach(
            {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
             "frac": round(achieved / HBM_PEAK_GBPS, 6), "kernel": "k_pred<false, 5, 5> (SMALL tier, layout compiled in for n = 5; every stream)",
             "kernel_ms_avg": round(k_main, 3) if k_main else None,
             "rerun_ms_avg": {"lds": round(kms[_lib.FX_PRED_TIER_LDS], 3) if kms[_lib.FX_PRED_TIER_LDS] else None,
                              "hbm": round(kms[_lib.FX_PRED_TIER_HBM], 3) if kms[_lib.FX_PRED_TIER_HBM] else None},
             "alg_bytes_per_cmd": round(alg_bytes / n_adds, 3), "alg_bytes_per_launch": int(alg_bytes),
             "alg_bytes_definition": "SURVEY.md 8(d): 32 + 4k + 8d per command, k = 1, plus the 8-byte Caesar clock"},
            bench_pmc.load("pred", args), alg_bytes),
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return line


def _cpu_baseline(args, S, steps, dmax, pw, dot, hdr, deps, clo, chi, order, release, nexec):
    """The oracle over the first tiles (64 streams each, a contiguous prefix of
    every plane), all usable host cores; GPU output compared on them."""
    from bench import host_cpus
    from fantoch_amd import _lib
    from oracle import oracle_lib as O

    host = host_cpus()
    threads = host["usable"]
    # a quarter of the batch (~10 s of oracle work at configs[1]'s shape), or
    # --cpu-baseline-seconds x 64 streams per second budgeted
    T = (S + 63) // 64
    tiles = max(1, min(T, int(args.cpu_baseline_seconds * 64) if args.cpu_baseline_seconds else (T + 3) // 4))
    Ss = min(S, 64 * tiles)
    tw = _lib.plane_words(Ss, steps)

    def pre(t, k=1):
        a = t.view(k, pw)[:, :tw].cpu().numpy().view(np.uint32)
        return np.ascontiguousarray(a.reshape(-1))
    planes = types.SimpleNamespace(dot=pre(dot), hdr=pre(hdr), deps=pre(deps, dmax), lengths=None, S=Ss,
                                   steps=steps, dmax=dmax, n=args.n, plane=tw)
    t0 = time.time()
    o_order, o_rel, o_nexec, o_err = O.pred_batch_execute(planes, pre(clo), pre(chi), threads=threads)
    dt = time.time() - t0
    g_nexec = nexec[:Ss].cpu().numpy().view(np.uint32)
    g_order, g_rel = pre(order), pre(release)
    same = bool(np.array_equal(o_nexec, g_nexec) and not o_err.any())
    if same and Ss % 64 == 0 and np.all(o_nexec == steps):  # every row of every plane is defined
        same = bool(np.array_equal(g_order, o_order) and np.array_equal(g_rel, o_rel))
        Ss_loop = 0
    else:
        Ss_loop = Ss
    for s in range(Ss_loop):
        rows = _lib.index(np.arange(int(o_nexec[s])), s, steps)
        allr = _lib.index(np.arange(steps), s, steps)
        same = same and np.array_equal(g_order[rows], o_order[rows]) and np.array_equal(g_rel[allr], o_rel[allr])
    return {"value": round(float(o_nexec.sum()) / dt, 1), "unit": "cmds/s", "cores": threads, "kind": "port",
            "host": host,
            "sample": "the first %d streams (%d Adds) through the C++ predecessors oracle in %.2f s on %d threads; "
                      "GPU output on them %s" % (Ss, Ss * steps, dt, threads, "identical" if same else "DIFFERS"),
            "sample_parity": same}
