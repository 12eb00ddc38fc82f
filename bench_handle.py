"""bench.py --mode handle: the drop-in GraphExecutor handle in the reference
simulator's calling pattern.

Runner::send_to_processes_and_executors (fantoch/src/sim/runner.rs:406-424)
hands every commit to `executor.handle(info, time)` and drains
`executor.to_clients()` right after it, one Add at a time.  Here: the commit
streams a configs[1]-shaped simulation (EPaxos n=5 f=2, GCP regions, 1 client
per region, `--conflicts` first rate) feeds each process's GraphExecutor,
captured from the simulator oracle, replayed through

  GPU   fx_graph_executor_handle_add + fx_graph_executor_drain_dots after
        every Add (the C-ABI handle of include/fantoch_amd.h: one resumable
        executor launch per pull);
  CPU   the oracle DependencyGraph (oracle/graph_oracle.hpp), the same Adds
        one handle_add at a time through ctypes, and the same stream as one
        C++ loop (oracle batch_execute), for the per-Add cost without the
        Python call overhead.

Both execution orders must equal the simulation's.  value = Adds per second of
the GPU handle (one process stream; latency-bound: one launch per Add)."""
import json
import os
import time

import numpy as np


def main_handle(args):
    import torch  # noqa: F401  (initialises the HIP runtime like the other modes)

    from bench import host_cpus
    from fantoch_amd import _lib
    from fantoch_amd import sim as S
    from fantoch_amd import streams as fs
    from fantoch_amd.executor import GraphExecutor
    from oracle import oracle_lib as O

    lib = _lib.load()
    if lib.fx_device_count() <= 0:
        raise SystemExit("no GPU visible to libfantoch_amd")
    cmds = args.cmds if args.cmds is not None else 200
    conflict = int(args.conflicts.split(",")[-1])
    pl = S.Planet()
    regs = pl.ids(S.GCP5[:5])
    spec = O.spec_from(S.spec(S.EPAXOS, 5, 2, regs, regs, commands_per_client=cmds, conflict_rate=conflict,
                              seed=args.seed, instance=0))
    streams, executed = O.sim_capture(spec)
    p = 0
    stream = streams[p]
    want = [(int(d) >> 24, int(d) & 0xFFFFFF) for d in executed[p]]
    # GPU handle, drained after every Add
    warm = GraphExecutor(p + 1, 0, 5, f=2, monitor=False)  # module load, first allocations
    for (dot, deps, t) in stream[:32]:
        warm.handle_add(dot, dot, [0], deps, t)
        warm.drain_dots()
    warm.close()
    ex = GraphExecutor(p + 1, 0, 5, f=2, monitor=False)
    got = []
    t0 = time.perf_counter()
    for (dot, deps, t) in stream:
        ex.handle_add(dot, dot, [0], deps, t)
        got += [d for d, _ in ex.drain_dots()]
    gpu_s = time.perf_counter() - t0
    ex.close()
    # CPU oracle, one handle_add per call (ctypes) and the same stream in one C++ loop
    g = O.Graph(p + 1, 5)
    t0 = time.perf_counter()
    for (dot, deps, t) in stream:
        g.handle_add(dot, deps, t)
    cpu_call_s = time.perf_counter() - t0
    cpu_order = [d for d, _, _ in g.drain()]
    planes = fs.pack_streams([[(dot, deps, t) for dot, deps, t in stream]], 5)
    t0 = time.perf_counter()
    reps = 20
    for _ in range(reps):
        o_order, _, o_nexec, _ = O.batch_execute(planes, threads=1)
    cpu_loop_s = (time.perf_counter() - t0) / reps
    nadd = len(stream)
    # the same loop in C++ over the C-ABI (tools/handle_latency.cpp): the
    # handle's own cost per Add, without ctypes argument marshalling
    cpp = _cpp_loop(stream, want, p + 1)
    parity = got == want and cpu_order == want and (cpp is None or cpp["order_parity"])
    # value: the handle driven by compiled code over the C-ABI, as the
    # reference's Rust runner drives its executor (the Python loop's rate, with
    # the ctypes marshalling of every call, is reported beside it)
    cpp_ok = bool(cpp and cpp.get("us_per_add_median"))
    step_s = cpp["us_per_add_median"] * nadd / 1e6 if cpp_ok else gpu_s
    line = {
        "metric": "GraphExecutor handle: Adds/s, drained after every Add (runner.rs:406-424 pattern)",
        "value": round(nadd / step_s, 1), "unit": "Adds/s", "n_gpus": 1, "steps": 1, "warmup": 0,
        "ms_per_step": round(step_s * 1e3, 3), "higher_is_better": True, "scaling": "none",
        "value_source": "C++ loop over the C-ABI (tools/handle_latency.cpp), median of 5 passes" if cpp_ok
                        else "Python loop (ctypes)",
        "python_adds_per_s": round(nadd / gpu_s, 1),
        "vs_baseline": None, "dtype": "u32",
        "data": "commit stream of process 1 captured from the simulator oracle",
        "config": {"workload": "EPaxos n=5 f=2, GCP regions, 1 client/region, %d cmds/client, %d%% conflicts: "
                               "process 1's %d Adds" % (cmds, conflict, nadd)},
        "gpu_us_per_add": round(gpu_s / nadd * 1e6, 2),
        "gpu_us_per_add_cpp_loop": cpp["us_per_add_median"] if cpp else None,
        "gpu_cpp_loop": {k: v for k, v in cpp.items() if k != "order"} if cpp else None,
        "cpu_oracle_us_per_add_ctypes": round(cpu_call_s / nadd * 1e6, 3),
        "cpu_oracle_us_per_add_cpp_loop": round(cpu_loop_s / nadd * 1e6, 4),
        "cpu_baseline": {"value": round(nadd / cpu_loop_s, 1), "unit": "Adds/s", "cores": 1, "kind": "port",
                         "host": host_cpus(),
                         "sample": "the same %d Adds through the oracle DependencyGraph in one C++ loop "
                                   "(batch_execute, 1 thread), %d repetitions" % (nadd, reps)},
        "order_parity": bool(parity),
        "note": "persistent mode: one resident wavefront executes the Adds a pull publishes in host-mapped "
                "memory (no launch, no stream synchronisation per pull); gpu_us_per_add includes the Python "
                "ctypes calls (handle_add + drain_dots), gpu_us_per_add_cpp_loop the same loop in C++ (value). "
                "Handle creation (stream with its own hardware queue, mapped buffers; pooled across handles) "
                "is outside both loops, as GraphExecutor::new is outside the reference's. The batched entry "
                "points (fx_batch_*, fx_sim_run) are the throughput path",
    }
    print(json.dumps(line), flush=True)
    if not parity:
        raise SystemExit("handle order differs from the simulation's")
    return line


def _cpp_loop(stream, want, pid, reps=5):
    """Runs tools/build/handle_latency on the stream (None if it is not built)."""
    import struct
    import subprocess
    import tempfile
    root = os.path.dirname(os.path.abspath(__file__))
    exe = os.path.join(root, "tools", "build", "handle_latency")
    if not os.path.exists(exe):
        return None
    buf = [struct.pack("<III", 5, pid, len(stream))]
    for (dot, deps, t) in stream:
        buf.append(struct.pack("<IIII", dot[0], dot[1], t, len(deps)))
        for d in deps:
            buf.append(struct.pack("<II", d[0], d[1]))
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as fh:
        fh.write(b"".join(buf))
        path = fh.name
    keep = os.environ.get("BENCH_HANDLE_KEEP_STREAM")  # tools/queue_probe.sh reuses the stream
    if keep:
        import shutil
        shutil.copyfile(path, keep)
    try:
        out = subprocess.run([exe, path, str(reps)], capture_output=True, text=True, timeout=120)
    finally:
        os.unlink(path)
    if out.returncode != 0:
        return {"error": out.returncode, "order_parity": False, "us_per_add_median": None}
    lines = out.stdout.strip().splitlines()
    d = json.loads(lines[-1])
    for ln in lines[:-1]:
        if ln.startswith('{"persist"'):
            d.update(json.loads(ln))
    d["order_parity"] = [(x >> 24, x & 0xFFFFFF) for x in d["order"]] == want
    return d
