"""World-size-2 (gloo, CPU) check of the simulator benches' multi-GPU plan
(DESIGN.md §6): bench_sim.py's rank enumeration (rank r owns
the contiguous global instance range [r P, (r + 1) P)), its histogram
all-reduce and per-instance row all-gather, and bench_placements.py's
contiguous placement ranges with their variable-size row gather.  The
simulator oracle stands in for the kernel (the GPU tests check the two bit
for bit); the enumeration, the row construction and the collectives are the
bench code itself.  The gathered output must equal one run over the union of
both ranks' instances, in global order."""
import os
import socket
import sys
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
ARGS = dict(seeds=2, conflicts="0,50,100", n=3, cmds=20, protocol="both", f=1, seed=5,
            clients_per_region=2)
LAT_BINS, CHAIN_BINS, DELAY_BINS = 2048, 64, 2048


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def oracle_outputs(specs):
    """The kernel's outputs for `specs`, produced by the simulator oracle:
    executed_len [N n], stats [N FX_SIM_STATS], err [N], and the batch
    histograms (latency per region, ChainSize, ExecutionDelay)."""
    from fantoch_amd import _lib
    from oracle import oracle_lib as O
    res = O.sim_batch([O.spec_from(s) for s in specs], threads=2, lat_bins=LAT_BINS,
                      chain_bins=CHAIN_BINS, delay_bins=DELAY_BINS)
    N, n = len(specs), specs[0].n
    el = np.zeros((N, n), np.int64)
    st = np.zeros((N, _lib.FX_SIM_STATS), np.int64)
    err = np.zeros(N, np.int64)
    lat = chain = delay = 0
    for i, r in enumerate(res):
        el[i] = [len(e) for e in r["executed"]]
        st[i, _lib.FX_SIM_STAT_FAST:_lib.FX_SIM_STAT_FAST + n] = r["fast"]
        st[i, _lib.FX_SIM_STAT_SLOW:_lib.FX_SIM_STAT_SLOW + n] = r["slow"]
        st[i, _lib.FX_SIM_STAT_LAT_SUM] = sum(ms * int(c) for h in r["latency"] for ms, c in enumerate(h) if c)
        err[i] = r["status"]
        lat = lat + r["latency"].astype(np.int64)
        chain = chain + r["chain"].astype(np.int64)
        delay = delay + r["delay"].astype(np.int64)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    return t(el.reshape(-1)), t(st.reshape(-1)), t(err), [t(lat.reshape(-1)), t(chain), t(delay)]


def sim_rank(rank, world):
    sys.path.insert(0, ROOT)
    import bench_sim as B
    from fantoch_amd import sim as S
    args = types.SimpleNamespace(**ARGS)
    specs, rates, _ = B.local_specs(S, args, rank, S.Planet())
    el, st, err, hists = oracle_outputs(specs)
    B.allreduce_hists(dist, world, hists)
    rows = B.gather_rows(dist, world, B.instance_rows(torch, rank * len(specs), rates, el, st, err, args.n))
    return hists, rows, specs


def placements_rank(rank, world, limit):
    sys.path.insert(0, ROOT)
    import bench_placements as BP
    from fantoch_amd import sim as S
    pl = S.Planet()
    allp = BP.enumerate_placements(pl.R, limit)
    lo, hi = BP.rank_range(len(allp), rank, world)
    ids = list(range(lo, hi))
    specs = [S.spec(S.ATLAS, allp[g][0], allp[g][1], list(allp[g][2]), list(allp[g][2]), commands_per_client=10,
                    conflict_rate=10, seed=3, instance=g) for g in ids]
    el, st, err, _ = oracle_outputs(specs)
    rows = BP.placement_rows(torch, ids, allp, allp[0][0], 10, el, st, err)
    return BP.gather_rows(dist, world, rows), len(ids)


def worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hists, rows, specs = sim_rank(rank, world)
    prow, pcount = placements_rank(rank, world, 41)
    if rank == 0:
        q.put(([h.numpy() for h in hists], rows.numpy(), prow.numpy()))
    q.put(("count", rank, len(specs), pcount, [int(s.instance) for s in specs]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(3)]
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    main = next(g for g in got if g[0] != "count")
    counts = sorted((g for g in got if g[0] == "count"), key=lambda g: g[1])
    return main, counts


def test_sim_two_ranks_equal_single_run_over_union(two_ranks):
    (hists2, rows2, _), counts = two_ranks
    sys.path.insert(0, ROOT)
    import bench_sim as B
    from fantoch_amd import sim as S
    args = types.SimpleNamespace(**ARGS)
    regs = S.Planet().ids(S.GCP5[:args.n])
    P = counts[0][2]
    assert counts[1][2] == P
    # the ranks tile the global enumeration: rank r holds instances [r P, (r + 1) P)
    assert counts[0][4] == list(range(P)) and counts[1][4] == list(range(P, 2 * P))
    union = [B.global_spec(S, args, g, regs) for g in range(2 * P)]
    specs = [s for s, _ in union]
    el, st, err, hists1 = oracle_outputs(specs)
    rows1 = B.instance_rows(torch, 0, [c for _, c in union], el, st, err, args.n).numpy()
    assert np.array_equal(rows2, rows1)
    assert list(rows1[:, 0]) == list(range(2 * P))
    assert sorted(set(rows1[:, 1])) == [0, 50, 100] and np.all(rows1[:, 5] == 0)
    for a, b in zip(hists2, hists1):
        assert np.array_equal(a, b.numpy())
    assert hists1[1].sum() > 0
    # --protocol both alternates Atlas f=1 and EPaxos over the global ids
    assert [s.protocol for s in specs[:4]] == [S.ATLAS, S.EPAXOS, S.ATLAS, S.EPAXOS]


def test_placements_two_ranks_cover_the_enumeration(two_ranks):
    (_, _, prow2), counts = two_ranks
    assert (counts[0][3], counts[1][3]) == (20, 21)  # 41 placements: ranges [0, 20), [20, 41)
    sys.path.insert(0, ROOT)
    import bench_placements as BP
    from fantoch_amd import sim as S
    pl = S.Planet()
    allp = BP.enumerate_placements(pl.R, 41)
    specs = [S.spec(S.ATLAS, n, f, list(sub), list(sub), commands_per_client=10, conflict_rate=10, seed=3,
                    instance=g) for g, (n, f, sub) in enumerate(allp)]
    el, st, err, _ = oracle_outputs(specs)
    rows1 = BP.placement_rows(torch, list(range(41)), allp, 5, 10, el, st, err).numpy()
    assert np.array_equal(prow2, rows1)
    assert list(rows1[:, 0]) == list(range(41)) and np.all(rows1[:, 8] == 0)
