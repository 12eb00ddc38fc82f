"""World-size-2 (gloo, CPU) check of the multi-GPU plan:
rank r owns instances [r*I, (r+1)*I) and only the integer histograms are
all-reduced.  The CPU oracle stands in for the executor kernel (same outputs,
checked bit-exactly by the GPU tests); the sharding, the synthetic-stream
enumeration and the reduction are the product code that bench.py runs."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CFG = dict(seeds=3, conflicts=(0, 50, 100), n=5, cmds=30, window=8, cycle_pct=30, seed=77)


def shard_hists(rank, world, **kw):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from fantoch_amd import sharding
    from fantoch_amd import streams as fs
    from oracle import oracle_lib
    import make_golden as G
    p = sharding.rank_params(rank, **kw)
    planes = fs.synth_host(p)
    order, release, nexec, err = oracle_lib.batch_execute(planes, threads=2)
    chain, delay = G.hists(planes, order, release, nexec)
    rows = sharding.instance_summaries(torch.from_numpy(nexec.astype(np.int64)),
                                       torch.from_numpy(err.astype(np.int64)), p)
    return (planes, torch.from_numpy(chain.astype(np.int64)),
            torch.from_numpy(delay.astype(np.int64)), rows)


def worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    from fantoch_amd import sharding
    planes, chain, delay, rows = shard_hists(rank, world, **CFG)
    sharding.allreduce_histograms(dist, chain, delay)
    table = sharding.gather_summaries(dist, rows, world)
    total = torch.tensor([int(planes.S)], dtype=torch.int64)
    dist.all_reduce(total)
    if rank == 0:
        out.put((chain.numpy(), delay.numpy(), int(total.item()), table.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_histograms_equal_single_run():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    chain2, delay2, streams2, table2 = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    # one process over the union of both shards (2x the instances from 0)
    cfg = dict(CFG)
    cfg["seeds"] = 2 * CFG["seeds"]
    sys.path.insert(0, ROOT)
    from fantoch_amd import sharding
    from fantoch_amd import streams as fs
    p1 = sharding.rank_params(0, **cfg)
    # conflict-major blocks of the per-rank seed count keep the enumeration identical
    p1.conflict_block = CFG["seeds"]
    planes = fs.synth_host(p1)
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_golden as G
    from oracle import oracle_lib
    order, release, nexec, err = oracle_lib.batch_execute(planes, threads=4)
    chain1, delay1 = G.hists(planes, order, release, nexec)
    assert streams2 == planes.S
    assert np.array_equal(chain2, chain1.astype(np.int64))
    assert np.array_equal(delay2, delay1.astype(np.int64))
    assert chain1.sum() > 0
    # the gathered per-instance rows equal the single run's rows, in global order
    table1 = sharding.instance_summaries(torch.from_numpy(nexec.astype(np.int64)),
                                         torch.from_numpy(err.astype(np.int64)), p1).numpy()
    assert np.array_equal(table2, table1)
    assert list(table1[:, 0]) == list(range(len(table1)))
    assert sorted(set(table1[:, 1])) == sorted(CFG["conflicts"])
    assert np.all(table1[:, 2] == CFG["n"] * CFG["n"] * CFG["cmds"]) and np.all(table1[:, 3] == 0)


def test_instance_summaries_status_and_rates():
    sys.path.insert(0, ROOT)
    from fantoch_amd import sharding
    from fantoch_amd import streams as fs
    p = fs.synth_params(seed=1, instances=4, n=3, cmds=10, conflicts=(0, 100), instance_base=6,
                        conflict_block=2)
    nexec = torch.arange(12, dtype=torch.int64)
    err = torch.zeros(12, dtype=torch.int64)
    err[4], err[5] = 2, 7  # instance 1: first nonzero status of its streams is 2
    rows = sharding.instance_summaries(nexec, err, p).tolist()
    assert rows == [[6, 100, 0 + 1 + 2, 0], [7, 100, 3 + 4 + 5, 2], [8, 0, 6 + 7 + 8, 0],
                    [9, 0, 9 + 10 + 11, 0]]


def test_rank_shards_tile_the_global_enumeration():
    sys.path.insert(0, ROOT)
    from fantoch_amd import sharding
    from fantoch_amd import streams as fs
    a = fs.synth_host(sharding.rank_params(0, **CFG))
    b = fs.synth_host(sharding.rank_params(1, **CFG))
    cfg = dict(CFG)
    cfg["seeds"] = 2 * CFG["seeds"]
    p = sharding.rank_params(0, **cfg)
    p.conflict_block = CFG["seeds"]
    u = fs.synth_host(p)
    for s in range(a.S):
        assert a.stream(s) == u.stream(s)
        assert b.stream(s) == u.stream(a.S + s)
