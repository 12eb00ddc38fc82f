"""Multi-GPU sharding of the batched executor.

Instances are independent (the reference runs them with rayon par_iter,
fantoch/src/bin/simulation.rs), so rank r of W owns the contiguous instance
range [r*I, (r+1)*I) of the global enumeration — no data-path collective.
The only exchange is the exact integer sum of the ChainSize / ExecutionDelay
histograms (Metrics::aggregate -> histogram_merge, fantoch/src/metrics/
histogram.rs:259-326), done with one all-reduce per histogram (RCCL on GPUs,
gloo in the CPU tests), so the merged histograms are bit-identical for any W.
"""
from . import streams as fs


def rank_params(rank, seeds, conflicts, n, cmds, window, cycle_pct, seed, conflict_block=-1,
                horizon=64):
    """Synthetic-stream parameters of rank `rank`: `seeds` x len(conflicts)
    instances starting at global instance rank * that count.  conflict_block
    -1 = conflict-major blocks of `seeds` instances per rate."""
    instances = seeds * len(conflicts)
    block = seeds if conflict_block < 0 else conflict_block
    return fs.synth_params(seed=seed, instances=instances, n=n, cmds=cmds, window=window,
                           cycle_pct=cycle_pct, horizon=horizon, conflicts=tuple(conflicts),
                           instance_base=rank * instances, conflict_block=block)


def allreduce_histograms(dist, *hists):
    """Sums integer histogram tensors over all ranks in place (exact)."""
    for h in hists:
        dist.all_reduce(h)
    return hists


# Per-instance result rows gathered across ranks ("one all-gather
# of fixed-size per-instance summary structs").  The reference collects one
# result per simulated configuration (fantoch/src/bin/simulation.rs, rayon
# par_iter over placements / seeds, results folded on the host); here a row is
# (global instance id, conflict rate %, commands executed over its n processes,
# first nonzero FX_* status of its streams or 0).
SUMMARY_FIELDS = ("instance", "conflict_pct", "executed", "status")


def instance_summaries(nexec, err, params):
    """[instances, 4] int64 rows on nexec's device from the per-stream nexec/err
    of a batch generated with `params` (stream = local * n + process - 1)."""
    import torch
    n = int(params.n)
    inst = int(params.instances)
    dev = nexec.device
    ex = nexec[:inst * n].to(torch.int64).view(inst, n).sum(1)
    e = err[:inst * n].to(torch.int64).view(inst, n)
    nz = e != 0
    first = torch.where(nz.any(1), e.gather(1, nz.to(torch.int64).argmax(1, keepdim=True))[:, 0],
                        torch.zeros_like(ex))
    gid = torch.arange(inst, dtype=torch.int64, device=dev) + int(params.instance_base)
    nc = max(int(params.num_conflicts), 1)
    rates = torch.tensor([int(params.conflict_pct[i]) for i in range(nc)], dtype=torch.int64,
                         device=dev)
    blk = int(params.conflict_block)
    ci = (gid // blk) % nc if blk else gid % nc
    return torch.stack([gid, rates[ci], ex, first], 1)


def gather_summaries(dist, rows, world):
    """all_gather of equal-sized per-rank row blocks -> the global table, in rank order."""
    import torch
    if world <= 1:
        return rows
    parts = [torch.empty_like(rows) for _ in range(world)]
    dist.all_gather(parts, rows.contiguous())
    return torch.cat(parts)
