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
