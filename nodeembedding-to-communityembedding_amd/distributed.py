"""Multi-GPU data parallelism for the SGNS path: walk sharding + periodic delta all-reduce.

The reference is one process with Hogwild threads over shared numpy tables; it has
no communication backend.  Across the GPUs of a node the same idea becomes: every rank (one
process per GPU) holds a full replica of node_embedding and context_embedding in HBM, trains its
own contiguous shard of the walks (each walk keeps its own seed, so a walk's negative stream is
identical to the single-GPU run), and every ``sync_every`` batches the ranks exchange what they
changed:

    delta_r = W_r - W_sync          (local progress since the last sync)
    W       = W_sync + sum_r delta_r  (all-reduce SUM over RCCL / xGMI)
    W_sync  = W

Summing deltas keeps every rank's Hogwild progress (plain averaging would shrink each rank's
steps by 1/N).  With N = 1 sync is a no-op.  The all-reduce runs on torch.distributed with the
"nccl" backend (= RCCL on ROCm); tests run the same code on "gloo" with CPU tensors.
"""
import numpy as np


def shard_range(n, rank, world):
    """Contiguous block [lo, hi) of n units for `rank` (sizes differ by at most one)."""
    base, rem = divmod(int(n), int(world))
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard_walks(walks, seeds, rank, world):
    """This rank's contiguous shard of (walks, seeds)."""
    lo, hi = shard_range(len(seeds), rank, world)
    return walks[lo:hi], seeds[lo:hi]


class DeltaAllReduce(object):
    """Delta-sum synchronisation of a list of replicated tables (torch tensors, same shape on
    every rank).  ``bucket_elems`` bounds the size of each all-reduce call (large fp32 buckets:
    xGMI collectives are bandwidth-bound per link, so few big calls beat many small ones)."""

    def __init__(self, tables, group=None, bucket_elems=1 << 26):
        import torch.distributed as dist
        self.tables = list(tables)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.bucket = int(bucket_elems)
        self.snap = [t.clone() for t in self.tables] if self.world > 1 else None

    def sync(self):
        if self.world == 1:
            return
        import torch.distributed as dist
        for t, s in zip(self.tables, self.snap):
            flat_t, flat_s = t.view(-1), s.view(-1)
            for lo in range(0, flat_t.numel(), self.bucket):
                hi = min(lo + self.bucket, flat_t.numel())
                d = flat_t[lo:hi]
                d.sub_(flat_s[lo:hi])                       # delta_r, in place
                dist.all_reduce(d, op=dist.ReduceOp.SUM, group=self.group)
                d.add_(flat_s[lo:hi])                       # W_sync + sum_r delta_r
                flat_s[lo:hi].copy_(d)                      # new W_sync

    def bytes_per_sync(self):
        return sum(t.numel() * t.element_size() for t in self.tables)


def reference_delta_sum(w_sync, locals_):
    """Host restatement of one sync for tests: w_sync + sum_r (w_r - w_sync)."""
    out = np.array(w_sync, np.float64, copy=True)
    for w in locals_:
        out += np.asarray(w, np.float64) - np.asarray(w_sync, np.float64)
    return out
