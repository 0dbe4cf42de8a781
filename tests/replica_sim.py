"""N ranks of the multi-GPU SGNS path simulated in ONE process on one GPU (TEST INFRASTRUCTURE).

Rank r holds its own replica of both tables and trains its contiguous shard of the walks
(distributed.shard_walks) with the product's Hogwild launch (hot-row bitmap, packed table), one
launch per ``sync_walks`` walks, exactly as Context2Vec.train_rows does on each rank; after each
launch the ranks exchange through the product's DeltaAllReduce -- the same fused HIP passes
(come_delta_begin / come_delta_end, come_delta_flags), the same combine rule (default: the
trainers' touched_mean) and the same overlapped start / finish protocol -- with the RCCL
all-reduce replaced by distributed.LocalReplicas (a SUM over the replicas in rank order).
The last exchange is blocking, so every replica ends equal (as after Context2Vec.train).
"""
import numpy as np
import torch

import come_amd.training_sdg_inner as tsi
from come_amd.distributed import DeltaAllReduce, LocalReplicas, shard_walks


def train_replicas(node0, ctx0, walks, seeds, world, sync_walks, window, negative, table, hot,
                   lr, alpha=1.0, overlap=True, device="cuda", combine="touched_mean",
                   mean_rows=None, pick_rows=None, stats=None):
    """Returns (node, ctx) CUDA tensors of replica 0 after the run (all replicas are equal).
    ``stats``: a dict that receives the number of exchanges each rank made."""
    dev = torch.device(device)
    group = LocalReplicas(world)
    reps, exs, shards = [], [], []
    for r in range(world):
        n_ = torch.from_numpy(np.ascontiguousarray(node0)).to(dev)
        c_ = torch.from_numpy(np.ascontiguousarray(ctx0)).to(dev)
        reps.append((n_, c_))
        exs.append(DeltaAllReduce([n_, c_], comm=group.comm(r), combine=combine,
                                  mean_rows=None if mean_rows is None else [mean_rows] * 2,
                                  pick_rows=None if pick_rows is None else [pick_rows] * 2))
        w, s = shard_walks(walks, seeds, r, world)
        shards.append((torch.from_numpy(np.ascontiguousarray(w, np.int32)).to(dev),
                       torch.from_numpy(np.ascontiguousarray(s, np.uint64).view(np.int64))
                       .to(dev)))
    n_batches = max(1, -(-max(w.shape[0] for w, _ in shards) // sync_walks))
    for b in range(n_batches):
        last = b + 1 == n_batches
        for r in range(world):
            w, s = shards[r]
            wb, sb = w[b * sync_walks:(b + 1) * sync_walks], s[b * sync_walks:(b + 1) * sync_walks]
            if wb.shape[0]:
                tsi.sgns_o2(reps[r][0], reps[r][1], wb.contiguous(), sb.contiguous(), window,
                            negative, table, lr, alpha, tsi.MODE_HOGWILD, hot=hot)
        # every rank posts its flag collectives before any rank waits on them (a blocking
        # wait inside one rank's start() could not complete in a sequential simulation)
        for e in exs:
            e.prepare()         # finishes the previous exchange, snapshots this one's delta
        for e in exs:
            e.start()           # launches this exchange (overlapped: finished by the next one)
        if overlap and not last and exs[0].overlap_safe:  # (as Context2Vec.train_rows)
            continue
        for e in exs:           # blocking exchange = start / finish / settle on every rank
            e.finish()
            e.settle()
    torch.cuda.synchronize(dev)
    for r in range(1, world):
        assert torch.equal(reps[r][0], reps[0][0]) and torch.equal(reps[r][1], reps[0][1])
    if stats is not None:
        stats["exchanges"] = exs[0].exchanges
    return reps[0]


def train_replicas_o1(node0, edges, seeds_per_pass, world, sync_edges, negative, table, hot, lr,
                      device="cuda", combine="pick", stats=None):
    """N ranks of Node2Vec(distributed=True).train (node_embeddings.py) in one process: every pass
    each rank trains its contiguous shard of the edge list (distributed.shard_range) in launches
    of ``sync_edges`` edges (None = the whole shard), each followed by the trainer's blocking
    exchange of node_embedding (DeltaAllReduce, RCCL replaced by LocalReplicas).
    seeds_per_pass: list of uint64 [E] arrays, one per pass (every rank draws every edge's seed).
    Returns the node table (a CUDA tensor; all replicas equal)."""
    from come_amd.distributed import shard_range
    dev = torch.device(device)
    group = LocalReplicas(world)
    reps, exs = [], []
    for r in range(world):
        n_ = torch.from_numpy(np.ascontiguousarray(node0)).to(dev)
        reps.append(n_)
        exs.append(DeltaAllReduce([n_], comm=group.comm(r), combine=combine))
    ed = torch.from_numpy(np.ascontiguousarray(edges, np.int32)).to(dev)
    E = ed.shape[0]
    for seeds in seeds_per_pass:
        sd = torch.from_numpy(np.ascontiguousarray(seeds, np.uint64).view(np.int64)).to(dev)
        biggest = shard_range(E, 0, world)[1]
        per = sync_edges or max(1, biggest)
        for b in range(max(1, -(-biggest // per))):
            for r in range(world):
                lo, hi = shard_range(E, r, world)
                s, e = min(hi, lo + b * per), min(hi, lo + (b + 1) * per)
                if e > s:
                    tsi.sgns_o1(reps[r], ed[s:e], sd[s:e], negative, table, lr, tsi.MODE_HOGWILD,
                                hot=hot)
            for x in exs:       # Node2Vec's exchange is blocking (ex.sync())
                x.prepare()
            for x in exs:
                x.start()
            for x in exs:
                x.finish()
                x.settle()
    torch.cuda.synchronize(dev)
    for r in range(1, world):
        assert torch.equal(reps[r], reps[0])
    if stats is not None:
        stats["exchanges"] = exs[0].exchanges
    return reps[0]
