"""O1 (first-order, edges) trainer -- reference: ADSCModel/node_embeddings.py.

``Node2Vec(lr, workers, negative).train(model, edges, chunksize, iter)`` keeps the reference
signature (:19-106): the edge list is repeated ``iter`` times (RepeatCorpusNTimes, :47), every
edge draws its own next_random from the global numpy RNG in edge order (pyx:427), and each edge
trains the pairs (edge[0] -> edge[1]) then (edge[1] -> edge[0]) on node_embedding only
(pyx:444-448).  One launch per pass over the edges (passes stay ordered), one wavefront per edge
(Hogwild across edges) or, with ``deterministic=True``, one wavefront in edge order (== the
reference with workers=1).  ``loss`` reproduces :26-31 (-sum log sigma(u.v) over the edges).

Multi-GPU (``distributed=True``): every rank is handed the same edge list, draws
every edge's seed per pass (the global numpy RNG advances as in one process), trains its
contiguous shard of each pass and exchanges its node_embedding progress with the other ranks
after every ``sync_edges`` of its edges and at the end of each pass (DeltaAllReduce over RCCL,
combine rule touched_mean as Context2Vec's; blocking: an O1 pass is ~1 ms at C2).
"""
import logging as log
import time

import numpy as np

from . import training_sdg_inner as tsi


class _SeedUpload(object):
    """Every edge's seed for one pass (training_sdg_inner.draw_seeds: the global numpy RNG, pyx:427)
    drawn straight into one of two pinned host buffers and copied to the device asynchronously, so
    the host draws pass p + 1's seeds while pass p trains (a pageable copy would wait for the
    launch before it).  A buffer is rewritten only after its previous copy has completed."""

    def __init__(self, dev):
        self.dev = dev
        self.bufs = [None, None]
        self.events = [None, None]
        self.k = 0

    def __call__(self, n):
        import torch
        if self.dev.type != "cuda":
            return torch.from_numpy(tsi.draw_seeds(n).view(np.int64))
        i = self.k % 2
        self.k += 1
        if self.bufs[i] is None or self.bufs[i].numel() != n:
            self.bufs[i] = torch.empty(n, dtype=torch.int64, pin_memory=True)
            self.events[i] = None
        if self.events[i] is not None:
            self.events[i].synchronize()
        tsi.draw_seeds(n, out=self.bufs[i].numpy().view(np.uint64))
        d = self.bufs[i].to(self.dev, non_blocking=True)
        self.events[i] = torch.cuda.Event()
        self.events[i].record(torch.cuda.current_stream(self.dev))
        return d


class Node2Vec(object):
    def __init__(self, lr=0.2, workers=1, negative=0, deterministic=False, distributed=False,
                 sync_edges=None, group=None, combine="touched_mean"):
        self.workers = workers
        self.lr = float(lr)
        self.negative = negative
        self.window_size = 1
        self.deterministic = deterministic
        self.distributed = bool(distributed)
        self.sync_edges = None if sync_edges is None else int(sync_edges)
        self.group = group
        self.combine = combine  # as Context2Vec's
        self._exchanges = {}
        if self.distributed and self.deterministic:
            raise ValueError("distributed=True trains Hogwild shards; deterministic=True is the "
                             "one-wavefront parity mode")

    def exchange(self, model):
        """Delta exchange of model.node_embedding (cached), based on the table as it is now."""
        from .distributed import DeltaAllReduce
        key = id(model.node_embedding)
        ex = self._exchanges.get(key)
        if ex is None:
            self._exchanges = {key: DeltaAllReduce([model.node_embedding], group=self.group,
                                                   combine=self.combine)}
            return self._exchanges[key]
        ex.reset()
        return ex

    def _edge_rows(self, model, edges):
        """Edges -> [E, 2] int32 rows as prepare_sentences would pass them to train_o1: OOV
        endpoints dropped and, with down-sampling, each endpoint kept by the reference's draw
        (embedding.py:126-136; the draws are consumed edge by edge, endpoint by endpoint).  An
        edge left with fewer than two endpoints makes the reference read an uninitialised index
        (pyx:433-440, undefined behaviour): such edges are skipped (-1)."""
        e = np.asarray(edges, np.int64).reshape(-1, 2)
        rows = model.rows_of(e.reshape(-1)).reshape(-1, 2)
        if model.down_sampling:
            from .embedding import downsample_rows
            kept = downsample_rows(model, [r[r >= 0] for r in rows])
            rows = np.array([k if len(k) == 2 else (-1, -1) for k in kept],
                            np.int64).reshape(-1, 2)
        bad = (rows < 0).any(axis=1)
        rows[bad] = -1
        return rows.astype(np.int32)

    def loss(self, model, edges):
        import torch
        rows = torch.from_numpy(self._edge_rows(model, edges)).to(model.node_embedding.device)
        rows = rows[(rows >= 0).all(dim=1)].long()
        x = model.node_embedding
        dots = (x[rows[:, 1]] * x[rows[:, 0]]).sum(dim=1).double()
        return float(-torch.nn.functional.logsigmoid(dots).sum())

    def train(self, model, edges, chunksize=150, iter=1):
        import torch
        assert model.node_embedding.dtype == torch.float32
        start = time.time()
        rows = self._edge_rows(model, edges)
        dev = model.node_embedding.device
        ed = torch.from_numpy(rows).to(dev)
        mode = tsi.MODE_SEQUENTIAL if self.deterministic else tsi.MODE_HOGWILD
        hot = None if self.deterministic else model.hot_rows()
        from .distributed import shard_range, world_of
        rank, world = world_of(self.group) if self.distributed else (0, 1)
        ex = self.exchange(model) if world > 1 else None
        pairs = 0
        n_valid = None
        seeds_to = _SeedUpload(dev)
        for it in range(int(iter)):
            if it > 0 and model.down_sampling:  # every pass draws its own sample (:47)
                rows = self._edge_rows(model, edges)
                ed = torch.from_numpy(rows).to(dev)
                n_valid = None
            lo, hi = shard_range(rows.shape[0], rank, world)
            if n_valid is None:
                n_valid = 2 * int((rows[lo:hi] >= 0).all(axis=1).sum())
            pairs += n_valid
            sd = seeds_to(rows.shape[0])
            if ex is None:
                tsi.sgns_o1(model.node_embedding, ed, sd, self.negative, model.negative_table(),
                            self.lr, mode, hot=hot)
                continue
            # every rank makes the same number of exchanges per pass (rank 0's shard is largest)
            per = self.sync_edges or max(1, shard_range(rows.shape[0], 0, world)[1])
            for b in range(max(1, -(-shard_range(rows.shape[0], 0, world)[1] // per))):
                s, e = min(hi, lo + b * per), min(hi, lo + (b + 1) * per)
                if e > s:
                    tsi.sgns_o1(model.node_embedding, ed[s:e], sd[s:e], self.negative,
                                model.negative_table(), self.lr, mode, hot=hot)
                ex.sync()
        if model.node_embedding.is_cuda:
            torch.cuda.synchronize(dev)
        elapsed = time.time() - start
        log.info("O1 training: %i pair updates took %.2fs, %.0f pairs/s", pairs, elapsed,
                 pairs / elapsed if elapsed else 0.0)
        return pairs
