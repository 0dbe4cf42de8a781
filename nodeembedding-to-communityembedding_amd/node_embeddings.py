"""O1 (first-order, edges) trainer -- reference: ADSCModel/node_embeddings.py.

``Node2Vec(lr, workers, negative).train(model, edges, chunksize, iter)`` keeps the reference
signature (:19-106): the edge list is repeated ``iter`` times (RepeatCorpusNTimes, :47), every
edge draws its own next_random from the global numpy RNG in edge order (pyx:427), and each edge
trains the pairs (edge[0] -> edge[1]) then (edge[1] -> edge[0]) on node_embedding only
(pyx:444-448).  One launch per pass over the edges (passes stay ordered), one wavefront per edge
(Hogwild across edges) or, with ``deterministic=True``, one wavefront in edge order (== the
reference with workers=1).  ``loss`` reproduces :26-31 (-sum log sigma(u.v) over the edges).
"""
import logging as log
import time

import numpy as np

from . import training_sdg_inner as tsi


class Node2Vec(object):
    def __init__(self, lr=0.2, workers=1, negative=0, deterministic=False):
        self.workers = workers
        self.lr = float(lr)
        self.negative = negative
        self.window_size = 1
        self.deterministic = deterministic

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
        pairs = 0
        for it in range(int(iter)):
            if it > 0 and model.down_sampling:  # every pass draws its own sample (:47)
                rows = self._edge_rows(model, edges)
                ed = torch.from_numpy(rows).to(dev)
            pairs += 2 * int((rows >= 0).all(axis=1).sum())
            seeds = tsi.draw_seeds(rows.shape[0])
            sd = torch.from_numpy(seeds.view(np.int64)).to(dev)
            tsi.sgns_o1(model.node_embedding, ed, sd, self.negative, model.negative_table(),
                        self.lr, mode, hot=hot)
        torch.cuda.synchronize(dev)
        elapsed = time.time() - start
        log.info("O1 training: %i pair updates took %.2fs, %.0f pairs/s", pairs, elapsed,
                 pairs / elapsed if elapsed else 0.0)
        return pairs
