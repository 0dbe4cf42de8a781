"""O2 (context over random walks) trainer -- reference: ADSCModel/context_embeddings.py.

``Context2Vec(lr, window_size, workers, negative).train(model, paths, total_nodes, alpha,
node_count, chunksize)`` keeps the reference signature and semantics (:26-113):
  * returns immediately when alpha <= 0 (:58-59);
  * walks are mapped to rows with OOV nodes dropped (prepare_sentences, utils/embedding.py:126);
  * every walk gets its own next_random from the global numpy RNG, two draws per walk, in walk
    order (pyx:477) -- identical to the reference with workers=1;
  * the learning rate is constant (no decay, :83).
Instead of a producer thread feeding ``workers`` Python threads that each call train_o2 per walk,
walks are uploaded once and trained by ONE launch per batch of ``batch_walks`` walks, one
wavefront per walk (``deterministic=False``: every walk in flight, Hogwild across walks as the
reference's threads are) or one wavefront in walk order (``deterministic=True``: bit-for-bit the
reference's workers=1 order; the parity mode).  ``workers`` and ``chunksize`` are accepted for
signature compatibility.
"""
import logging as log
import time

import numpy as np

from . import training_sdg_inner as tsi
from .embedding import walks_to_rows


class Context2Vec(object):
    def __init__(self, lr=0.1, window_size=5, workers=1, negative=5, deterministic=False,
                 batch_walks=1 << 20):
        self.lr = float(lr)
        self.workers = workers
        self.negative = negative
        self.window_size = int(window_size)
        self.deterministic = deterministic
        self.batch_walks = int(batch_walks)

    def train(self, model, paths, total_nodes, alpha=1.0, node_count=0, chunksize=150):
        """Train the context embedding on ``paths`` (iterable of node-id walks, a [P, L] id
        array, or a CUDA id tensor [P, L] with -1 after each walk's end -- converted and trained
        without leaving the device).  Returns the number of pair updates performed."""
        import torch
        assert model.node_embedding.dtype == torch.float32
        assert model.context_embedding.dtype == torch.float32
        if alpha <= 0.:
            return 0
        if total_nodes is None:
            raise AttributeError('need the number of node')
        start = time.time()
        rows = walks_to_rows(model, paths, max_len=tsi.MAX_SENTENCE_LEN)
        seeds = tsi.draw_seeds(rows.shape[0])
        dev = model.node_embedding.device
        if isinstance(rows, torch.Tensor):  # device walks: count on the device
            lens = (rows >= 0).sum(dim=1).long()
            w_ = self.window_size
            pairs = int(torch.where(lens >= w_ + 1, 2 * w_ * lens - w_ * (w_ + 1),
                                    lens * (lens - 1)).sum())
            n_valid = int(lens.sum())
        else:
            pairs = tsi.count_o2_pairs(rows, self.window_size)
            n_valid = int((rows >= 0).sum())
        mode = tsi.MODE_SEQUENTIAL if self.deterministic else tsi.MODE_HOGWILD
        hot = None if self.deterministic else model.hot_rows()
        for s in range(0, rows.shape[0], self.batch_walks):
            w = rows[s:s + self.batch_walks]
            w = w.contiguous() if isinstance(w, torch.Tensor) else \
                torch.from_numpy(np.ascontiguousarray(w)).to(dev)
            sd = torch.from_numpy(seeds[s:s + self.batch_walks].view(np.int64)).to(dev)
            tsi.sgns_o2(model.node_embedding, model.context_embedding, w, sd, self.window_size,
                        self.negative, model.negative_table(), self.lr, alpha, mode, hot=hot)
        torch.cuda.synchronize(dev)
        elapsed = time.time() - start
        nodes = n_valid + node_count
        log.info("O2 training on %i nodes (%i pair updates) took %.2fs, %.0f pairs/s",
                 nodes, pairs, elapsed, pairs / elapsed if elapsed else 0.0)
        return pairs
