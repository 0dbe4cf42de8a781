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

Multi-GPU (``distributed=True``): the reference's worker pool (:72-109) becomes one
process per GPU.  Every rank is handed the same corpus, draws the seeds of ALL walks (so the global
numpy RNG advances exactly as in a one-process run and each walk keeps the seed it would have had),
trains its contiguous shard, and after every ``sync_walks`` of its walks the ranks all-reduce
their tables' progress over RCCL (come_amd.distributed.DeltaAllReduce), the exchange of one batch
overlapped with the next batch's launch.  The combine rule is ``touched_mean``: a row changed by
k ranks since the last exchange moves by the mean of their k deltas (model averaging restricted
to the ranks that trained the row, as Spark MLlib's Word2Vec merges partitions).  Summing the
deltas ("sum", the first-order merge) diverges at lr 0.1: within any practical period a row's
trajectory saturates on every rank (hub rows take thousands of updates per rank per period), so
N saturated displacements add up to N times the step (held-out loss 6-100 vs the sequential
oracle's 2.56 at 2-8 ranks).  Averaging is stable and trains to a LOWER held-out
loss than the sequential oracle (less SGD noise, -12..-19%); it is not the reference's trajectory,
which no periodic exchange reproduces at this learning rate: ``combine="pick"`` (each row takes one
rank's delta, blocking exchanges) keeps the reference's noise level but only 1/N of the shared
rows' progress (+0.8% at 2 ranks, +10% at 8).  Distributed training is therefore NOT a parity mode
(INTEGRATION.md).  The exchange starts every replica from rank 0's tables; train() ends with a
blocking exchange, so every replica then holds the same tables.
"""
import logging as log
import time

import numpy as np

from . import training_sdg_inner as tsi
from .embedding import walks_to_rows

# Walks each rank trains between two exchanges in distributed mode (half of a batch_walks launch):
# the held-out loss vs the sequential oracle over 4,194,304 walks is -12..-19% at 131,072 /
# 262,144 / 524,288 walks per rank and 2-8 ranks (profiles/r04_tierc_replicas_c3_4m.json,
# DESIGN.md §6); the longest period makes the fewest exchanges (2 per 1M-walk step).
DEFAULT_SYNC_WALKS = 1 << 19


def o2_pairs(rows, window):
    """Pair updates train_o2 performs on walk rows (numpy [P, L] or a CUDA tensor)."""
    import torch
    if isinstance(rows, torch.Tensor):
        lens = (rows >= 0).sum(dim=1).long()
        return int(torch.where(lens >= window + 1, 2 * window * lens - window * (window + 1),
                               lens * (lens - 1)).sum())
    return tsi.count_o2_pairs(rows, window)


class Context2Vec(object):
    def __init__(self, lr=0.1, window_size=5, workers=1, negative=5, deterministic=False,
                 batch_walks=1 << 20, distributed=False, sync_walks=DEFAULT_SYNC_WALKS,
                 sparse_sync=False, overlap=True, group=None, hot_share=None, launch_opts=None,
                 combine="touched_mean"):
        self.lr = float(lr)
        self.workers = workers
        self.negative = negative
        self.window_size = int(window_size)
        self.deterministic = deterministic
        self.batch_walks = int(batch_walks)
        self.distributed = bool(distributed)
        self.sync_walks = int(sync_walks)
        self.sparse_sync = bool(sparse_sync)
        self.overlap = bool(overlap)
        self.group = group
        self.hot_share = hot_share      # None = training_sdg_inner.default_hot_share(d)
        self.launch_opts = launch_opts  # per-call come_launch_opts fields (A/B runs)
        self.combine = combine          # DeltaAllReduce combine rule
        self._exchanges = {}
        if self.distributed and self.deterministic:
            raise ValueError("distributed=True trains Hogwild shards; deterministic=True is the "
                             "one-wavefront parity mode")

    def world(self):
        from .distributed import world_of
        return world_of(self.group) if self.distributed else (0, 1)

    def exchange(self, model):
        """The delta exchange of this model's two tables (cached per table pair), with the tables
        as they are now as its sync base."""
        from .distributed import DeltaAllReduce, SparseDeltaAllReduce
        key = (id(model.node_embedding), id(model.context_embedding))
        ex = self._exchanges.get(key)
        if ex is None:
            cls = SparseDeltaAllReduce if self.sparse_sync else DeltaAllReduce
            self._exchanges = {key: cls([model.node_embedding, model.context_embedding],
                                        group=self.group, combine=self.combine)}
            return self._exchanges[key]
        ex.reset()
        return ex

    def train(self, model, paths, total_nodes, alpha=1.0, node_count=0, chunksize=150):
        """Train the context embedding on ``paths`` (iterable of node-id walks, a [P, L] id
        array, or a CUDA id tensor [P, L] with -1 after each walk's end -- converted and trained
        without leaving the device).  Returns the number of pair updates performed (by this rank
        in distributed mode)."""
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
        rank, world = self.world()
        n_batches = None
        if world > 1:
            from .distributed import shard_range, shard_walks
            lo, hi = shard_range(rows.shape[0], 0, world)  # rank 0's shard is the largest
            n_batches = max(1, -(-(hi - lo) // self.sync_walks))
            rows, seeds = shard_walks(rows, seeds, rank, world)
        pairs = o2_pairs(rows, self.window_size)
        n_valid = int((rows >= 0).sum())
        self.train_rows(model, rows, seeds, alpha, n_batches=n_batches)
        if model.node_embedding.is_cuda:
            torch.cuda.synchronize(model.node_embedding.device)
        elapsed = time.time() - start
        nodes = n_valid + node_count
        log.info("O2 training on %i nodes (%i pair updates%s) took %.2fs, %.0f pairs/s",
                 nodes, pairs, " on rank %d of %d" % (rank, world) if world > 1 else "",
                 elapsed, pairs / elapsed if elapsed else 0.0)
        return pairs

    def train_rows(self, model, rows, seeds, alpha=1.0, n_batches=None, update_count=None,
                   launch_events=None):
        """The launches (and, distributed, the exchanges) of train() over walk rows already
        mapped: ``rows`` [P, L] int32 (numpy or CUDA, -1 = None), ``seeds`` [P] uint64 (numpy)
        or int64 (CUDA) -- this rank's shard in distributed mode.  ``n_batches``: exchanges to
        make (every rank must make the same number; default ceil(P / sync_walks)).
        ``update_count``: CUDA int64 [1] += applied target-row updates (come_launch_opts);
        ``launch_events``: a list that receives a (start, end) torch.cuda.Event pair recorded
        around every launch on the launch stream.  Asynchronous: nothing waits for the device
        except the exchanges' own collectives."""
        import torch
        dev = model.node_embedding.device
        mode = tsi.MODE_SEQUENTIAL if self.deterministic else tsi.MODE_HOGWILD
        hot = None if self.deterministic else model.hot_rows(self.hot_share)
        table = model.negative_table()
        rank, world = self.world()
        ex = self.exchange(model) if world > 1 else None
        P = rows.shape[0]
        if ex is None:
            batch = self.batch_walks
            n_batches = -(-P // batch)
        else:
            batch = self.sync_walks
            n_batches = n_batches if n_batches is not None else max(1, -(-P // batch))
        stream = torch.cuda.current_stream(dev) if launch_events is not None else None
        for b in range(n_batches):
            w = rows[b * batch:(b + 1) * batch]
            if w.shape[0]:
                w = w.contiguous() if isinstance(w, torch.Tensor) else \
                    torch.from_numpy(np.ascontiguousarray(w, np.int32)).to(dev)
                sd = seeds[b * batch:(b + 1) * batch]
                sd = sd if isinstance(sd, torch.Tensor) else \
                    torch.from_numpy(np.ascontiguousarray(sd, np.uint64).view(np.int64)).to(dev)
                if launch_events is not None:
                    ev = (torch.cuda.Event(enable_timing=True),
                          torch.cuda.Event(enable_timing=True))
                    ev[0].record(stream)
                tsi.sgns_o2(model.node_embedding, model.context_embedding, w, sd,
                            self.window_size, self.negative, table, self.lr, alpha, mode,
                            opts=self.launch_opts, hot=hot, update_count=update_count)
                if launch_events is not None:
                    ev[1].record(stream)
                    launch_events.append(ev)
            if ex is not None:
                if b + 1 < n_batches and self.overlap and getattr(ex, "overlap_safe", True):
                    ex.start()  # runs beside the next batch; finished by the next start()
                else:
                    ex.sync()   # blocking (the last batch: replicas leave train() identical)
