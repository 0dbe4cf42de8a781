"""Corpus helpers of the reference ``utils/embedding.py`` (host side of the hot path).

Same names and behaviour as the reference: ``Vocab`` (:164-175), ``chunkize_serial`` (:103-124),
``prepare_sentences`` (:126-136), ``batch_generator`` (:138-145), ``RepeatCorpusNTimes``
(:147-160).  Added: ``walks_to_rows`` -- the vectorised form of prepare_sentences that the batched
trainers use (node ids -> row indices, OOV dropped, ragged walks padded with -1).

The reference's pure-Python ``train_sg`` fallback (:10-100) targets an older API that no current
code calls; it is not reproduced.
"""
import itertools

import numpy as np


class Vocab(object):
    """A single vocabulary item (utils/embedding.py:164-175)."""

    def __init__(self, **kwargs):
        self.count = 0
        self.__dict__.update(kwargs)

    def __lt__(self, other):
        return self.count < other.count

    def __str__(self):
        vals = ['%s:%r' % (key, self.__dict__[key]) for key in sorted(self.__dict__)
                if not key.startswith('_')]
        return "<" + ', '.join(vals) + ">"


def chunkize_serial(iterable, chunksize, as_numpy=False):
    """Elements of `iterable` in `chunksize`-ed lists; the last may be shorter."""
    it = iter(iterable)
    while True:
        if as_numpy:
            wrapped_chunk = [[np.array(doc) for doc in itertools.islice(it, int(chunksize))]]
        else:
            wrapped_chunk = [list(itertools.islice(it, int(chunksize)))]
        if not wrapped_chunk[0]:
            break
        yield wrapped_chunk.pop()


def prepare_sentences(model, paths):
    """Node ids -> Vocab objects, dropping OOV nodes and applying the down-sampling draw
    (utils/embedding.py:126-136)."""
    for path in paths:
        sampled = [model.vocab[node] for node in path
                   if node in model.vocab and (model.vocab[node].sample_probability >= 1.0 or
                                               model.vocab[node].sample_probability >=
                                               np.random.random_sample())]
        yield sampled


def batch_generator(iterable, batch_size=1):
    args = [iterable] * batch_size
    return itertools.zip_longest(*args, fillvalue=None)


class RepeatCorpusNTimes():
    def __init__(self, corpus, n):
        self.corpus = corpus
        self.n = n

    def __iter__(self):
        for _ in range(self.n):
            for document in self.corpus:
                yield document


def _device_rows(model, ids, max_len):
    """CUDA id tensor [P, L] -> CUDA int32 rows, or None when the host path is needed (OOV ids
    inside a walk must be dropped and the walk compacted; down-sampling draws on the host)."""
    import torch
    if model.down_sampling or ids.dim() != 2:
        return None
    ids = ids.long()
    if model._contiguous:
        rows = torch.where((ids >= 1) & (ids <= model.vocab_size), ids - 1,
                           torch.full_like(ids, -1))
    else:
        nid = torch.from_numpy(model.node_ids).to(ids.device)
        pos = torch.searchsorted(nid, ids).clamp_max(model.vocab_size - 1)
        rows = torch.where(nid[pos] == ids, pos, torch.full_like(ids, -1))
    if bool(((rows < 0) & (ids >= 0)).any()):
        return None  # OOV inside a walk
    valid = rows >= 0
    # trailing padding only (a valid entry after a -1 would need compaction)
    if ids.shape[1] > 1 and bool((valid[:, 1:] & ~valid[:, :-1]).any()):
        return None
    if max_len is not None and rows.shape[1] > max_len:
        rows = rows[:, :max_len]
    return rows.to(torch.int32).contiguous()


def walks_to_rows(model, paths, max_len=None):
    """Vectorised prepare_sentences for the batched kernels.

    paths: a 2-D integer array of node ids [P, L] or any iterable of id sequences.
    Returns an int32 array [P, Lmax] of row indices, OOV ids dropped (as prepare_sentences does),
    ragged rows padded with -1 (train_o2 treats trailing None exactly like a shorter path).
    Down-sampling (model.down_sampling > 0) draws one np.random.random_sample per in-vocabulary
    node whose sample_probability < 1, walk by walk, node by node.
    A CUDA tensor of node ids (e.g. come_amd.graph_utils.device_walks output mapped to ids, -1
    after a walk's end) is converted on the device and returned as a CUDA int32 tensor."""
    if hasattr(paths, "is_cuda") and paths.is_cuda:
        rows = _device_rows(model, paths, max_len)
        if rows is not None:
            return rows
        paths = paths.cpu().numpy()
    if isinstance(paths, np.ndarray) and paths.ndim == 2:
        rows = model.rows_of(paths.reshape(-1)).reshape(paths.shape)
        if not model.down_sampling and (rows >= 0).all():
            return rows.astype(np.int32, copy=False)
        seqs = [r[r >= 0] for r in rows]
    else:
        seqs = []
        for path in paths:
            r = model.rows_of(np.asarray(path, np.int64).reshape(-1))
            seqs.append(r[r >= 0])
    if model.down_sampling:
        prob = model.sample_probability_rows()
        kept = []
        for r in seqs:
            p = prob[r]
            keep = p >= 1.0
            low = ~keep
            if low.any():
                keep[low] = p[low] >= np.random.random_sample(int(low.sum()))
            kept.append(r[keep])
        seqs = kept
    L = max((len(s) for s in seqs), default=0)
    if max_len is not None:
        L = min(L, max_len)
    out = np.full((len(seqs), L), -1, np.int32)
    for i, s in enumerate(seqs):
        n = min(len(s), L)
        out[i, :n] = s[:n]
    return out
