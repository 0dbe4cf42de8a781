"""Host side of the hot path's input: node-id walks -> row indices for the batched kernels.

The reference feeds its per-walk Cython calls through ``utils/embedding.py``: ``prepare_sentences``
(:126-136) maps every node id of a walk to its ``Vocab`` entry, drops ids outside the vocabulary
and, with down-sampling, drops each node with probability 1 - sample_probability;
``chunkize_serial`` / ``RepeatCorpusNTimes`` (:103-124, :147-160) only batch and repeat that
stream for the worker threads.  Here the whole corpus becomes ONE int32 row matrix
(``walks_to_rows``): the same ids dropped, the same random draws in the same order, ragged walks
padded with -1 (train_o2 treats trailing None exactly like a shorter path), and walks already on
the GPU converted without leaving it.  Batching and repetition are the trainers' loops.

``Vocab`` is the record ``Model.vocab`` maps ids to (the reference's count / index /
sample_probability fields).  The pure-Python ``train_sg`` fallback (:10-100) targets an older
API that no current code calls; it is not reproduced.
"""
import numpy as np


class Vocab(object):
    """One vocabulary entry: ``count`` (degree), ``index`` (row), ``sample_probability``."""
    __slots__ = ("count", "index", "sample_probability")

    def __init__(self, count=0, index=-1, sample_probability=1.0):
        self.count = count
        self.index = index
        self.sample_probability = sample_probability

    def __lt__(self, other):
        return self.count < other.count

    def __repr__(self):
        return "Vocab(count=%r, index=%r, sample_probability=%r)" % (
            self.count, self.index, self.sample_probability)


def downsample_rows(model, seqs):
    """Apply the reference's down-sampling draw to row sequences in order: every row whose
    sample_probability is below 1 consumes one np.random.random_sample() and is kept when its
    probability is >= the draw (embedding.py:132-134); rows with probability 1 draw nothing."""
    if not model.down_sampling:
        return seqs
    prob = model.sample_probability_rows()
    out = []
    for r in seqs:
        p = prob[r]
        keep = p >= 1.0
        low = ~keep
        if low.any():
            keep[low] = p[low] >= np.random.random_sample(int(low.sum()))
        out.append(r[keep])
    return out


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
    after a walk's end) is converted on the device and returned as a CUDA int32 tensor; so is a
    host 2-D id array when the model's tables are on the GPU (uploaded, then mapped there), unless
    it needs the host path (OOV ids inside a walk, down-sampling)."""
    if hasattr(paths, "is_cuda") and paths.is_cuda:
        rows = _device_rows(model, paths, max_len)
        if rows is not None:
            return rows
        paths = paths.cpu().numpy()
    if (isinstance(paths, np.ndarray) and paths.ndim == 2 and paths.size and
            not model.down_sampling and paths.dtype.kind in "iu" and
            getattr(getattr(model, "node_embedding", None), "is_cuda", False)):
        # a host id array for a model on the GPU: upload the ids and map them there (1M walks x
        # 80: ~0.1 s instead of 1.3 s of numpy on the host, beside a 0.8 s launch); the host path
        # below remains for OOV ids inside a walk and for down-sampling
        import torch
        ids = paths if paths.dtype in (np.int32, np.int64) else paths.astype(np.int64)
        rows = _device_rows(model, torch.from_numpy(np.ascontiguousarray(ids)).to(
            model.node_embedding.device), max_len)
        if rows is not None:
            return rows
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
    seqs = downsample_rows(model, seqs)
    L = max((len(s) for s in seqs), default=0)
    if max_len is not None:
        L = min(L, max_len)
    out = np.full((len(seqs), L), -1, np.int32)
    for i, s in enumerate(seqs):
        n = min(len(s), L)
        out[i, :n] = s[:n]
    return out
