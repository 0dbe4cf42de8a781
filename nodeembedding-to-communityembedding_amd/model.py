"""Model state (reference: ADSCModel/model.py), with the tables resident in HBM.

Same constructor and attribute names as the reference ``Model`` (model.py:18-140):
``vocab`` (node id -> Vocab with .count/.index/.sample_probability), ``layer1_size``,
``vocab_size``, ``node_embedding``, ``context_embedding``, ``centroid``, ``covariance_mat``,
``inv_covariance_mat``, ``pi``, ``table``, ``k``, ``ground_true``.

Differences, all deliberate:
  * the embedding tables, the GMM buffers and the negative table are torch tensors on the GPU
    (fp32 / uint32-as-int32); ``table_host`` keeps the numpy uint32 table;
  * ``make_table`` runs the exact native builder (come_make_table: same double accumulation,
    same start at node id 1 and the same clamp as model.py:107-121, O(V + T) instead of a Python
    loop over T slots) and packs it on the device (``table_packed``, come_pack_table: the same
    draws from a 16x smaller structure);
  * ``k`` may be given directly (no label file needed), ``device`` selects the GPU;
  * ``save``/``load_model`` use torch.save / torch.load(weights_only=True) (the reference's
    pickle-based load_model, model.py:133-140, is broken and unsafe);
  * ``vocab`` is materialised lazily (a dict of 1M Python objects is only built if asked for);
    the trainers use the vectorised ``rows_of``.
Random draws follow the reference: reset_weights draws node_embedding from the global numpy RNG
with np.random.uniform(-1, 1, (V, d)) (model.py:86); nothing else in the constructor draws.
"""
import logging as log

import numpy as np

from . import _lib
from .embedding import Vocab
from .io_utils import load_ground_true


class Model(object):
    def __init__(self, nodes_degree, size=2, down_sampling=0, seed=1, table_size=100000000,
                 path_labels='data/', input_file=None, k=None, device=None):
        self.down_sampling = down_sampling
        self.seed = seed
        self.table_size = int(table_size)
        if size % 4 != 0:
            log.warning("consider setting layer size to a multiple of 4 for greater performance")
        self.layer1_size = int(size)
        self.device = device
        if nodes_degree is None:
            raise Exception("Model not initialized, need the nodes degree")
        self.build_vocab_(nodes_degree)
        if k is not None:
            self.ground_true, self.k = None, int(k)
        else:
            self.ground_true, self.k = load_ground_true(path=path_labels, file_name=input_file)
        self.reset_weights()
        self.make_table()

    # ---- vocabulary (model.py:52-80) ----
    def build_vocab_(self, vocab):
        """Row index = rank of the node id (sorted ids, model.py:60-64); min id must be 1."""
        if isinstance(vocab, dict):
            ids = np.fromiter(vocab.keys(), np.int64, len(vocab))
            counts = np.fromiter(vocab.values(), np.float64, len(vocab))
        else:  # (ids, counts) arrays
            ids, counts = (np.asarray(vocab[0], np.int64), np.asarray(vocab[1], np.float64))
        order = np.argsort(ids, kind="stable")
        self.node_ids = ids[order]
        self.counts = counts[order]
        assert self.node_ids.min() == 1  # model.py:66
        self.vocab_size = len(self.node_ids)
        self._contiguous = bool(self.node_ids[-1] == self.vocab_size)
        self._vocab = None
        self._hot_cache = {}  # bitmaps depend on the vocabulary and the table
        self.precalc_sampling()

    def precalc_sampling(self):
        """Per-node down-sampling probability (model.py:69-80)."""
        if self.down_sampling:
            total = self.counts.sum()
            thr = float(self.down_sampling) * total
            prob = (np.sqrt(self.counts / thr) + 1) * (thr / self.counts)
            self._sample_prob = np.minimum(prob, 1.0)
        else:
            self._sample_prob = np.ones(self.vocab_size)

    def sample_probability_rows(self):
        return self._sample_prob

    @property
    def vocab(self):
        if self._vocab is None:
            self._vocab = {}
            for i, (nid, c) in enumerate(zip(self.node_ids.tolist(), self.counts.tolist())):
                self._vocab[nid] = Vocab(count=c, index=i, sample_probability=self._sample_prob[i])
        return self._vocab

    def rows_of(self, ids):
        """Node ids -> row indices (int64), -1 for ids not in the vocabulary."""
        ids = np.asarray(ids, np.int64)
        if self._contiguous:
            r = ids - 1
            r[(ids < 1) | (ids > self.vocab_size)] = -1
            return r
        pos = np.searchsorted(self.node_ids, ids)
        pos_c = np.minimum(pos, self.vocab_size - 1)
        return np.where(self.node_ids[pos_c] == ids, pos_c, -1)

    # ---- weights (model.py:83-92) ----
    def _torch_device(self):
        import torch
        if self.device is not None:
            return torch.device(self.device)
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
            else torch.device("cpu")

    def reset_weights(self):
        import torch
        dev = self._torch_device()
        V, d, K = self.vocab_size, self.layer1_size, self.k
        # = np.random.uniform(low=-1, high=1, size=(V, d)).astype(np.float32) (model.py:86): the
        # same draws from the global stream, taken in row blocks so that no V x d float64
        # temporary exists (20 GB at C5's 10M x 256, per rank)
        node = np.empty((V, d), np.float32)
        step = max(1, (1 << 22) // max(1, d))
        for r0 in range(0, V, step):
            r1 = min(V, r0 + step)
            node[r0:r1] = np.random.uniform(low=-1, high=1, size=(r1 - r0, d))
        self.node_embedding = torch.from_numpy(node).to(dev)
        self.context_embedding = torch.zeros((V, d), dtype=torch.float32, device=dev)
        self.centroid = torch.zeros((K, d), dtype=torch.float32, device=dev)
        self.covariance_mat = torch.zeros((K, d, d), dtype=torch.float32, device=dev)
        self.inv_covariance_mat = torch.zeros((K, d, d), dtype=torch.float32, device=dev)
        self.pi = torch.zeros((V, K), dtype=torch.float32, device=dev)

    # ---- negative table (model.py:97-122) ----
    def make_table(self, power=0.75):
        import torch
        log.info("constructing a table with noise distribution from %i words" % self.vocab_size)
        c = np.zeros(self.vocab_size + 1, np.float64)
        c[1:] = self.counts  # indexed by node id when ids are 1..V (model.py:112,119 look up ids)
        if not self._contiguous:
            # the reference looks counts up by node id widx (model.py:112,119); emulate that for
            # sparse ids (a missing id would raise KeyError there; here it counts as 0)
            c = np.zeros(self.vocab_size + 1, np.float64)
            ids = self.node_ids
            m = ids <= self.vocab_size
            c[ids[m]] = self.counts[m]
        table = np.zeros(self.table_size, np.uint32)
        _lib.check(_lib.lib().come_make_table(_lib.ptr(c), self.vocab_size, _lib.ptr(table),
                                             self.table_size, float(power)), "come_make_table")
        self.table_host = table
        self.table = torch.from_numpy(table.view(np.int32)).to(self._torch_device())
        self._hot_cache = {}
        self.table_packed = None
        if self.table.is_cuda:
            from .training_sdg_inner import pack_table
            self.table_packed = pack_table(self.table)

    def hot_rows(self, share=None):
        """Bitmap (CUDA) of the contended rows for Hogwild launches: rows holding at least `share`
        of the negative table (default training_sdg_inner.default_hot_share(layer1_size)) -- see
        come_hot.hip.
        Cached per (share, table buffer, V, T) -- rebuilt after build_vocab_ / make_table; None
        when the tables are not on a GPU or share <= 0 (no contended rows)."""
        from . import training_sdg_inner as tsi
        share = tsi.default_hot_share(self.layer1_size) if share is None else float(share)
        if not getattr(self.table, "is_cuda", False) or share <= 0:
            return None
        cache = self.__dict__.setdefault("_hot_cache", {})
        key = (share, self.table.data_ptr(), int(self.vocab_size), int(self.table.numel()))
        if key not in cache:
            cache[key] = tsi.hot_rows(self.table, self.vocab_size,
                                      max(1, int(share * self.table.numel())))
        return cache[key]

    def negative_table(self):
        """What the trainers pass to the kernels: the exact packed form of the uint32 table
        (come_pack_table: same draws, 16 B per 64 slots -- 25 MB instead of 400 MB at T = 1e8),
        or the plain table when ``use_packed_table`` is False or the table did not pack.  With the
        streaming O2 kernel's non-temporal negative-row loads the packed words stay cached:
        105.7-106.0 vs 108.1 ms per C3 launch (profiles/r03_ab_nt_sites.txt)."""
        if getattr(self, "use_packed_table", True) and \
                getattr(self, "table_packed", None) is not None:
            return self.table_packed
        return self.table

    # ---- persistence ----
    def save(self, path='data', file_name=None):
        """torch.save of the model state; numpy arrays are stored as tensors so that
        load_model can use torch.load(weights_only=True)."""
        import os
        import torch
        os.makedirs(path, exist_ok=True)
        state = {}
        for k, v in self.__dict__.items():
            if k in ("_vocab", "table_packed", "_hot_cache"):
                continue
            if isinstance(v, np.ndarray):
                state["np:" + k] = torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32
                                                    else v)
            elif isinstance(v, torch.Tensor):
                state[k] = v.detach().cpu()
            else:
                state[k] = v
        torch.save(state, os.path.join(path, file_name + '.bin'))

    @staticmethod
    def load_model(path='data', file_name=None, device=None):
        import os
        import torch
        state = torch.load(os.path.join(path, file_name + '.bin'), weights_only=True,
                           map_location="cpu")
        m = Model.__new__(Model)
        for k, v in state.items():
            if k.startswith("np:"):
                arr = v.numpy()
                if k == "np:table_host":
                    arr = arr.view(np.uint32)
                setattr(m, k[3:], arr)
            else:
                setattr(m, k, v)
        m._vocab = None
        if device is not None:
            m.device = device
        dev = m._torch_device()
        for k in ("node_embedding", "context_embedding", "centroid", "covariance_mat",
                  "inv_covariance_mat", "pi", "table"):
            setattr(m, k, getattr(m, k).to(dev))
        m.table_packed = None
        if m.table.is_cuda:
            from .training_sdg_inner import pack_table
            m.table_packed = pack_table(m.table)
        log.info('model loaded, size: %d table_size: %d down_sampling: %.5f communities %d' %
                 (m.layer1_size, m.table_size, m.down_sampling, m.k))
        return m
