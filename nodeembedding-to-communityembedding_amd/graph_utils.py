"""Graph loading and random-walk corpora -- reference: ``utils/graph_utils.py``.

Same names, arguments and outputs as the reference module, backed by libcome.so:

  load_adjacencylist(file_, undirected=False, chunksize=10000)          (:72-109)
      -> Graph.  The file is parsed natively (come_read_int_rows) and the graph is built in
         networkx order (come_graph_from_edges): nodes in first appearance, adjacencies in
         insertion order, exactly what nx.Graph().add_edges_from gives the reference (:60-69);
         undirected=True applies to_undirected()'s adjacency reordering (:106-107), which the
         walks depend on.
  build_deepwalk_corpus(G, num_paths, path_length, alpha=0, rand=random.Random(0))  (:172-185)
  build_deepwalk_corpus_iter(...)                                       (:187-192)
      -> the reference's walks, bit for bit: the caller's ``random.Random`` stream is continued
         by the native restatement of CPython's MT19937 / shuffle / choice / random()
         (come_walks_reference) and handed back advanced, as if the reference had consumed it.
  write_walks_to_disk(G, filebase, num_paths, path_length, alpha=0, rand=random.Random(0),
                      num_workers=cpu_count())                          (:122-146)
      -> same files, same per-file seeds (rand.randint(0, 2**31) per file, in file order), same
         split of passes over files; the files' streams run on native threads.
  combine_files_iter(file_list), count_lines(f), count_textfiles(files, workers=1),
  count_words(file), grouper(n, iterable, padvalue=None)               (:149-226)

Added for the GPU path: ``read_walk_files`` (all walk files -> one padded int64 array, natively)
and ``device_walks`` (the HIP walker, come_random_walks: same walk distribution, Philox stream,
walks written straight into HBM as train_o2 rows).

Graph here is the minimal networkx-like object the reference's callers use: ``nodes()``,
``edges()`` (np.array(G.edges()) order), ``degree()`` (dict, a self-loop counts twice),
``neighbors(n)``, ``number_of_nodes()``, ``number_of_edges()``, ``len(G)``, ``to_undirected()``.
"""
import ctypes
import os
import random
from collections import Counter
from itertools import zip_longest
from multiprocessing import cpu_count

import numpy as np

from . import _lib
from ._lib import check, ptr


class Graph(object):
    """Undirected graph in networkx order over node positions 0..V-1 (CSR)."""

    def __init__(self, node_ids, rowptr, col, degree, edge_pos):
        self.node_ids = node_ids      # int64 [V]: list(G.nodes())
        self.rowptr = rowptr          # int64 [V + 1]
        self.col = col                # int32 [nnz]: neighbour positions, insertion order
        self.degree_arr = degree      # int64 [V]: G.degree() values
        self.edge_pos = edge_pos      # int32 [E, 2]: G.edges() as positions
        self._pos = None

    @staticmethod
    def from_edges(edges):
        """nx.Graph().add_edges_from(edges) for an [E, 2] array of node ids (file order)."""
        e = np.ascontiguousarray(np.asarray(edges, np.int64).reshape(-1, 2))
        E = len(e)
        cap = max(2 * E, 1)
        node_ids = np.empty(cap, np.int64)
        rowptr = np.empty(cap + 1, np.int64)
        col = np.empty(cap, np.int32)
        degree = np.empty(cap, np.int64)
        edge_pos = np.empty((cap, 2), np.int32)
        V, Eo = ctypes.c_int64(), ctypes.c_int64()
        check(_lib.lib().come_graph_from_edges(ptr(e), E, ptr(node_ids), ctypes.byref(V),
                                               ptr(rowptr), ptr(col), ptr(degree), ptr(edge_pos),
                                               ctypes.byref(Eo)), "come_graph_from_edges")
        V, Eo = V.value, Eo.value
        return Graph(node_ids[:V].copy(), rowptr[:V + 1].copy(), col[:rowptr[V]].copy(),
                     degree[:V].copy(), edge_pos[:Eo].copy())

    # ---- the networkx surface the reference uses ----
    def nodes(self):
        return self.node_ids.tolist()

    def edges(self):
        return self.node_ids[self.edge_pos]

    def degree(self):
        return dict(zip(self.node_ids.tolist(), self.degree_arr.tolist()))

    def degree_by_id(self):
        return self.node_ids.copy(), self.degree_arr.copy()

    def positions_of(self, ids):
        if self._pos is None:
            order = np.argsort(self.node_ids, kind="stable")
            self._pos = (self.node_ids[order], order)
        sid, order = self._pos
        ids = np.asarray(ids, np.int64)
        p = np.minimum(np.searchsorted(sid, ids), len(sid) - 1)
        if not (sid[p] == ids).all():
            raise KeyError("node id not in graph")
        return order[p]

    def neighbors(self, n):
        p = int(self.positions_of([n])[0])
        return self.node_ids[self.col[self.rowptr[p]:self.rowptr[p + 1]]].tolist()

    def number_of_nodes(self):
        return len(self.node_ids)

    def number_of_edges(self):
        return len(self.edge_pos)

    def __len__(self):
        return len(self.node_ids)

    def to_undirected(self):
        """nx.Graph.to_undirected() (load_adjacencylist(..., undirected=True), :106-107): a copy
        rebuilt by add_edges_from over (u, v) for u in node order, v in adj[u] order.  Node order
        and G.edges() are unchanged, but every adjacency is reordered: first the neighbours that
        precede the node (in node order), then the rest in their old order."""
        V = len(self.node_ids)
        deg = np.diff(self.rowptr)
        row = np.repeat(np.arange(V, dtype=np.int64), deg)
        k = np.arange(len(self.col), dtype=np.int64) - np.repeat(self.rowptr[:-1], deg)
        key = np.where(self.col < row, self.col.astype(np.int64), V + k)
        order = np.lexsort((key, row))
        return Graph(self.node_ids.copy(), self.rowptr.copy(), self.col[order].copy(),
                     self.degree_arr.copy(), self.edge_pos.copy())


def load_adjacencylist(file_, undirected=False, chunksize=10000):
    """graph_utils.load_adjacencylist (:72-109): lines of integer node ids, '#' comments; every
    line is one edge row for add_edges_from (the reference builds an nx.Graph, so the result is
    undirected either way)."""
    rows = read_int_rows(file_)
    if rows.shape[0] and rows.shape[1] != 2:
        raise ValueError("%s: expected 2 node ids per line (got up to %d)" % (file_,
                                                                           rows.shape[1]))
    G = Graph.from_edges(rows)
    return G.to_undirected() if undirected else G


def read_int_rows(path, width=None):
    """All integer lines of a text file as an int64 array [rows, width], -1 padded."""
    L = _lib.lib()
    n, mx = ctypes.c_int64(), ctypes.c_int()
    check(L.come_read_int_rows(path.encode(), None, 0, 0, ctypes.byref(n), ctypes.byref(mx)),
          "come_read_int_rows")
    w = mx.value if width is None else int(width)
    out = np.empty((n.value, max(w, 1)), np.int64)
    n2 = ctypes.c_int64()
    check(L.come_read_int_rows(path.encode(), ptr(out), n.value, max(w, 1), ctypes.byref(n2),
                               ctypes.byref(mx)), "come_read_int_rows")
    return out[:, :w] if w else out[:, :0]


def _states_of(randoms):
    st = np.empty((len(randoms), 625), np.uint32)
    for i, r in enumerate(randoms):
        v, s, _ = r.getstate()
        if v != 3:
            raise ValueError("unsupported random.Random state version %r" % v)
        st[i] = s
    return st


def _put_states(randoms, st):
    for r, s in zip(randoms, st):
        _, _, gauss = r.getstate()
        r.setstate((3, tuple(int(x) for x in s), gauss))


def _corpus(G, paths_per_stream, path_length, alpha, randoms, threads=1, emit=None):
    """Walks of len(randoms) independent streams (positions, or emit[position]), [P, L] int32."""
    V = G.number_of_nodes()
    pps = np.asarray(paths_per_stream, np.int32)
    st = _states_of(randoms)
    out = np.empty((int(pps.sum()) * V, int(path_length)), np.int32)
    em = None if emit is None else np.ascontiguousarray(emit, np.int32)
    check(_lib.lib().come_walks_reference(ptr(G.rowptr), ptr(G.col), V, len(randoms), ptr(pps),
                                          ptr(st), int(path_length), float(alpha),
                                          None if em is None else ptr(em), int(threads),
                                          ptr(out)), "come_walks_reference")
    _put_states(randoms, st)
    return out


def _ids_of(G, walks_pos):
    out = np.full(walks_pos.shape, -1, np.int64)
    m = walks_pos >= 0
    out[m] = G.node_ids[walks_pos[m]]
    return out


def build_deepwalk_corpus(G, num_paths, path_length, alpha=0, rand=random.Random(0)):
    """[num_paths * V, path_length] node ids (-1 after a walk that stopped early)."""
    return _ids_of(G, _corpus(G, [num_paths], path_length, alpha, [rand]))


def build_deepwalk_corpus_iter(G, num_paths, path_length, alpha=0, rand=random.Random(0)):
    for w in build_deepwalk_corpus(G, num_paths, path_length, alpha=alpha, rand=rand):
        yield w[w >= 0].tolist()


def _paths_per_worker(num_paths, num_workers):
    if num_paths <= num_workers:
        return [1 for _ in range(num_paths)]
    return [len([y for y in x if y is not None])
            for x in grouper(int(num_paths / num_workers) + 1, range(1, num_paths + 1))]


def write_walks_to_disk(G, filebase, num_paths, path_length, alpha=0, rand=random.Random(0),
                        num_workers=cpu_count()):
    """Same files as the reference (:122-146): file i holds paths_per_worker[i] passes drawn from
    random.Random(rand.randint(0, 2**31)) (seeds drawn in file order from ``rand``)."""
    files_list = ["{}.{}".format(filebase, str(x)) for x in range(num_paths)]
    ppw = _paths_per_worker(num_paths, num_workers)
    files = files_list[:len(ppw)]
    randoms = [random.Random(rand.randint(0, 2 ** 31)) for _ in files]
    walks = _corpus(G, ppw, path_length, alpha, randoms, threads=max(1, int(num_workers)))
    L = _lib.lib()
    start = 0
    V = G.number_of_nodes()
    for f, p in zip(files, ppw):
        block = _ids_of(G, walks[start:start + p * V])
        start += p * V
        check(L.come_write_int_rows(f.encode(), ptr(block), block.shape[0], block.shape[1], 0),
              "come_write_int_rows")
    return files


def read_walk_files(file_list, max_len=None):
    """Every line of every existing file, in order, as int64 [P, Lmax] node ids (-1 padded)."""
    parts = [read_int_rows(f) for f in file_list if os.path.isfile(f)]
    if not parts:
        return np.zeros((0, 0), np.int64)
    L = max(p.shape[1] for p in parts)
    if max_len is not None:
        L = min(L, int(max_len))
    out = np.full((sum(p.shape[0] for p in parts), L), -1, np.int64)
    r = 0
    for p in parts:
        w = min(L, p.shape[1])
        out[r:r + p.shape[0], :w] = p[:, :w]
        r += p.shape[0]
    return out


def combine_files_iter(file_list):
    for f in file_list:
        if os.path.isfile(f):
            for row in read_int_rows(f):
                yield row[row >= 0]


def count_lines(f):
    if os.path.isfile(f):
        return int(read_int_rows(f).shape[0])
    return 0


def count_words(file):
    rows = read_int_rows(file)
    ids, counts = np.unique(rows[rows >= 0], return_counts=True)
    return Counter(dict(zip(ids.tolist(), counts.tolist())))


def count_textfiles(files, workers=1):
    c = Counter()
    for f in files:
        c.update(count_words(f))
    return c


def grouper(n, iterable, padvalue=None):
    "grouper(3, 'abcdefg', 'x') --> ('a','b','c'), ('d','e','f'), ('g','x','x')"
    return zip_longest(*[iter(iterable)] * n, fillvalue=padvalue)


def device_walks(rowptr, col, starts, path_length, alpha=0.0, seed=0, walk_offset=0,
                 emit=None, out=None):
    """HIP walker (come_random_walks): one walk per entry of ``starts`` (CUDA int32 positions);
    rowptr (CUDA int64 [V+1]) / col (CUDA int32) the CSR; returns CUDA int32 [P, path_length]
    (``emit[position]`` per step if given, else positions; -1 after an early stop)."""
    import torch
    from ._lib import stream_handle
    for t, nm, dt in ((rowptr, "rowptr", torch.int64), (col, "col", torch.int32),
                      (starts, "starts", torch.int32)):
        if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == dt
                and t.is_contiguous()):
            raise TypeError("%s must be a contiguous CUDA %s tensor" % (nm, dt))
    V = rowptr.numel() - 1
    P = starts.numel()
    if emit is not None and (emit.dtype != torch.int32 or not emit.is_cuda or emit.numel() != V):
        raise TypeError("emit must be a CUDA int32 tensor of V entries")
    if out is None:
        out = torch.empty((P, int(path_length)), dtype=torch.int32, device=starts.device)
    elif out.shape != (P, int(path_length)) or out.dtype != torch.int32 or not out.is_contiguous():
        raise ValueError("out must be a contiguous int32 [P, path_length] tensor")
    check(_lib.lib().come_random_walks(ptr(rowptr), ptr(col), V, ptr(starts), P,
                                       int(path_length), float(alpha), int(seed) & (2 ** 64 - 1),
                                       int(walk_offset), None if emit is None else ptr(emit),
                                       ptr(out), stream_handle(starts.device)),
          "come_random_walks")
    return out
