"""Graphs and random walks: the producers of the hot path's input.

Reference counterparts: ``utils/graph_utils.py`` -- ``load_adjacencylist`` (:72-109), the uniform
truncated walk with restart ``__random_walk__`` (:20-46) and ``build_deepwalk_corpus_iter``
(:187-192: per pass, shuffle the node list and start one walk at every node).  Walks here are
generated for whole batches at once on the device from a CSR adjacency (uniform neighbour choice,
restart probability alpha, a walk stops at a node without neighbours; HIP kernel
come_random_walks) -- same distribution as the reference walker, not the same random stream.  The
reference's exact stream (CPython random.Random) is graph_utils.build_deepwalk_corpus.

Synthetic generators for the benchmark configurations: ``chung_lu`` (power-law
expected degrees) and ``sbm`` (stochastic block model).  Node ids are 1..V (row = id - 1).
"""
import numpy as np


class CSRGraph(object):
    """Undirected simple graph in CSR form over rows 0..V-1 (node id = row + 1)."""

    def __init__(self, V, edges_rows):
        self.V = int(V)
        e = np.asarray(edges_rows, np.int64).reshape(-1, 2)
        e = e[e[:, 0] != e[:, 1]]
        a = np.minimum(e[:, 0], e[:, 1])
        b = np.maximum(e[:, 0], e[:, 1])
        key = np.unique(a * V + b)
        a, b = key // V, key % V
        self.edges = np.stack([a, b], axis=1)  # unique undirected edges (rows)
        src = np.concatenate([a, b])
        dst = np.concatenate([b, a])
        order = np.argsort(src, kind="stable")
        self.col = dst[order].astype(np.int32)
        self.degree = np.bincount(src, minlength=V).astype(np.int64)
        self.rowptr = np.zeros(V + 1, np.int64)
        np.cumsum(self.degree, out=self.rowptr[1:])

    @classmethod
    def from_device_pairs(cls, V, u, v):
        """The same graph as CSRGraph(V, stack([u, v], 1)) from 1-D CUDA int64 endpoint tensors,
        with torch's sort / unique on the device (integer operations with the same stable,
        sorted semantics: identical output, seconds instead of minutes at 100M pairs).  Only
        1-D tensors, and gathers in slices of 2^24 indices: on this ROCm build torch's row
        gathers of [1e8, 2] int64 tensors (boolean mask / index_select) return wrong rows
        silently, and fail to launch at 2^27 rows (scripts/bisect_torch_gather.py)."""
        import torch
        g = cls.__new__(cls)
        g.V = V = int(V)
        a = torch.minimum(u, v)
        b = torch.maximum(u, v)
        key = torch.where(u == v, torch.full_like(a, -1), a * V + b)  # self-loops -> -1
        del a, b
        key = torch.unique(key, sorted=True)
        if key.numel() and int(key[0]) < 0:
            key = key[1:]
        a, b = key // V, key % V
        del key
        g.edges = torch.stack([a, b], dim=1).cpu().numpy()
        src = torch.cat([a, b])
        dst = torch.cat([b, a])
        del a, b
        order = torch.sort(src, stable=True).indices
        step = 1 << 24
        g.col = torch.cat([dst[order[i:i + step]] for i in range(0, order.numel(), step)]
                          ).to(torch.int32).cpu().numpy()
        del dst, order
        g.degree = torch.bincount(src, minlength=V).cpu().numpy().astype(np.int64)
        g.rowptr = np.zeros(V + 1, np.int64)
        np.cumsum(g.degree, out=g.rowptr[1:])
        return g

    @property
    def num_edges(self):
        return len(self.edges)

    def degree_by_id(self):
        """(ids, degrees) as Model(nodes_degree=...) accepts (G.degree() of the reference)."""
        return np.arange(1, self.V + 1, dtype=np.int64), self.degree.copy()

    def edge_ids(self):
        """[E, 2] node ids (np.array(G.edges()) of the reference)."""
        return self.edges + 1

    @staticmethod
    def from_adjlist(path):
        """graph_utils.load_adjacencylist (:72-109): lines 'u v1 v2 ...' of node ids, '#'
        comments; returns (graph, ids sorted) with rows = rank of the id."""
        pairs = []
        with open(path) as f:
            for line in f:
                if not line.strip() or line[0] == "#":
                    continue
                t = [int(x) for x in line.split()]
                pairs.extend((t[0], v) for v in t[1:])
        p = np.array(pairs, np.int64).reshape(-1, 2)
        ids = np.unique(p)
        rows = np.searchsorted(ids, p)
        return CSRGraph(len(ids), rows), ids


def chung_lu(V, mean_degree, gamma=2.5, seed=1, device=None):
    """Power-law graph with expected degrees w_i ~ (i+1)^(-1/(gamma-1)) scaled to the mean
    degree; V*mean_degree/2 endpoint pairs drawn independently ~ w, self-loops and duplicates
    removed.  ``device``: run the searches and sorts with torch on that device (same graph)."""
    rng = np.random.default_rng(seed)
    w = (np.arange(V, dtype=np.float64) + 1.0) ** (-1.0 / (gamma - 1.0))
    w *= mean_degree * V / w.sum()
    cw = np.cumsum(w)
    cw /= cw[-1]
    m = int(V * mean_degree / 2)
    if device is not None:
        import torch
        cwt = torch.as_tensor(cw, device=device)
        u = torch.searchsorted(cwt, torch.as_tensor(rng.random(m), device=device), right=True)
        v = torch.searchsorted(cwt, torch.as_tensor(rng.random(m), device=device), right=True)
        perm = torch.as_tensor(rng.permutation(V), device=device)
        return CSRGraph.from_device_pairs(V, perm[torch.clamp(u, max=V - 1)],
                                          perm[torch.clamp(v, max=V - 1)])
    u = np.searchsorted(cw, rng.random(m), side="right")
    v = np.searchsorted(cw, rng.random(m), side="right")
    perm = rng.permutation(V)  # decorrelate degree from node id
    return CSRGraph(V, np.stack([perm[np.minimum(u, V - 1)], perm[np.minimum(v, V - 1)]], 1))


def sbm(blocks, block_size, p_in, p_out, seed=0):
    """Stochastic block model: each intra-block pair with p_in, each inter-block pair with p_out
    (pair counts drawn binomially, pairs sampled uniformly; collisions removed)."""
    rng = np.random.default_rng(seed)
    V = blocks * block_size
    parts = []
    pairs_in = block_size * (block_size - 1) // 2
    for b in range(blocks):
        m = rng.binomial(pairs_in, p_in)
        u = rng.integers(0, block_size, m) + b * block_size
        v = rng.integers(0, block_size, m) + b * block_size
        parts.append(np.stack([u, v], 1))
    pairs_out = V * (V - 1) // 2 - blocks * pairs_in
    m = rng.binomial(pairs_out, p_out)
    u = rng.integers(0, V, m)
    v = rng.integers(0, V, m)
    keep = (u // block_size) != (v // block_size)
    parts.append(np.stack([u[keep], v[keep]], 1))
    return CSRGraph(V, np.concatenate(parts))


def random_walks(g, num_paths, path_length, alpha=0.0, seed=0, device="cuda", starts=None,
                 walk_offset=0):
    """Walks [num_paths * V, path_length] of ROW indices (int32 tensor on `device`), -1 after a
    walk stops.  Per pass the start nodes are a fresh permutation of all nodes (graph_utils.py:
    187-192); the walks themselves come from the HIP walker (come_random_walks: uniform
    neighbour, restart to the first node with probability alpha, Philox stream keyed by seed).
    With ``starts`` given (one walk per entry), ``walk_offset`` is the global index of its first
    walk: a shard [lo, hi) of a corpus generated with starts[lo:hi], walk_offset=lo equals rows
    lo..hi-1 of the whole corpus."""
    import torch
    from .graph_utils import device_walks
    dev = torch.device(device)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    rowptr = torch.from_numpy(g.rowptr).to(dev)
    col = torch.from_numpy(g.col.astype(np.int32)).to(dev)
    if starts is None:
        starts = torch.cat([torch.randperm(g.V, generator=gen, device=dev)
                            for _ in range(num_paths)])
    starts = torch.as_tensor(starts, device=dev).to(torch.int32).contiguous()
    return device_walks(rowptr, col, starts, path_length, alpha=alpha, seed=seed,
                        walk_offset=walk_offset)
