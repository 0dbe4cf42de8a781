"""Python face of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker.  The product package (come_amd) never imports it.

* SGNS O1/O2 and make_table: ctypes over liboracle_come.so (come_oracle.c), a sequential C
  restatement of utils/training_sdg_inner.pyx:105-509 and ADSCModel/model.py:97-122.
* Community gradient: numpy restatement of ADSCModel/community_embeddings.py:61-78 (same fp32
  numpy operations, same order).
* GMM responsibilities: numpy restatement (float64) of what GaussianMixture.predict_proba does
  for covariance_type='full' (sklearn 1.7.2 `_estimate_log_gaussian_prob` +
  `_estimate_weighted_log_prob` + logsumexp normalisation), called by
  community_embeddings.py:37, plus the fp32 np.linalg.inv of :36.
* Device walker: come_oracle_walks.c restates come_random_walks (Philox stream) bit for bit.
* Graph + walks: pure-Python restatement of utils/graph_utils.py -- networkx's add_edges_from /
  nodes / edges / degree order (graph_utils.py:60-69) and build_deepwalk_corpus (:172-185) +
  __random_walk__ (:20-46) driven by CPython's own random.Random (the reference's RNG), for small
  graphs.  Pinned against tests/golden/walks.npz (make_golden_walks.py, produced by the
  reference's graph_utils itself).

Parity pin: tests/test_oracle_golden.py checks every function here against the fixtures that
tests/golden/make_golden.py produced from the reference itself.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle_come.so")
DOT_REF, DOT_WAVE64 = 0, 1

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle_come.so"])


def lib():
    global _lib
    if _lib is None:
        srcs = [os.path.join(HERE, s) for s in ("come_oracle.c", "come_oracle_mt.c",
                                                 "come_oracle_walks.c")]
        if not os.path.exists(LIB) or any(
                os.path.exists(s) and os.path.getmtime(LIB) < os.path.getmtime(s) for s in srcs):
            build()
        L = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        i64, u64, i32, f32, f64 = (ctypes.c_int64, ctypes.c_uint64, ctypes.c_int, ctypes.c_float,
                                   ctypes.c_double)
        L.oracle_exp_table.argtypes = [P]
        L.oracle_lcg_next.argtypes = [u64]
        L.oracle_lcg_next.restype = u64
        L.oracle_sgns_o2.argtypes = [P, P, i32, P, i64, i32, P, i32, i32, P, u64, f32, f32, i32]
        L.oracle_sgns_o2.restype = i64
        L.oracle_sgns_o1.argtypes = [P, i32, P, i64, P, i32, P, u64, f32, i32]
        L.oracle_sgns_o1.restype = i64
        L.oracle_make_table.argtypes = [P, i64, P, u64, f64]
        L.oracle_min_margin.restype = f64
        L.oracle_updates.restype = i64
        L.oracle_sgns_o2_hogwild.argtypes = [P, P, i64, i32, P, i64, i32, P, i32, i32, P, u64,
                                             f32, f32, i32, f64, i64, P]
        L.oracle_sgns_o2_hogwild.restype = i64
        L.oracle_sgns_o1_hogwild.argtypes = [P, i64, i32, P, i64, P, i32, P, u64, f32, i32, f64,
                                             i64, P]
        L.oracle_sgns_o1_hogwild.restype = i64
        L.oracle_philox_walks.argtypes = [P, P, i64, P, i64, i32, f32, u64, i64, P, P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _chk(a, dt):
    assert a.dtype == dt and a.flags.c_contiguous, (a.dtype, dt)
    return a


def exp_table():
    out = np.zeros(1000, np.float32)
    lib().oracle_exp_table(_p(out))
    return out


def lcg_next(s):
    return int(lib().oracle_lcg_next(int(s)))


def reset_margin():
    lib().oracle_reset_margin()


def min_margin():
    return float(lib().oracle_min_margin())


def reset_updates():
    lib().oracle_reset_updates()


def updates():
    """Target-row updates (targets past the +-6 skip) since reset_updates()."""
    return int(lib().oracle_updates())


def sgns_o2(node, ctx, walks, seeds, window, negative, table, lr, alpha, dot_mode=DOT_REF):
    """In-place train_o2 over every walk in order (sequential, workers=1 semantics)."""
    _chk(node, np.float32), _chk(ctx, np.float32), _chk(table, np.uint32)
    walks = np.ascontiguousarray(walks, np.int32)
    seeds = np.ascontiguousarray(seeds, np.uint64)
    assert node.shape == ctx.shape and walks.shape[0] == seeds.shape[0]
    return int(lib().oracle_sgns_o2(_p(node), _p(ctx), node.shape[1], _p(walks), walks.shape[0],
                                    walks.shape[1], _p(seeds), window, negative, _p(table),
                                    table.shape[0], lr, alpha, dot_mode))


def sgns_o1(node, edges, seeds, negative, table, lr, dot_mode=DOT_REF):
    """In-place train_o1 over every edge in order."""
    _chk(node, np.float32), _chk(table, np.uint32)
    edges = np.ascontiguousarray(edges, np.int32).reshape(-1, 2)
    seeds = np.ascontiguousarray(seeds, np.uint64)
    return int(lib().oracle_sgns_o1(_p(node), node.shape[1], _p(edges), edges.shape[0],
                                    _p(seeds), negative, _p(table), table.shape[0], lr, dot_mode))


def sgns_o2_hogwild(node, ctx, walks, seeds, window, negative, table, lr, alpha, threads,
                    max_seconds=0.0, chunk=150):
    """Hogwild train_o2 on `threads` host threads, jobs of `chunk` walks (come_oracle_mt.c,
    context_embeddings.py:72-102, chunksize default 150).  Returns (pair updates, walks)."""
    _chk(node, np.float32), _chk(ctx, np.float32), _chk(table, np.uint32)
    walks = np.ascontiguousarray(walks, np.int32)
    seeds = np.ascontiguousarray(seeds, np.uint64)
    assert node.shape == ctx.shape and walks.shape[0] == seeds.shape[0]
    done = np.zeros(1, np.int64)
    pairs = lib().oracle_sgns_o2_hogwild(_p(node), _p(ctx), node.shape[0], node.shape[1],
                                         _p(walks), walks.shape[0], walks.shape[1], _p(seeds),
                                         window, negative, _p(table), table.shape[0], lr, alpha,
                                         int(threads), float(max_seconds), int(chunk),
                                         _p(done))
    return int(pairs), int(done[0])


def sgns_o1_hogwild(node, edges, seeds, negative, table, lr, threads, max_seconds=0.0,
                    chunk=150):
    """Hogwild train_o1 on `threads` host threads, jobs of `chunk` edges (node_embeddings.py:
    58-95, chunksize default 150).  Returns (pair updates, edges processed)."""
    _chk(node, np.float32), _chk(table, np.uint32)
    edges = np.ascontiguousarray(edges, np.int32).reshape(-1, 2)
    seeds = np.ascontiguousarray(seeds, np.uint64)
    done = np.zeros(1, np.int64)
    pairs = lib().oracle_sgns_o1_hogwild(_p(node), node.shape[0], node.shape[1], _p(edges),
                                         edges.shape[0], _p(seeds), negative, _p(table),
                                         table.shape[0], lr, int(threads), float(max_seconds),
                                         int(chunk), _p(done))
    return int(pairs), int(done[0])


def philox_walks(rowptr, col, starts, path_length, alpha=0.0, seed=0, walk_offset=0, emit=None):
    """The device walker's walks (come_random_walks) restated on the host: [P, L] int32."""
    rowptr = np.ascontiguousarray(rowptr, np.int64)
    col = np.ascontiguousarray(col, np.int32)
    starts = np.ascontiguousarray(starts, np.int32)
    out = np.empty((len(starts), int(path_length)), np.int32)
    em = None if emit is None else np.ascontiguousarray(emit, np.int32)
    lib().oracle_philox_walks(_p(rowptr), _p(col), len(rowptr) - 1, _p(starts), len(starts),
                              int(path_length), float(alpha), int(seed) & (2 ** 64 - 1),
                              int(walk_offset), None if em is None else _p(em), _p(out))
    return out


def usable_cpus():
    """CPUs this process may actually run on: the affinity mask, further limited by a cgroup v2
    CPU quota (the GPU box shows 256 CPUs but grants a 16-CPU quota)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(-(-int(q) // int(per)))))
    except (OSError, ValueError):
        pass
    return n


def make_table(counts_by_row, T, power=0.75):
    """counts_by_row[r] = count of node id r+1 (ids 1..V, model.py:66)."""
    V = len(counts_by_row)
    c = np.zeros(V + 1, np.float64)
    c[1:] = counts_by_row
    out = np.zeros(int(T), np.uint32)
    lib().oracle_make_table(_p(c), V, _p(out), int(T), power)
    return out


def community_train(x, pi, mu, inv, beta, lr, iters, chunksize=150, rows=None):
    """community_embeddings.py:61-78 restated; `rows` = the rows of `nodes` in order (default:
    every vocab entry).  grad[ni] += bg is numpy's fancy-index add, as in the reference."""
    x = x.copy()
    V, K = pi.shape
    idx_all = np.arange(V) if rows is None else np.asarray(rows, np.int64)
    for _ in range(iters):
        grad = np.zeros(x.shape, np.float32)
        for s in range(0, len(idx_all), chunksize):
            ni = idx_all[s:s + chunksize]
            inp = x[ni]
            bg = np.zeros(inp.shape, np.float32)
            for k in range(K):
                diff = np.expand_dims(inp - mu[k], axis=-1)
                m = pi[ni, k].reshape(len(ni), 1, 1) * inv[k]
                bg += np.squeeze(np.matmul(m, diff), axis=-1)
            grad[ni] += bg
        grad *= (beta / K)
        x -= grad.clip(min=-5, max=5) * lr
    return x


def precision_cholesky(cov):
    """sklearn _compute_precision_cholesky('full') in float64."""
    K, d, _ = cov.shape
    out = np.empty((K, d, d))
    for k in range(K):
        c = np.linalg.cholesky(cov[k])
        out[k] = np.linalg.solve(c, np.eye(d)).T  # == solve_triangular(c, I, lower=True).T
    return out


def gmm_log_resp(X, weights, means, cov):
    """log responsibilities (V x K) of a full-covariance GMM, float64."""
    X = np.asarray(X, np.float64)
    pc = precision_cholesky(np.asarray(cov, np.float64))
    K, d = means.shape
    log_det = np.array([np.sum(np.log(np.diag(pc[k]))) for k in range(K)])
    lp = np.empty((X.shape[0], K))
    for k in range(K):
        y = X @ pc[k] - means[k] @ pc[k]
        lp[:, k] = np.sum(np.square(y), axis=1)
    lp = -0.5 * (d * np.log(2 * np.pi) + lp) + log_det + np.log(weights)
    m = lp.max(axis=1, keepdims=True)
    lse = m + np.log(np.exp(lp - m).sum(axis=1, keepdims=True))
    return lp - lse


def gmm_predict_proba(X, weights, means, cov):
    return np.exp(gmm_log_resp(X, weights, means, cov))


# ---- graph_utils (graph_utils.py:20-46, 60-69, 172-185) -------------------------------------
def nx_graph(edges):
    """networkx.Graph().add_edges_from(edges) as plain dicts: {node: {nbr: None}} in insertion
    order (first appearance of a node, first insertion of a neighbour)."""
    adj = {}
    for u, v in edges:
        u, v = int(u), int(v)
        adj.setdefault(u, {})
        adj.setdefault(v, {})
        adj[u][v] = None
        adj[v][u] = None
    return adj


def nx_to_undirected(adj):
    """nx.Graph.to_undirected(): add_edges_from((u, v) for u in adj for v in adj[u]) into a
    fresh graph that already holds every node in order."""
    new = {n: {} for n in adj}
    for u, nbrs in adj.items():
        for v in nbrs:
            new[u][v] = None
            new[v][u] = None
    return new


def nx_edges(adj):
    """np.array(G.edges()) order: nodes in order, neighbours not yet visited."""
    seen, out = set(), []
    for n, nbrs in adj.items():
        for m in nbrs:
            if m not in seen:
                out.append((n, m))
        seen.add(n)
    return out


def nx_degree(adj):
    return [len(nbrs) + (1 if n in nbrs else 0) for n, nbrs in adj.items()]


def deepwalk_corpus(adj, num_paths, path_length, alpha, rand):
    """build_deepwalk_corpus with start=node for every node per pass; returns lists of ids."""
    nodes = list(adj)
    walks = []
    for _ in range(num_paths):
        rand.shuffle(nodes)
        for node in nodes:
            path = [node]
            while len(path) < path_length:
                nb = list(adj[path[-1]])
                if len(nb) > 0:
                    if rand.random() >= alpha:
                        path.append(rand.choice(nb))
                    else:
                        path.append(path[0])
                else:
                    break
            walks.append(path)
    return walks
