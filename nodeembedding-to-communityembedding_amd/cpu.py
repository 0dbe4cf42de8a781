"""The CPU twins of the hot-path entry points (include/come.h ``come_cpu_*``):
the same computations on host numpy arrays with ``threads`` worker threads, in libcome.so's
plain C++ (csrc/come_cpu.cpp).  For callers without a GPU; the GPU entry points never fall back
to them.

    sgns_o2(node, ctx, walks, seeds, window, negative, table, lr, alpha, mode, threads) -> pairs
    sgns_o1(node, edges, seeds, negative, table, lr, mode, threads)                   -> pairs
    community_grad(x, pi, mu, inv_cov, beta, lr, iters, threads)    (community_embeddings.py:61-78)
    gmm_estep(x, prec_chol, mu_prec, log_norm, threads) -> (resp, lse)  (predict_proba, :37)

Tables are updated in place (float32, C-contiguous, as the reference's numpy arrays).  ``mode``:
MODE_HOGWILD = ``threads`` workers taking jobs of 150 walks / edges with lock-free updates, as the
reference's worker threads (context_embeddings.py:72-102, node_embeddings.py:58-95);
MODE_SEQUENTIAL = walks in order on the calling thread, bit-identical to the GPU's sequential mode.
"""
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import MODE_HOGWILD, MODE_SEQUENTIAL, check, ptr  # noqa: F401


def default_threads():
    """CPUs this process may use (affinity mask)."""
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except AttributeError:
        return os.cpu_count() or 1


def _threads(threads):
    return default_threads() if threads is None else int(threads)


def _arr(a, dtype, name, writable=False):
    if not isinstance(a, np.ndarray) or a.dtype != dtype or not a.flags.c_contiguous:
        raise TypeError("%s must be a C-contiguous numpy %s array" % (name, np.dtype(dtype).name))
    if writable and not a.flags.writeable:
        raise ValueError("%s must be writable (updated in place)" % name)
    return a


def sgns_o2(node, ctx, walks, seeds, window, negative, table, lr, alpha=1.0,
            mode=MODE_HOGWILD, threads=None):
    """train_o2 (pyx:454-509) over walk rows [P, L] int32 (-1 = None) with per-walk seeds
    (uint64 [P]); returns the pair updates performed."""
    _arr(node, np.float32, "node", True)
    _arr(ctx, np.float32, "ctx", True)
    _arr(walks, np.int32, "walks")
    _arr(seeds, np.uint64, "seeds")
    _arr(table, np.uint32, "table")
    assert node.shape == ctx.shape and walks.ndim == 2 and seeds.shape == (walks.shape[0],)
    pairs = ctypes.c_int64(0)
    check(_lib.lib().come_cpu_sgns_o2(
        ptr(node), ptr(ctx), node.shape[0], node.shape[1], ptr(walks), walks.shape[0],
        walks.shape[1], ptr(seeds), int(window), int(negative), ptr(table), len(table),
        float(lr), float(alpha), int(mode), _threads(threads),
        ctypes.byref(pairs)), "come_cpu_sgns_o2")
    return pairs.value


def sgns_o1(node, edges, seeds, negative, table, lr, mode=MODE_HOGWILD, threads=None):
    """train_o1 (pyx:407-450) over edge rows [E, 2] int32 with per-edge seeds (uint64 [E]);
    returns the pair updates performed."""
    _arr(node, np.float32, "node", True)
    _arr(edges, np.int32, "edges")
    _arr(seeds, np.uint64, "seeds")
    _arr(table, np.uint32, "table")
    assert edges.ndim == 2 and edges.shape[1] == 2 and seeds.shape == (edges.shape[0],)
    pairs = ctypes.c_int64(0)
    check(_lib.lib().come_cpu_sgns_o1(
        ptr(node), node.shape[0], node.shape[1], ptr(edges), edges.shape[0], ptr(seeds),
        int(negative), ptr(table), len(table), float(lr), int(mode),
        _threads(threads), ctypes.byref(pairs)), "come_cpu_sgns_o1")
    return pairs.value


def community_grad(x, pi, mu, inv_cov, beta, lr, iters=1, threads=None):
    """Community2Vec.train's update on all rows of x [V, d] in place (community_embeddings.py:
    61-78): x -= lr * clip((beta / K) * sum_k pi[:, k] inv_cov[k] (x - mu[k]), -5, 5), `iters`
    times."""
    _arr(x, np.float32, "x", True)
    for a, n in ((pi, "pi"), (mu, "mu"), (inv_cov, "inv_cov")):
        _arr(a, np.float32, n)
    V, d = x.shape
    K = mu.shape[0]
    assert pi.shape == (V, K) and mu.shape == (K, d) and inv_cov.shape == (K, d, d)
    check(_lib.lib().come_cpu_community_grad(ptr(x), V, d, ptr(pi), ptr(mu), ptr(inv_cov), K,
                                             float(beta), float(lr), int(iters),
                                             _threads(threads)),
          "come_cpu_community_grad")
    return x


def gmm_estep(x, prec_chol, mu_prec, log_norm, threads=None):
    """Responsibilities [V, K] and per-row log-sum-exp [V] of a full-covariance GMM given its
    precision Cholesky factors (as come_gmm_estep: mu_prec[k] = mu_k @ prec_chol[k], log_norm[k] =
    log w_k + log det(prec_chol[k]) - d/2 log(2 pi))."""
    for a, n in ((x, "x"), (prec_chol, "prec_chol"), (mu_prec, "mu_prec"),
                 (log_norm, "log_norm")):
        _arr(a, np.float32, n)
    V, d = x.shape
    K = log_norm.shape[0]
    assert prec_chol.shape == (K, d, d) and mu_prec.shape == (K, d)
    resp = np.empty((V, K), np.float32)
    lse = np.empty(V, np.float32)
    check(_lib.lib().come_cpu_gmm_estep(ptr(x), V, d, ptr(prec_chol), ptr(mu_prec),
                                        ptr(log_norm), K, ptr(resp), ptr(lse),
                                        _threads(threads)), "come_cpu_gmm_estep")
    return resp, lse
