"""Community embedding trainer -- reference: ADSCModel/community_embeddings.py.

``Community2Vec(model, lr, reg_covar, gmm_backend="gpu")``:
  * ``fit(model)`` (:20-37): fits a GaussianMixture(n_components=k, covariance_type='full',
    n_init=10, reg_covar) -- by default the GPU EM of come_amd.gmm (MFMA E-step and M-step
    kernels, k-means init; unseeded like the reference's: the init draws its seed from the global
    numpy RNG), or with ``gmm_backend="sklearn"`` sklearn's own estimator on the host exactly as
    the reference does -- then stores centroid / covariance_mat (fp32 casts) and
    inv_covariance_mat (the inverse of the fp32 covariances, :36) on the GPU, and computes the
    responsibilities pi (:37, predict_proba) on the GPU with come_gmm_resp.
  * ``train(nodes, model, beta, chunksize, iter)`` (:61-78): the full-batch community gradient
    x -= lr * clip((beta/K) sum_k pi_ik inv_cov_k (x_i - mu_k), +-5), ``iter`` times, on the GPU
    (come_community_grad).  Every row's gradient depends only on that row (:65 snapshot), so rows
    outside ``nodes`` are left untouched by gathering/scattering the selected rows.
  * ``responsibilities(model)``: predict_proba of the fitted mixture on the current embedding.

Multi-GPU (``distributed=True``): every rank holds a full replica of
node_embedding (as after the SGNS phase) and owns the contiguous row block
``shard_range(V, rank, N)``.  ``fit`` runs the GMM EM over the ranks' blocks with all-reduced
sufficient statistics (come_amd.gmm, distributed=True) and all-gathers the responsibilities;
``train`` applies the community gradient to the rank's block only (rows are independent, :65) and
all-gathers the updated rows once per call (after all ``iter`` steps), so the replicas agree
bit for bit with a single-GPU run.  No other exchange is needed.
"""
import logging as log

import numpy as np

from . import _lib
from ._lib import check, ptr, stream_handle
from .distributed import all_gather_rows, shard_range, world_of


def gmm_resp(x, prec_chol, mu_prec, log_norm):
    """Responsibilities [V, K] of a full-covariance GMM for rows x [V, d] (CUDA fp32)."""
    import torch
    V, d = x.shape
    K = prec_chol.shape[0]
    out = torch.empty((V, K), dtype=torch.float32, device=x.device)
    rc = _lib.lib().come_gmm_resp(ptr(x), V, d, ptr(prec_chol), ptr(mu_prec), ptr(log_norm), K,
                                  ptr(out), stream_handle(x.device))
    check(rc, "come_gmm_resp")
    return out


def gmm_resp_params(weights, means, precisions_cholesky, device):
    """Host precomputation (float64, then fp32) of what come_gmm_resp consumes: prec_chol,
    mu_k @ prec_chol_k and log w_k + log det(prec_chol_k) - d/2 log(2 pi)."""
    import torch
    pc = np.asarray(precisions_cholesky, np.float64)
    mu = np.asarray(means, np.float64)
    K, d = mu.shape
    mu_prec = np.einsum("kd,kde->ke", mu, pc)
    log_det = np.array([np.sum(np.log(np.diag(pc[k]))) for k in range(K)])
    log_norm = np.log(np.asarray(weights, np.float64)) + log_det - 0.5 * d * np.log(2 * np.pi)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(device)  # noqa: E731
    return t(pc), t(mu_prec), t(log_norm)


def community_grad(x, pi, mu, inv_cov, beta, lr, iters):
    """In-place community gradient steps on all rows of x (CUDA fp32 [V, d])."""
    V, d = x.shape
    K = pi.shape[1]
    rc = _lib.lib().come_community_grad(ptr(x), V, d, ptr(pi), ptr(mu), ptr(inv_cov), K,
                                        float(beta), float(lr), int(iters),
                                        stream_handle(x.device))
    check(rc, "come_community_grad")


class Community2Vec(object):
    def __init__(self, model, lr, reg_covar=0, gmm_backend="gpu", distributed=False,
                 group=None):
        self.lr = lr
        self.gmm_backend = gmm_backend
        self.distributed = bool(distributed)
        self.group = group
        if gmm_backend == "gpu":
            from .gmm import GaussianMixture
            self.g_mixture = GaussianMixture(n_components=model.k, reg_covar=reg_covar,
                                             covariance_type='full', n_init=10,
                                             distributed=distributed, group=group)
        elif gmm_backend == "sklearn":
            if distributed:
                raise ValueError("distributed=True needs gmm_backend='gpu'")
            from sklearn import mixture
            self.g_mixture = mixture.GaussianMixture(n_components=model.k, reg_covar=reg_covar,
                                                     covariance_type='full', n_init=10)
        else:
            raise ValueError("gmm_backend must be 'gpu' or 'sklearn'")

    def _shard(self, V):
        """(lo, hi) rows this rank owns ((0, V) on one process)."""
        rank, world = world_of(self.group) if self.distributed else (0, 1)
        return shard_range(V, rank, world)

    def fit(self, model):
        import torch
        log.info("Fitting: {} communities".format(model.k))
        dev = model.node_embedding.device
        if self.gmm_backend == "gpu":
            lo, hi = self._shard(model.node_embedding.shape[0])
            self.g_mixture.fit(model.node_embedding[lo:hi])
        else:
            self.g_mixture.fit(model.node_embedding.detach().cpu().numpy())
        cov32 = torch.from_numpy(self.g_mixture.covariances_.astype(np.float32)).to(dev)
        model.centroid = torch.from_numpy(self.g_mixture.means_.astype(np.float32)).to(dev)
        model.covariance_mat = cov32
        model.inv_covariance_mat = torch.linalg.inv(cov32).contiguous()  # :36, fp32 inverse
        model.pi = self.responsibilities(model)

    def responsibilities(self, model):
        import torch
        g = self.g_mixture
        x = model.node_embedding
        pc, mp, ln = gmm_resp_params(g.weights_, g.means_, g.precisions_cholesky_, x.device)
        if not self.distributed:
            return gmm_resp(x, pc, mp, ln)
        V = x.shape[0]
        lo, hi = self._shard(V)
        pi = torch.empty((V, pc.shape[0]), dtype=torch.float32, device=x.device)
        pi[lo:hi] = gmm_resp(x[lo:hi], pc, mp, ln)
        return all_gather_rows(pi, self.group)

    def train(self, nodes, model, beta, chunksize=150, iter=1):
        """community_embeddings.py:61-78.  The reference walks `nodes` in chunks of `chunksize`
        and adds each chunk's gradient with grad_input[node_index] += batch (numpy fancy-index
        add: a node listed twice in ONE chunk counts once, a node in m different chunks m
        times), then updates every row.  So row r moves by clip(m_r * coef * G_r) with m_r the
        number of chunks that list it; here m_r scales pi's row (G is linear in it).  Ids outside
        the vocabulary raise KeyError, as model.vocab[x] does."""
        import torch
        ids = np.fromiter((int(n) for n in nodes), np.int64)
        rows = model.rows_of(ids)
        if (rows < 0).any():
            raise KeyError(int(ids[np.argmax(rows < 0)]))
        x = model.node_embedding
        chunksize = max(1, int(chunksize))
        if len(rows) == model.vocab_size and (np.sort(rows) == np.arange(len(rows))).all():
            lo, hi = self._shard(x.shape[0])
            if hi > lo:  # a row block of a C-contiguous table is itself contiguous
                community_grad(x[lo:hi], model.pi[lo:hi], model.centroid,
                               model.inv_covariance_mat, beta, self.lr, iter)
            if self.distributed:
                all_gather_rows(x, self.group)
            return
        # multiplicity: the number of chunks that list the row
        chunk = np.arange(len(rows)) // chunksize
        pairs = np.unique(chunk * np.int64(model.vocab_size) + rows)
        uniq, mult = np.unique(pairs % model.vocab_size, return_counts=True)
        idx = torch.from_numpy(uniq).to(x.device)
        sub = x.index_select(0, idx).contiguous()
        pi = model.pi.index_select(0, idx)
        if (mult > 1).any():
            pi = pi * torch.from_numpy(mult.astype(np.float32)).to(x.device)[:, None]
        pi = pi.contiguous()
        lo, hi = self._shard(len(uniq))
        if hi > lo:
            community_grad(sub[lo:hi], pi[lo:hi], model.centroid, model.inv_covariance_mat, beta,
                           self.lr, iter)
        if self.distributed:
            all_gather_rows(sub, self.group)
        x.index_copy_(0, idx, sub)
