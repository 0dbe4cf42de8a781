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
"""
import logging as log

import numpy as np

from . import _lib
from ._lib import check, ptr, stream_handle


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
    def __init__(self, model, lr, reg_covar=0, gmm_backend="gpu"):
        self.lr = lr
        self.gmm_backend = gmm_backend
        if gmm_backend == "gpu":
            from .gmm import GaussianMixture
            self.g_mixture = GaussianMixture(n_components=model.k, reg_covar=reg_covar,
                                             covariance_type='full', n_init=10)
        elif gmm_backend == "sklearn":
            from sklearn import mixture
            self.g_mixture = mixture.GaussianMixture(n_components=model.k, reg_covar=reg_covar,
                                                     covariance_type='full', n_init=10)
        else:
            raise ValueError("gmm_backend must be 'gpu' or 'sklearn'")

    def fit(self, model):
        import torch
        log.info("Fitting: {} communities".format(model.k))
        dev = model.node_embedding.device
        if self.gmm_backend == "gpu":
            self.g_mixture.fit(model.node_embedding)
        else:
            self.g_mixture.fit(model.node_embedding.detach().cpu().numpy())
        cov32 = torch.from_numpy(self.g_mixture.covariances_.astype(np.float32)).to(dev)
        model.centroid = torch.from_numpy(self.g_mixture.means_.astype(np.float32)).to(dev)
        model.covariance_mat = cov32
        model.inv_covariance_mat = torch.linalg.inv(cov32).contiguous()  # :36, fp32 inverse
        model.pi = self.responsibilities(model)

    def responsibilities(self, model):
        g = self.g_mixture
        pc, mp, ln = gmm_resp_params(g.weights_, g.means_, g.precisions_cholesky_,
                                     model.node_embedding.device)
        return gmm_resp(model.node_embedding, pc, mp, ln)

    def train(self, nodes, model, beta, chunksize=150, iter=1):
        import torch
        rows = model.rows_of(np.fromiter((int(n) for n in nodes), np.int64))
        rows = rows[rows >= 0]
        x = model.node_embedding
        if len(rows) == model.vocab_size and (np.sort(rows) == np.arange(len(rows))).all():
            community_grad(x, model.pi, model.centroid, model.inv_covariance_mat, beta, self.lr,
                           iter)
            return
        idx = torch.from_numpy(np.unique(rows)).to(x.device)
        sub = x.index_select(0, idx).contiguous()
        community_grad(sub, model.pi.index_select(0, idx).contiguous(), model.centroid,
                       model.inv_covariance_mat, beta, self.lr, iter)
        x.index_copy_(0, idx, sub)
