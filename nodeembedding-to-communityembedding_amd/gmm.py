"""Full-covariance Gaussian mixture EM on the GPU -- replaces the reference's
``sklearn.mixture.GaussianMixture(n_components=k, covariance_type='full', n_init=10,
reg_covar=...).fit(X)`` (ADSCModel/community_embeddings.py:18,27).

Same estimator surface as sklearn for the parts the reference uses: constructor arguments
(n_components, covariance_type='full' only, tol, reg_covar, max_iter, n_init, init_params=
'kmeans' | 'random', weights_init, means_init, precisions_init, random_state), ``fit``,
``predict_proba``, ``predict``, ``score``, and the fitted attributes ``weights_``, ``means_``,
``covariances_``, ``precisions_cholesky_``, ``precisions_``, ``converged_``, ``n_iter_``,
``lower_bound_`` (numpy float64, as sklearn returns them).

The EM loop follows sklearn's BaseMixture.fit_predict: for each init, E-step / M-step until the
change of the mean log-likelihood is below ``tol`` (or ``max_iter``), keep the init with the best
lower bound, and finish with one more E-step.  Per iteration the two 2 V K d^2 contractions run
in libcome.so: the E-step (come_gmm_estep: MFMA X P_k, per-row logsumexp, responsibilities) and
the M-step scatter matrices (come_gmm_scatter: MFMA sum_i r_ik (x_i - mu_k)(x_i - mu_k)^T).
The K x d plain GEMM for the means (resp^T X) and the K small Cholesky factorisations (float64)
run through torch on the same device.

Parity: with fixed initial parameters the iterations match sklearn's within fp32 tolerance
(tests/test_gpu_gmm.py).  The default k-means initialisation (k-means++ seeding then Lloyd,
sklearn's KMeans(n_init=1) semantics) draws from its own device generator, so -- like the
reference, whose GaussianMixture is unseeded -- which local optimum a fit reaches is not pinned.

Multi-GPU (``distributed=True``): every rank passes ITS shard of the rows to
``fit``; the E-step stays local and the M-step all-reduces the sufficient statistics over the
process group -- nk and resp^T X (K + K d floats, float64) before the means, then the scatter
matrices (K d^2) -- so every rank holds the same parameters after every iteration, equal to a
single-process fit over the concatenated rows up to the summation order.  The lower bound is an
all-reduced sum, so all ranks take the same convergence decision.  k-means init: k-means++ seeding
on rank 0's shard, centres broadcast, Lloyd iterations with all-reduced centre sums and counts.
"""
import math

import numpy as np

from . import _lib
from ._lib import check, ptr, stream_handle
from .distributed import all_reduce_sum, world_of


def _as_device_x(X, device=None):
    import torch
    if isinstance(X, torch.Tensor):
        t = X.detach()
        if device is not None:
            t = t.to(device)
    else:
        t = torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32))
        t = t.to(device if device is not None else torch.device("cuda",
                                                                 torch.cuda.current_device()))
    if not t.is_cuda:
        raise TypeError("GaussianMixture runs on the GPU: X must be (or move to) a CUDA tensor")
    return t.to(torch.float32).contiguous()


def estep(X, prec_chol, mu_prec, log_norm):
    """(resp [V, K], lse [V]) for device fp32 X and precomputed component parameters."""
    import torch
    V, d = X.shape
    K = prec_chol.shape[0]
    resp = torch.empty((V, K), dtype=torch.float32, device=X.device)
    lse = torch.empty((V,), dtype=torch.float32, device=X.device)
    check(_lib.lib().come_gmm_estep(ptr(X), V, d, ptr(prec_chol), ptr(mu_prec), ptr(log_norm), K,
                                    ptr(resp), ptr(lse), stream_handle(X.device)),
          "come_gmm_estep")
    return resp, lse


def resp_t_x(resp, X, chunks=256):
    """[K, d] float64: resp^T X (the M-step means numerator, sklearn np.dot(resp.T, X)).  The
    product is K x V x d with V >> K, d: one library GEMM runs it as a skinny GEMM (1.87 ms at C4,
    V = 1M, K = 50, d = 128); split over `chunks` row blocks as a batched GEMM with the partials
    summed in float64 it takes 0.17-0.22 ms (round-2 A/B on one MI355X; DESIGN.md §3.3 prices the
    whole nk + means step at 0.44 ms)."""
    import torch
    V, K = resp.shape
    d = X.shape[1]
    n = V // chunks * chunks
    if n == 0:
        return (resp.t() @ X).double()
    r = resp[:n].reshape(chunks, n // chunks, K)
    x = X[:n].reshape(chunks, n // chunks, d)
    part = torch.bmm(r.transpose(1, 2), x).double().sum(0)
    if n < V:
        part = part + (resp[n:].t() @ X[n:]).double()
    return part


def resp_sum(resp, chunks=256):
    """[K] float64: resp.sum(0) as fp32 sums over `chunks` row blocks added in float64 (0.06 vs
    0.27 ms for a float64-accumulating column sum at C4)."""
    import torch
    V, K = resp.shape
    n = V // chunks * chunks
    if n == 0:
        return resp.sum(0, dtype=torch.float64)
    part = resp[:n].reshape(chunks, n // chunks, K).sum(1).double().sum(0)
    if n < V:
        part = part + resp[n:].sum(0, dtype=torch.float64)
    return part


def scatter_chunks(V, K, d, cus):
    """Row chunks of the scatter's grid.  The MFMA kernels (d = 64, 128) run (K / components per
    workgroup) x chunks workgroups, two resident per CU (k_gmm_cov16, k_gmm_cov_fb3; k_gmm_cov_bf3
    holds one, so the same count is twice as many rounds of half the slots): the chunk count makes
    that a whole number of rounds of the 2 x CUs slots, 8 of them (~4k workgroups: enough to even
    out, the partials <= 512 MB).  A ragged last round costs its whole length: at C4 (25 component
    pairs) 163 chunks = 7.96 rounds ran 7.44 ms, 168 (-> 169 used) = 8.25 rounds 7.75 ms
    (profiles/r05_ab_gmm_diag.txt).  Four rounds (81 chunks) ran 0.8% faster with the bf16-part
    kernels but doubles each chunk's fp32 accumulation: their error against float64 then exceeds
    1.5x the fp32 kernel's (test_c4_scatter_bf3_error_is_fp32_level; profiles/
    r07_ab_scatter_fused.txt).  Other widths (the VALU kernel): ~8192 workgroups."""
    cap = max(1, min((128 << 20) // max(1, K * d * d), -(-V // 64)))
    if d not in (64, 128) or cus <= 0:
        return max(1, min(-(-8192 // K), cap))
    groups = -(-K // (2 if d == 128 else 4))
    slots = 2 * cus
    for rounds in range(8, 0, -1):
        c = rounds * slots // groups
        if 1 <= c <= cap:
            return c
    return max(1, min(cap, slots // groups))


def scatter(X, resp, means, chunks=None):
    """[K, d, d] device fp32: sum_i resp[i,k] (x_i - means_k)(x_i - means_k)^T."""
    import torch
    V, d = X.shape
    K = resp.shape[1]
    if chunks is None:
        cus = torch.cuda.get_device_properties(X.device).multi_processor_count
        chunks = scatter_chunks(V, K, d, cus)
    out = torch.empty((K, d, d), dtype=torch.float32, device=X.device)
    scratch = torch.empty((chunks * K * d * d,) if chunks > 1 else (1,), dtype=torch.float32,
                          device=X.device)
    means = means.to(torch.float32).contiguous()
    resp = resp.contiguous()
    check(_lib.lib().come_gmm_scatter(ptr(X), V, d, ptr(resp), ptr(means), K, int(chunks),
                                      ptr(scratch), ptr(out), stream_handle(X.device)),
          "come_gmm_scatter")
    return out


def params(S, nk, means, weights, reg_covar):
    """come_gmm_params on device float64 scatter matrices [K, d, d] (d <= 128), nk [K], means
    [K, d], weights [K]: (cov, prec_chol, e_prec_chol, e_mu_prec, e_log_norm, info), the last
    four the E-step's fp32 inputs and a device int32 [K] Cholesky status (0 = fine)."""
    import torch
    K, d = means.shape
    dev = S.device
    cov = torch.empty((K, d, d), dtype=torch.float64, device=dev)
    pc = torch.empty((K, d, d), dtype=torch.float64, device=dev)
    e_pc = torch.empty((K, d, d), dtype=torch.float32, device=dev)
    e_mp = torch.empty((K, d), dtype=torch.float32, device=dev)
    e_ln = torch.empty((K,), dtype=torch.float32, device=dev)
    info = torch.empty((K,), dtype=torch.int32, device=dev)
    check(_lib.lib().come_gmm_params(ptr(S), ptr(nk), ptr(means), ptr(weights), K, d,
                                     float(reg_covar), ptr(cov), ptr(pc), ptr(e_pc), ptr(e_mp),
                                     ptr(e_ln), ptr(info), stream_handle(dev)),
          "come_gmm_params")
    return cov, pc, e_pc, e_mp, e_ln, info


class GaussianMixture(object):
    def __init__(self, n_components=1, covariance_type='full', tol=1e-3, reg_covar=1e-6,
                 max_iter=100, n_init=1, init_params='kmeans', weights_init=None,
                 means_init=None, precisions_init=None, random_state=None, kmeans_max_iter=300,
                 kmeans_tol=1e-4, device=None, distributed=False, group=None):
        if covariance_type != 'full':
            raise NotImplementedError("only covariance_type='full' (the reference's) is "
                                      "implemented")
        if init_params not in ('kmeans', 'random'):
            raise ValueError("init_params must be 'kmeans' or 'random'")
        self.n_components = int(n_components)
        self.covariance_type = covariance_type
        self.tol = float(tol)
        self.reg_covar = float(reg_covar)
        self.max_iter = int(max_iter)
        self.n_init = int(n_init)
        self.init_params = init_params
        self.weights_init = weights_init
        self.means_init = means_init
        self.precisions_init = precisions_init
        self.random_state = random_state
        self.kmeans_max_iter = int(kmeans_max_iter)
        self.kmeans_tol = float(kmeans_tol)
        self.device = device
        self.distributed = bool(distributed)
        self.group = group

    def _rank_world(self):
        return world_of(self.group) if self.distributed else (0, 1)

    def _prepare_x(self, X):
        return _as_device_x(X, self.device)

    def _global_sum(self, value, device):
        """float64 scalar summed over the ranks (the value itself on one process)."""
        import torch
        if self._rank_world()[1] == 1:
            return float(value)
        t = torch.tensor([float(value)], dtype=torch.float64, device=device)
        all_reduce_sum([t], self.group)
        return float(t[0])

    # ---- parameters -------------------------------------------------------------------------
    def _m_step(self, X, resp):
        """sklearn _estimate_gaussian_parameters (full): nk, means, covariances (+ reg)."""
        import torch
        V, d = X.shape
        world = self._rank_world()[1]
        nk = resp_sum(resp)
        sx = resp_t_x(resp, X)
        if world > 1:
            all_reduce_sum([nk, sx], self.group)
        nk = nk + 10 * np.finfo(np.float64).eps
        means = sx / nk[:, None]
        S = scatter(X, resp, means.float()).double()
        if world > 1:
            all_reduce_sum([S], self.group)
        cov = S / nk[:, None, None]
        cov += self.reg_covar * torch.eye(d, dtype=torch.float64, device=X.device)
        return nk / (self._n_total if world > 1 else V), means, cov

    def _m_step_params(self, X, resp):
        """One M-step and the E-step inputs it implies: _m_step + _set_params with everything
        after the scatter in one launch (come_gmm_params: cov, Cholesky, prec_chol = L^-T and the
        E-step constants in float64, one workgroup per component), for d <= 128.  Returns a
        device int32 [K] info tensor (non-zero: that component's covariance is not positive
        definite) for the caller to check with its next host read -- no sync here."""
        import torch
        V, d = X.shape
        K = resp.shape[1]
        if d > 128:
            self._set_params(*self._m_step(X, resp))
            return torch.zeros(K, dtype=torch.int32, device=X.device)
        world = self._rank_world()[1]
        nk = resp_sum(resp)
        sx = resp_t_x(resp, X)
        if world > 1:
            all_reduce_sum([nk, sx], self.group)
        nk = (nk + 10 * np.finfo(np.float64).eps).contiguous()
        means = (sx / nk[:, None]).contiguous()
        S = scatter(X, resp, means.float()).double()
        if world > 1:
            all_reduce_sum([S], self.group)
        S = S.contiguous()
        weights = (nk / (self._n_total if world > 1 else V)).contiguous()
        cov, pc, e_pc, e_mp, e_ln, info = params(S, nk, means, weights, self.reg_covar)
        self._w, self._mu, self._cov, self._pc = weights, means, cov, pc
        self._e_pc, self._e_mp, self._e_ln = e_pc, e_mp, e_ln
        return info

    @staticmethod
    def _raise_ill_defined():
        raise ValueError("Fitting the mixture model failed because some components have "
                         "ill-defined empirical covariance (for instance caused by "
                         "singleton or collapsed samples). Try to decrease the number of "
                         "components, or increase reg_covar.")

    def _set_params(self, weights, means, cov):
        import torch
        d = means.shape[1]
        chol, info = torch.linalg.cholesky_ex(cov)
        if bool((info != 0).any()):
            raise ValueError("Fitting the mixture model failed because some components have "
                             "ill-defined empirical covariance (for instance caused by "
                             "singleton or collapsed samples). Try to decrease the number of "
                             "components, or increase reg_covar.")
        eye = torch.eye(d, dtype=torch.float64, device=cov.device).expand_as(cov)
        prec_chol = torch.linalg.solve_triangular(chol, eye, upper=False).transpose(-1, -2)
        self._w, self._mu, self._cov, self._pc = weights, means, cov, prec_chol.contiguous()
        self._prepare_estep()

    def _set_params_from_precisions(self, weights, means, precisions):
        import torch
        pchol = torch.linalg.cholesky(precisions)  # sklearn: cholesky of the precision, lower
        self._w, self._mu, self._pc = weights, means, pchol.contiguous()
        self._cov = torch.cholesky_inverse(pchol)
        self._prepare_estep()

    def _prepare_estep(self):
        import torch
        d = self._mu.shape[1]
        log_det = torch.log(torch.diagonal(self._pc, dim1=-2, dim2=-1)).sum(-1)
        self._e_pc = self._pc.float().contiguous()
        self._e_mp = torch.einsum("kd,kde->ke", self._mu, self._pc).float().contiguous()
        self._e_ln = (torch.log(self._w) + log_det - 0.5 * d * math.log(2 * math.pi)).float() \
            .contiguous()

    # ---- initialisation ------------------------------------------------------------------------
    def _generator(self, device):
        import torch
        g = torch.Generator(device=device)
        rs = self.random_state
        if rs is None:
            seed = int(np.random.randint(0, 2 ** 31 - 1))  # like sklearn: the global RNG
        elif isinstance(rs, (int, np.integer)):
            seed = int(rs)
        else:
            seed = int(rs.randint(0, 2 ** 31 - 1))
        if self._rank_world()[1] > 1:  # one stream for the job: rank 0's seed
            import torch.distributed as dist
            t = torch.tensor([seed], dtype=torch.int64, device=device)
            dist.broadcast(t, 0, group=self.group)
            seed = int(t[0])
        g.manual_seed(seed)
        return g

    def _kmeans_labels(self, X, gen):
        """KMeans(n_clusters=K, n_init=1): greedy k-means++ seeding (2 + log K local trials,
        sklearn's _kmeans_plusplus) then Lloyd iterations until the squared centre shift is
        <= tol * mean feature variance."""
        import torch
        V, d = X.shape
        K = self.n_components
        rank, world = self._rank_world()
        xx = (X * X).sum(1)
        if rank == 0:
            C = self._kmeans_plusplus(X, xx, gen)
        else:
            C = torch.empty((K, d), dtype=torch.float32, device=X.device)
        if world > 1:
            import torch.distributed as dist
            dist.broadcast(C, 0, group=self.group)
            s1 = X.sum(0, dtype=torch.float64)
            s2 = (X.double() ** 2).sum(0)
            all_reduce_sum([s1, s2], self.group)
            n = float(self._n_total)
            tol = self.kmeans_tol * float(((s2 - s1 * s1 / n) / n).mean())  # np.var: ddof 0
        else:
            tol = self.kmeans_tol * float(X.var(0, unbiased=False).mean())  # sklearn _tolerance
        labels = None
        for _ in range(self.kmeans_max_iter):
            dist_ = xx[:, None] - 2 * X @ C.t() + (C * C).sum(1)[None]
            labels = torch.argmin(dist_, 1)
            cnt = torch.bincount(labels, minlength=K).float()
            S = torch.zeros((K, d), dtype=torch.float32, device=X.device)
            S.index_add_(0, labels, X)
            if world > 1:
                all_reduce_sum([cnt, S], self.group)
            newC = torch.where(cnt[:, None] > 0, S / cnt.clamp_min(1)[:, None], C)
            shift = float(((newC - C) ** 2).sum())
            C = newC
            if shift <= tol:
                break
        dist_ = xx[:, None] - 2 * X @ C.t() + (C * C).sum(1)[None]
        return torch.argmin(dist_, 1)

    def _kmeans_plusplus(self, X, xx, gen):
        """sklearn's greedy k-means++ seeding on the rows X: [K, d] centres."""
        import torch
        V, d = X.shape
        K = self.n_components
        if V < K:
            raise ValueError("k-means++ seeding needs >= n_components rows on rank 0")
        trials = 2 + int(math.log(K))
        first = torch.randint(0, V, (1,), generator=gen, device=X.device)
        centers = [X[first[0]]]
        closest = (xx - 2 * X @ centers[0] + centers[0].dot(centers[0])).clamp_min(0)
        pot = closest.sum()
        for _ in range(1, K):
            r = torch.rand(trials, generator=gen, device=X.device, dtype=torch.float64) * pot
            cand = torch.searchsorted(torch.cumsum(closest.double(), 0), r).clamp_max(V - 1)
            C = X[cand]
            dist = (xx[:, None] - 2 * X @ C.t() + (C * C).sum(1)[None]).clamp_min(0)
            dist = torch.minimum(dist, closest[:, None])
            pots = dist.sum(0)
            best = int(torch.argmin(pots))
            closest, pot = dist[:, best].contiguous(), pots[best]
            centers.append(C[best])
        return torch.stack(centers)

    def _initialize(self, X, gen):
        import torch
        V, d = X.shape
        K = self.n_components
        if self.init_params == 'kmeans':
            labels = self._kmeans_labels(X, gen)
            resp = torch.zeros((V, K), dtype=torch.float32, device=X.device)
            resp[torch.arange(V, device=X.device), labels] = 1.0
        else:
            resp = torch.rand((V, K), generator=gen, device=X.device)
            resp /= resp.sum(1, keepdim=True)
        w, mu, cov = self._m_step(X, resp)
        dev = X.device
        if self.weights_init is not None:
            w = torch.as_tensor(np.asarray(self.weights_init, np.float64), device=dev)
        if self.means_init is not None:
            mu = torch.as_tensor(np.asarray(self.means_init, np.float64), device=dev)
        if self.precisions_init is not None:
            P = torch.as_tensor(np.asarray(self.precisions_init, np.float64), device=dev)
            self._set_params_from_precisions(w, mu, P)
        else:
            self._set_params(w, mu, cov)

    # ---- EM ------------------------------------------------------------------------------------
    def fit(self, X, y=None):
        self.fit_predict(X)
        return self

    def fit_predict(self, X, y=None):
        import torch
        X = self._prepare_x(X)
        V, d = X.shape
        self._n_total = int(round(self._global_sum(V, X.device)))
        if self._n_total < self.n_components:
            raise ValueError("Expected n_samples >= n_components but got n_components = %d, "
                             "n_samples = %d" % (self.n_components, self._n_total))
        if d > 512 or self.n_components > (4096 if d in (64, 128) or d > 128 else 64):
            raise ValueError("GPU GaussianMixture supports d <= 512 and n_components <= 64 "
                             "(<= 4096 for d = 64, 128 and d > 128)")
        gen = self._generator(X.device)
        best, max_lb = None, -np.inf
        self.converged_ = False
        for _ in range(self.n_init):
            self._initialize(X, gen)
            lb = -np.inf
            converged, n_iter = False, 0
            for n_iter in range(1, self.max_iter + 1):
                prev = lb
                resp, lse = estep(X, self._e_pc, self._e_mp, self._e_ln)
                info = self._m_step_params(X, resp)
                # one host read per iteration: the lower bound and the Cholesky status together
                lb_info = torch.stack([lse.double().sum(), (info != 0).any().double()]).cpu()
                if lb_info[1] != 0:
                    self._raise_ill_defined()
                lb = self._global_sum(float(lb_info[0]), X.device) / self._n_total
                if abs(lb - prev) < self.tol:
                    converged = True
                    break
            if lb > max_lb or max_lb == -np.inf:
                max_lb = lb
                best = (self._w, self._mu, self._cov, self._pc, n_iter, converged)
        self._w, self._mu, self._cov, self._pc, self.n_iter_, self.converged_ = best
        self._prepare_estep()
        self.lower_bound_ = max_lb
        resp, _ = estep(X, self._e_pc, self._e_mp, self._e_ln)
        self._export()
        return torch.argmax(resp, 1)

    def _export(self):
        import torch
        self.weights_ = self._w.cpu().numpy()
        self.means_ = self._mu.cpu().numpy()
        self.covariances_ = self._cov.cpu().numpy()
        self.precisions_cholesky_ = self._pc.cpu().numpy()
        pc = self._pc
        self.precisions_ = torch.matmul(pc, pc.transpose(-1, -2)).cpu().numpy()

    # ---- inference ----------------------------------------------------------------------------
    def predict_proba(self, X):
        X = self._prepare_x(X)
        return estep(X, self._e_pc, self._e_mp, self._e_ln)[0]

    def predict(self, X):
        import torch
        return torch.argmax(self.predict_proba(X), 1)

    def score(self, X, y=None):
        """Mean log-likelihood over all rows (over every rank's shard when distributed)."""
        X = self._prepare_x(X)
        lse = estep(X, self._e_pc, self._e_mp, self._e_ln)[1]
        n = self._global_sum(X.shape[0], X.device)
        return self._global_sum(lse.double().sum(), X.device) / n
