"""GPU GMM EM (come_amd.gmm) against numpy / sklearn.

* E-step kernel (come_gmm_estep): responsibilities and per-row logsumexp vs the oracle's float64
  restatement of sklearn's _estimate_log_prob (full covariance).
* M-step kernel (come_gmm_scatter): weighted scatter matrices vs float64 numpy, MFMA (d = 64, 128)
  and VALU (other d) paths, ragged chunks.
* EM iterations from fixed initial parameters vs sklearn.mixture.GaussianMixture with the same
  weights_init / means_init / precisions_init (max_iter iterations, tol = 0): the same algorithm in
  fp32 kernels vs sklearn's float64 -- rtol/atol 2e-3 on the fitted parameters.
* a full fit with the GPU k-means init on separated blobs reaches sklearn's lower bound.
The default fit's k-means init is seeded from its own generator; like the reference's unseeded
GaussianMixture, the optimum a fit lands in is not pinned (parity unpinned for the init).
"""
import numpy as np
import pytest

from come_amd import gmm
from oracle import oracle as orc

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


class opts(object):
    """Process-wide launch options set for a block and restored afterwards."""

    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        from come_amd import _lib
        cur = _lib.launch_opts()
        self.old = {k: getattr(cur, k) for k in self.kv}
        for k, v in self.kv.items():
            _lib.set_option(k, v)

    def __exit__(self, *exc):
        from come_amd import _lib
        for k, v in self.old.items():
            _lib.set_option(k, v)


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def problem(V, K, d, seed, sep=3.0):
    rng = np.random.RandomState(seed)
    mu = rng.normal(size=(K, d)) * sep
    A = rng.normal(size=(K, d, d)) / np.sqrt(d)
    cov = np.einsum("kij,klj->kil", A, A) * 0.5 + np.eye(d)[None] * 0.5
    w = rng.dirichlet(np.ones(K) * 3)
    lab = rng.choice(K, V, p=w)
    X = np.empty((V, d))
    for k in range(K):
        m = lab == k
        X[m] = rng.multivariate_normal(mu[k], cov[k], m.sum())
    return X.astype(np.float32), w, mu, cov


@pytest.mark.parametrize("V,K,d", [(1000, 4, 8), (3000, 6, 64), (2500, 5, 128), (777, 3, 100),
                                   (900, 4, 256), (300, 70, 200)])
def test_estep_vs_numpy(V, K, d):
    X, w, mu, cov = problem(V, K, d, V + d)
    pc = orc.precision_cholesky(cov)
    g = gmm.GaussianMixture(K)
    t = lambda a: torch.as_tensor(a, device=dev())  # noqa: E731
    g._w, g._mu, g._pc = t(w), t(mu), t(pc)
    g._prepare_estep()
    resp, lse = gmm.estep(t(X), g._e_pc, g._e_mp, g._e_ln)
    ref_lr = orc.gmm_log_resp(X.astype(np.float64), w, mu, cov)
    np.testing.assert_allclose(resp.cpu().numpy(), np.exp(ref_lr), atol=2e-4)
    # lse: log sum_k w_k N(x; mu_k, S_k), float64 reference
    from scipy.special import logsumexp
    from scipy.stats import multivariate_normal
    lp = np.stack([np.log(w[k]) + multivariate_normal(mu[k], cov[k]).logpdf(X.astype(np.float64))
                   for k in range(K)], 1)
    np.testing.assert_allclose(lse.cpu().numpy(), logsumexp(lp, 1), rtol=2e-5, atol=2e-3)


@pytest.mark.parametrize("d", [64, 128])
@pytest.mark.parametrize("r16", [2, 3])
def test_estep_mixed_factor_shapes(d, r16):
    """The MFMA E-step skips the zero blocks of upper-triangular factors only: components with a
    lower factor (sklearn's cholesky(precisions_init, lower=True)) or a dense factor run the full
    loop.  Mixed in one launch, every component must match the float64 quadratic form -- for the
    bf16-part k_gmm_resp_b16 (gmm_resp16 = 3) and the fp32 k_gmm_resp16t (= 2): a lower or dense
    factor in the launch sends every component to the separate k_gmm_resp16_full launch."""
    V, K = 1500, 6
    rng = np.random.RandomState(d)
    X = rng.standard_normal((V, d)).astype(np.float32)
    mu = (rng.standard_normal((K, d)) * 0.3).astype(np.float32)
    P = []
    for k in range(K):
        A = rng.standard_normal((d, d)) / np.sqrt(d)
        kind = k % 3
        P.append(np.triu(A) + 2 * np.eye(d) if kind == 0 else
                 np.tril(A) + 2 * np.eye(d) if kind == 1 else A + 2 * np.eye(d))
    P = np.stack(P)
    ln = np.log(np.full(K, 1.0 / K))
    mp = np.einsum("kd,kde->ke", mu.astype(np.float64), P)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.float32), device=dev())  # noqa: E731
    with opts(gmm_resp16=r16):
        resp, lse = gmm.estep(t(X), t(P), t(mp), t(ln))
    Y = np.einsum("vd,kde->vke", X.astype(np.float64), P) - mp[None]
    lp = ln[None] - 0.5 * (Y ** 2).sum(-1)
    from scipy.special import logsumexp
    ref_lse = logsumexp(lp, 1)
    np.testing.assert_allclose(resp.cpu().numpy(), np.exp(lp - ref_lse[:, None]), atol=2e-4)
    np.testing.assert_allclose(lse.cpu().numpy(), ref_lse, rtol=2e-5, atol=2e-3)


@pytest.mark.parametrize("V,K,d", [(4097, 50, 128), (70_001, 7, 64), (300, 3, 64), (129, 1, 128),
                                   (1, 4, 128), (5000, 2, 128)])
def test_estep_default_and_fallback_agree(V, K, d):
    """The E-step forms -- k_gmm_resp_b16 (bf16 parts) and k_gmm_resp16t (16-wide fp32 blocks) --
    on sklearn-shaped upper factors, ragged row counts: the same quantities summed in different
    orders, equal to float tolerance, responsibilities summing to 1."""
    rng = np.random.RandomState(V + 7 * K)
    X = rng.standard_normal((V, d)).astype(np.float32)
    P = np.stack([np.triu(rng.standard_normal((d, d)) / np.sqrt(d)) + 2 * np.eye(d)
                  for _ in range(K)])
    mu = rng.standard_normal((K, d)) * 0.3
    mp = np.einsum("kd,kde->ke", mu, P)
    ln = np.log(rng.dirichlet(np.ones(K)))
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.float32), device=dev())  # noqa: E731
    out = {}
    for r16 in (3, 2):
        with opts(gmm_resp16=r16):
            resp, lse = gmm.estep(t(X), t(P), t(mp), t(ln))
        out[r16] = resp.cpu().numpy(), lse.cpu().numpy()
        assert np.isfinite(out[r16][0]).all() and np.abs(out[r16][0].sum(1) - 1).max() < 1e-4
    np.testing.assert_allclose(out[3][0], out[2][0], atol=1e-4)
    np.testing.assert_allclose(out[3][1], out[2][1], rtol=1e-5, atol=1e-3)


def test_variant_options_outside_the_kept_set_are_rejected():
    """The launch options that pick a GMM / community kernel accept only the default (bf16 parts)
    and its one fallback (the fp32-MFMA form; include/come.h); any other value fails the call with COME_E_INVALID instead of
    silently running some other kernel."""
    from come_amd import _lib
    from come_amd import community_embeddings as ce
    d, K, V = 128, 3, 200
    rng = np.random.RandomState(3)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.float32), device=dev())  # noqa: E731
    X = t(rng.standard_normal((V, d)))
    P = t(np.stack([np.eye(d)] * K))
    mp, ln = t(np.zeros((K, d))), t(np.log(np.full(K, 1.0 / K)))
    R = t(rng.dirichlet(np.ones(K), V))
    for bad in (0, 1, 4, 7, 16, 19):
        with opts(gmm_resp16=bad):
            with pytest.raises(_lib.ComeError, match="gmm_resp16"):
                gmm.estep(X, P, mp, ln)
    for bad in (0, 1, 2, 6):
        with opts(gmm_cov_async=bad):
            with pytest.raises(_lib.ComeError, match="gmm_cov_async"):
                gmm.scatter(X, R, mp)
    for bad in (0, 1, 4):
        with opts(community_async=bad):
            with pytest.raises(_lib.ComeError, match="community_async"):
                ce.community_grad(X.clone(), R, mp, P, 0.01, 0.1, 1)


@pytest.mark.parametrize("V,K,d,chunks", [(5000, 3, 64, None), (4097, 5, 128, 7),
                                          (300, 2, 128, 1), (1000, 4, 8, 3), (999, 3, 96, None),
                                          (1500, 3, 256, 4), (200, 2, 330, None)])
@pytest.mark.parametrize("cov", [3, 4])
def test_scatter_vs_numpy(V, K, d, chunks, cov):
    rng = np.random.RandomState(V + K)
    X = rng.normal(size=(V, d)).astype(np.float32)
    R = rng.dirichlet(np.ones(K), V).astype(np.float32)
    M = rng.normal(size=(K, d)).astype(np.float32)
    with opts(gmm_cov_async=cov):
        S = gmm.scatter(torch.as_tensor(X, device=dev()), torch.as_tensor(R, device=dev()),
                        torch.as_tensor(M, device=dev()), chunks=chunks).cpu().numpy()
    X64 = X.astype(np.float64)
    for k in range(K):
        D = X64 - M[k]
        ref = (R[:, k, None] * D).T @ D
        np.testing.assert_allclose(S[k], ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max())


@pytest.mark.parametrize("V,K,d,iters", [(2000, 3, 8, 4), (4000, 5, 64, 3), (3000, 4, 128, 3)])
def test_em_iterations_match_sklearn(V, K, d, iters):
    import warnings
    from sklearn.exceptions import ConvergenceWarning
    from sklearn.mixture import GaussianMixture as SkGMM
    X, w, mu, cov = problem(V, K, d, 7 * V + d, sep=1.5)
    rng = np.random.RandomState(1)
    w0 = np.full(K, 1.0 / K)
    mu0 = mu + rng.normal(size=mu.shape) * 0.5
    prec0 = np.stack([np.linalg.inv(c + np.eye(d) * 0.3) for c in cov])
    kw = dict(n_components=K, covariance_type="full", tol=0.0, reg_covar=1e-5, max_iter=iters,
              weights_init=w0, means_init=mu0, precisions_init=prec0)
    sk = SkGMM(random_state=0, **kw)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", ConvergenceWarning)
        sk.fit(X.astype(np.float64))
    g = gmm.GaussianMixture(random_state=0, **kw).fit(torch.as_tensor(X, device=dev()))
    assert g.n_iter_ == sk.n_iter_ == iters
    np.testing.assert_allclose(g.weights_, sk.weights_, rtol=2e-3, atol=1e-5)
    np.testing.assert_allclose(g.means_, sk.means_, rtol=2e-3, atol=2e-3)
    np.testing.assert_allclose(g.covariances_, sk.covariances_, rtol=2e-3, atol=2e-3)
    np.testing.assert_allclose(g.lower_bound_, sk.lower_bound_, rtol=1e-4)
    pp = g.predict_proba(X).cpu().numpy()
    np.testing.assert_allclose(pp, sk.predict_proba(X.astype(np.float64)), atol=5e-3)


def test_full_fit_kmeans_init_reaches_sklearn_optimum():
    from sklearn.mixture import GaussianMixture as SkGMM
    X, w, mu, cov = problem(20000, 5, 64, 3, sep=4.0)
    g = gmm.GaussianMixture(5, reg_covar=1e-5, n_init=2, random_state=0).fit(X)
    sk = SkGMM(5, covariance_type="full", reg_covar=1e-5, n_init=2, random_state=0).fit(X)
    assert g.converged_
    np.testing.assert_allclose(g.lower_bound_, sk.lower_bound_, rtol=1e-3)
    # same partition up to a relabelling
    a = g.predict(X).cpu().numpy()
    b = sk.predict(X)
    conf = np.zeros((5, 5), np.int64)
    np.add.at(conf, (a, b), 1)
    assert (conf.max(1).sum() / len(a)) > 0.999


def test_community2vec_gpu_fit_sets_model_buffers():
    from come_amd.community_embeddings import Community2Vec
    from come_amd.model import Model
    X, w, mu, cov = problem(3000, 3, 64, 11, sep=4.0)
    np.random.seed(0)
    m = Model((np.arange(1, 3001), np.ones(3000)), size=64, table_size=1000, k=3)
    m.node_embedding.copy_(torch.as_tensor(X, device=m.node_embedding.device))
    c = Community2Vec(m, lr=0.1, reg_covar=1e-5)
    c.fit(m)
    assert m.pi.shape == (3000, 3)
    np.testing.assert_allclose(m.pi.sum(1).cpu().numpy(), 1.0, atol=1e-5)
    inv = m.inv_covariance_mat.cpu().numpy()
    covm = m.covariance_mat.cpu().numpy()
    np.testing.assert_allclose(np.einsum("kij,kjl->kil", inv, covm),
                               np.broadcast_to(np.eye(64), covm.shape), atol=1e-3)


def test_community2vec_distributed_flag_single_process_matches():
    """distributed=True without an initialised process group is the single-GPU path: the row
    shard is every row and no collective runs (tests/test_distributed_c4.py covers world 2)."""
    from come_amd.community_embeddings import Community2Vec
    from come_amd.model import Model
    X, w, mu, cov = problem(2000, 3, 128, 5, sep=4.0)
    outs = []
    for distributed in (False, True):
        np.random.seed(0)
        m = Model((np.arange(1, 2001), np.ones(2000)), size=128, table_size=1000, k=3)
        m.node_embedding.copy_(torch.as_tensor(X, device=m.node_embedding.device))
        c = Community2Vec(m, lr=0.1, reg_covar=1e-5, distributed=distributed)
        np.random.seed(1)
        c.fit(m)
        c.train(np.arange(1, 2001), m, beta=0.1, iter=2)
        outs.append((m.pi.cpu().numpy(), m.node_embedding.cpu().numpy()))
    # (k-means' index_add_ is atomic on the GPU, so fits agree to rounding, not bit for bit)
    np.testing.assert_allclose(outs[0][0], outs[1][0], atol=1e-4)
    np.testing.assert_allclose(outs[0][1], outs[1][1], atol=1e-4)


@pytest.mark.parametrize("V,K,d,chunks", [(4097, 5, 128, 7), (999, 3, 128, None),
                                          (5000, 3, 64, None), (65, 4, 64, 2), (700, 1, 128, 3),
                                          (517, 7, 64, 2), (1031, 9, 64, None)])
def test_scatter_default_and_fallback_agree(V, K, d, chunks):
    """The fp32 k_gmm_cov16 (16x16x4 tiles) and the bf16-part kernels (E^T E, E = sqrt(r) (x - m):
    option 4 = k_gmm_cov_fb3 at d = 128 / k_gmm_cov_bf3 at d = 64, option 5 = k_gmm_cov_bf3; 2
    (d=128) / 4 (d=64) components per workgroup, operands centred and weighted once per block into
    transposed LDS images): equal up to the order and form of the products (atol 1e-5 of the
    matrix scale), symmetric (off-diagonal tiles are stored transposed; inside a diagonal tile
    (w x_a) x_b and (w x_b) x_a round apart, as sklearn's np.dot(resp * diff.T, diff) does).  K
    not a multiple of the components per workgroup included."""
    rng = np.random.RandomState(V + K + d)
    t = lambda a: torch.as_tensor(a, device=dev())  # noqa: E731
    x = t(rng.standard_normal((V, d)).astype(np.float32))
    resp = t(rng.dirichlet(np.ones(K), V).astype(np.float32))
    mu = t(rng.standard_normal((K, d)).astype(np.float32))
    out = []
    for opt in (3, 4, 5):
        with opts(gmm_cov_async=opt):
            out.append(gmm.scatter(x, resp, mu, chunks=chunks).cpu().numpy())
    for o in out[1:]:
        np.testing.assert_allclose(o, out[0], rtol=0, atol=1e-5 * np.abs(out[0]).max())
    for o in out:
        np.testing.assert_allclose(o, np.swapaxes(o, 1, 2), rtol=0, atol=1e-6 * np.abs(o).max())


def test_community2vec_trains_at_d256():
    """A model with layer1_size = 256 (the SGNS kernels' C5 width) goes through the whole
    community phase: GPU GMM fit, responsibilities, community step (wide VALU kernels); the
    sklearn backend too (its predict_proba goes through come_gmm_resp as well)."""
    from come_amd.community_embeddings import Community2Vec
    from come_amd.model import Model
    V, d, K = 1200, 256, 3
    X, w, mu, cov = problem(V, K, d, 5, sep=4.0)
    for backend in ("gpu", "sklearn"):
        np.random.seed(0)
        m = Model((np.arange(1, V + 1), np.full(V, 3)), size=d, table_size=10000, k=K,
                  device=dev())
        m.node_embedding = torch.as_tensor(X, device=dev())
        cm = Community2Vec(m, lr=0.1, reg_covar=1e-5, gmm_backend=backend)
        cm.g_mixture.n_init = 1
        cm.fit(m)
        pi = m.pi.cpu().numpy()
        assert pi.shape == (V, K) and np.allclose(pi.sum(1), 1, atol=1e-4)
        x0 = m.node_embedding.clone()
        cm.train(range(1, V + 1), m, 0.1, iter=2)
        ref = orc.community_train(x0.cpu().numpy(), pi, m.centroid.cpu().numpy(),
                                  m.inv_covariance_mat.cpu().numpy(), 0.1, 0.1, 2)
        np.testing.assert_allclose(m.node_embedding.cpu().numpy(), ref, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("V,K,d", [(4097, 50, 128), (1000, 5, 128), (2049, 9, 64), (300, 3, 64),
                                   (129, 1, 128)])
@pytest.mark.parametrize("r16", [2, 3])
def test_estep_upper_factors_vs_float64(V, K, d, r16):
    """k_gmm_resp_b16 (gmm_resp16 = 3) and k_gmm_resp16t (= 2) with
    sklearn-shaped (upper-triangular) precision factors only -- the launches that take the
    triangular skip -- against the float64 quadratic form, ragged rows."""
    from scipy.special import logsumexp
    rng = np.random.RandomState(V + K)
    X = rng.standard_normal((V, d)).astype(np.float32)
    P = np.stack([np.triu(rng.standard_normal((d, d)) / np.sqrt(d)) + 2 * np.eye(d)
                  for _ in range(K)])
    mu = (rng.standard_normal((K, d)) * 0.3)
    mp = np.einsum("kd,kde->ke", mu, P)
    ln = np.log(rng.dirichlet(np.ones(K)))
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.float32), device=dev())  # noqa: E731
    with opts(gmm_resp16=r16):
        resp, lse = gmm.estep(t(X), t(P), t(mp), t(ln))
    Y = np.einsum("vd,kde->vke", X.astype(np.float64), P.astype(np.float32).astype(np.float64)) \
        - mp.astype(np.float32)[None]
    lp = ln.astype(np.float32)[None] - 0.5 * (Y ** 2).sum(-1)
    ref_lse = logsumexp(lp, 1)
    np.testing.assert_allclose(resp.cpu().numpy(), np.exp(lp - ref_lse[:, None]), atol=2e-4)
    np.testing.assert_allclose(lse.cpu().numpy(), ref_lse, rtol=2e-5, atol=2e-3)


def _torch_params(S, nk, means, weights, reg):
    """The unfused path (GaussianMixture._m_step / _set_params / _prepare_estep): float64 cov,
    torch Cholesky, prec_chol = solve_triangular(L, I).T, the E-step constants."""
    import math
    d = S.shape[-1]
    cov = S / nk[:, None, None]
    cov += reg * torch.eye(d, dtype=torch.float64, device=S.device)
    chol, info = torch.linalg.cholesky_ex(cov)
    eye = torch.eye(d, dtype=torch.float64, device=S.device).expand_as(cov)
    pc = torch.linalg.solve_triangular(chol, eye, upper=False).transpose(-1, -2)
    log_det = torch.log(torch.diagonal(pc, dim1=-2, dim2=-1)).sum(-1)
    e_mp = torch.einsum("kd,kde->ke", means, pc)
    e_ln = torch.log(weights) + log_det - 0.5 * d * math.log(2 * math.pi)
    return cov, pc, e_mp, e_ln, info


@pytest.mark.parametrize("K,d", [(50, 128), (3, 64), (5, 17), (1, 128), (7, 100), (2, 1)])
def test_gmm_params_fused_matches_unfused(K, d):
    """come_gmm_params (one workgroup per component: cov = S / nk + reg I, in-LDS Cholesky,
    prec_chol = L^-T by rows of back substitution, the E-step's constants) against torch's
    Cholesky / triangular solve in float64: cov bit-identical (the same two operations), prec_chol
    and the constants to 1e-10 relative (another summation order), the fp32 copies to one
    rounding.  The scatter inputs are Gram matrices of a few hundred samples (condition numbers
    up to ~1e3)."""
    from come_amd import _lib
    from come_amd._lib import ptr, stream_handle
    dev = torch.device("cuda", 0)
    rng = np.random.RandomState(K * 1000 + d)
    n = 3 * d + 20
    Y = rng.standard_normal((K, n, d)) * rng.uniform(0.5, 2.0, (K, 1, d))
    nk = rng.uniform(50.0, 500.0, K)
    S = np.einsum("kni,knj->kij", Y, Y) * (nk[:, None, None] / n)
    means = rng.standard_normal((K, d))
    weights = rng.dirichlet(np.ones(K))
    reg = 1e-5
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    S_, nk_, mu_, w_ = t(S), t(nk), t(means), t(weights)
    cov = torch.empty((K, d, d), dtype=torch.float64, device=dev)
    pc = torch.empty_like(cov)
    e_pc = torch.empty((K, d, d), dtype=torch.float32, device=dev)
    e_mp = torch.empty((K, d), dtype=torch.float32, device=dev)
    e_ln = torch.empty((K,), dtype=torch.float32, device=dev)
    info = torch.full((K,), -1, dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().come_gmm_params(ptr(S_), ptr(nk_), ptr(mu_), ptr(w_), K, d, reg,
                                          ptr(cov), ptr(pc), ptr(e_pc), ptr(e_mp), ptr(e_ln),
                                          ptr(info), stream_handle(dev)), "come_gmm_params")
    rcov, rpc, remp, reln, rinfo = _torch_params(S_, nk_, mu_, w_, reg)
    assert int(rinfo.abs().sum()) == 0 and info.cpu().numpy().tolist() == [0] * K
    assert torch.equal(cov, rcov)
    assert torch.equal(torch.tril(pc, -1), torch.zeros_like(pc))
    np.testing.assert_allclose(pc.cpu().numpy(), rpc.cpu().numpy(), rtol=1e-10,
                               atol=1e-10 * float(rpc.abs().max()))
    np.testing.assert_allclose(e_pc.cpu().numpy(), rpc.float().cpu().numpy(), rtol=1e-6,
                               atol=1e-6 * float(rpc.abs().max()))
    np.testing.assert_allclose(e_mp.cpu().numpy(), remp.float().cpu().numpy(), rtol=1e-5,
                               atol=1e-5 * float(remp.abs().max()))
    np.testing.assert_allclose(e_ln.cpu().numpy(), reln.float().cpu().numpy(), rtol=1e-6)


def test_gmm_params_reports_a_non_positive_pivot():
    """A component whose covariance is not positive definite (here: a negative eigenvalue past
    reg_covar) sets info[k] = (first bad pivot) + 1 and leaves the others 0; fit() raises
    sklearn's ValueError from it (GaussianMixture._raise_ill_defined)."""
    from come_amd import _lib
    from come_amd._lib import ptr, stream_handle
    dev = torch.device("cuda", 0)
    K, d = 3, 8
    S = np.stack([np.eye(d) * 2.0] * K)
    S[1, 3, 3] = -1.0
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    outs = [torch.empty((K, d, d), dtype=torch.float64, device=dev) for _ in range(2)]
    e_pc = torch.empty((K, d, d), dtype=torch.float32, device=dev)
    e_mp = torch.empty((K, d), dtype=torch.float32, device=dev)
    e_ln = torch.empty((K,), dtype=torch.float32, device=dev)
    info = torch.full((K,), -1, dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().come_gmm_params(ptr(t(S)), ptr(t(np.ones(K))), ptr(t(np.zeros((K, d)))),
                                          ptr(t(np.full(K, 1.0 / K))), K, d, 1e-6, ptr(outs[0]),
                                          ptr(outs[1]), ptr(e_pc), ptr(e_mp), ptr(e_ln),
                                          ptr(info), stream_handle(dev)), "come_gmm_params")
    assert info.cpu().numpy().tolist() == [0, 4, 0]
    with pytest.raises(_lib.ComeError, match="gmm_params"):
        _lib.check(_lib.lib().come_gmm_params(ptr(t(S)), ptr(t(np.ones(K))), ptr(t(np.zeros((K, d)))),
                                              ptr(t(np.ones(K))), K, 129, 1e-6, ptr(outs[0]),
                                              ptr(outs[1]), ptr(e_pc), ptr(e_mp), ptr(e_ln),
                                              ptr(info), stream_handle(dev)), "come_gmm_params")
    # collapsed samples (every row equal, reg_covar 0): zero covariances, sklearn's ValueError
    with pytest.raises(ValueError, match="ill-defined"):
        gmm.GaussianMixture(2, reg_covar=0.0, max_iter=3, init_params="random",
                            random_state=0).fit(torch.as_tensor(np.zeros((40, 8), np.float32) +
                                                                np.arange(8, dtype=np.float32),
                                                                device=dev))
