"""configs[3]/C4 at its own size: K = 50 communities, d = 128, the community
gradient and the GMM responsibilities at V = 1M rows (checked on sampled rows against float64
numpy), the EM M-step scatter and whole EM iterations at V = 100k (every row enters the sums)
against float64 numpy and sklearn.  Reference: ADSCModel/community_embeddings.py:27,36-37,61-78.

Tolerances: the kernels are fp32 MFMA contractions (2 V K d^2 flops in another order) against
float64: rtol 1e-4 on the community update, 2e-4 abs on responsibilities, 1e-4 of the matrix
scale on scatter matrices, sklearn's EM within 2e-3 (as tests/test_gpu_gmm.py)."""
import numpy as np
import pytest
import torch

from come_amd import community_embeddings as ce
from come_amd import gmm
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
K, D = 50, 128


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(DEV)


def params(seed, sep=1.0):
    rng = np.random.RandomState(seed)
    mu = rng.normal(size=(K, D)) * sep
    A = rng.normal(size=(K, D, D)) / np.sqrt(D)
    cov = np.einsum("kij,klj->kil", A, A) * 0.5 + np.eye(D)[None] * 0.5
    w = rng.dirichlet(np.ones(K) * 3)
    return w, mu, cov


@pytest.fixture(scope="module")
def c4_rows():
    """C4's inputs: 1M x 128 N(0, 1) node embeddings (seed 2), pi a
    row-normalised Dirichlet(1) (seed 3), K = 50 components."""
    x = np.random.RandomState(2).standard_normal((1_000_000, D)).astype(np.float32)
    pi = np.random.RandomState(3).dirichlet(np.ones(K), x.shape[0]).astype(np.float32)
    return x, pi


@pytest.mark.parametrize("iters,kern", [(1, 2), (2, 2), (1, 3), (2, 3)])
def test_c4_community_grad_k50_1m(c4_rows, iters, kern):
    """x -= lr clip((beta/K) sum_k pi_ik inv_k (x_i - mu_k), +-5) (:61-78) on all 1M rows; 4,000
    sampled rows (incl. the first and last row tile) against float64, `iters` rounds;
    community_async 2 (fp32 16x16x4 MFMAs) and 3 (fp32 operands as bf16 parts), one tolerance."""
    from come_amd import _lib
    x0, pi = c4_rows
    w, mu, cov = params(4)
    inv = np.linalg.inv(cov.astype(np.float32)).astype(np.float32)  # :36, fp32 inverse
    beta, lr = 2.0 * K, 0.1  # beta/K = 2: some entries reach the +-5 clip
    x = t(x0)
    prev = _lib.launch_opts().community_async
    _lib.set_option("community_async", kern)
    try:
        ce.community_grad(x, t(pi), t(mu), t(inv), beta, lr, iters)
    finally:
        _lib.set_option("community_async", prev)
    got = x.cpu().numpy()
    rng = np.random.RandomState(5)
    rows = np.concatenate([np.arange(64), rng.choice(len(x0), 3872, replace=False),
                           np.arange(len(x0) - 64, len(x0))])
    ref = x0[rows].astype(np.float64)
    mu64, inv64, p64 = mu.astype(np.float32).astype(np.float64), inv.astype(np.float64), \
        pi[rows].astype(np.float64)
    clipped = 0
    for _ in range(iters):
        G = np.zeros_like(ref)
        for k in range(K):
            G += p64[:, k:k + 1] * ((ref - mu64[k]) @ inv64[k].T)  # pi_ik inv_k (x_i - mu_k)
        G *= beta / K
        clipped += int((np.abs(G) >= 5).sum())
        ref = ref - np.clip(G, -5, 5) * lr
    assert clipped > 0
    step = ref - x0[rows]
    np.testing.assert_allclose(got[rows] - x0[rows], step, rtol=1e-4,
                               atol=1e-5 * np.abs(step).max())
    assert np.isfinite(got).all()


def test_c4_community_bf3_error_is_fp32_level(c4_rows):
    """k_community_b16 carries each fp32 operand as three bf16 parts and sums six exact part
    products per multiply-add (|dropped terms| < 2^-26 |a b|): a product more accurate than one
    fp32 rounding, so its error against float64 must be that of the fp32-MFMA kernel
    (k_community16), not a reduced-precision one.  Unclipped update (beta/K = 0.5, lr = 1) on
    200k rows, all of them against float64: RMS and max error within 1.5x of k_community16's."""
    from come_amd import _lib
    x0, pi = c4_rows[0][:200_000], c4_rows[1][:200_000]
    w, mu, cov = params(4)
    inv = np.linalg.inv(cov.astype(np.float32)).astype(np.float32)
    beta, lr = 0.5 * K, 1.0
    X = x0.astype(np.float64)
    G = np.zeros_like(X)
    for k in range(K):
        G += pi[:, k:k + 1].astype(np.float64) * ((X - mu[k].astype(np.float32)) @
                                                  inv[k].astype(np.float64).T)
    G *= beta / K
    assert np.abs(G).max() < 5  # no clipping: the step is the gradient itself
    step64 = -lr * G
    errs = {}
    prev = _lib.launch_opts().community_async
    try:
        for kern in (2, 3):
            _lib.set_option("community_async", kern)
            x = t(x0)
            ce.community_grad(x, t(pi), t(mu), t(inv), beta, lr, 1)
            e = (x.cpu().numpy().astype(np.float64) - X) - step64
            errs[kern] = (np.sqrt((e ** 2).mean() / (step64 ** 2).mean()),
                          np.abs(e).max() / np.abs(step64).max())
    finally:
        _lib.set_option("community_async", prev)
    print("rms / max relative error vs float64: fp32 MFMA %.3g / %.3g, bf16 parts %.3g / %.3g"
          % (errs[2] + errs[3]))
    assert errs[3][0] <= 1.5 * errs[2][0] and errs[3][1] <= 1.5 * errs[2][1], errs


@pytest.mark.parametrize("r16", [2, 3])
def test_c4_responsibilities_k50_1m(c4_rows, r16):
    """predict_proba (:37) of a K = 50 full-covariance mixture on all 1M rows (come_gmm_resp,
    sklearn's upper-triangular precision factors) and the EM E-step (come_gmm_estep, + per-row
    log-sum-exp) on 4,000 sampled rows against the float64 restatement of sklearn;
    gmm_resp16 2 (fp32 16x16x4 MFMAs) and 3 (fp32 operands as bf16 parts), one tolerance."""
    from come_amd import _lib
    prev = _lib.launch_opts().gmm_resp16
    _lib.set_option("gmm_resp16", r16)
    try:
        _c4_responsibilities(c4_rows)
    finally:
        _lib.set_option("gmm_resp16", prev)


def test_c4_estep_bf3_error_is_fp32_level(c4_rows):
    """k_gmm_resp_b16's per-row log-sum-exp (the EM log-likelihood term) against float64 on 100k
    C4 rows: RMS and max error within 1.5x of the fp32-MFMA E-step's (k_gmm_resp16t) -- the
    bf16-part products are not a reduced-precision form (see the community test above)."""
    from come_amd import _lib
    from scipy.special import logsumexp
    x0 = c4_rows[0][:100_000]
    w, mu, cov = params(6, sep=0.3)
    pc = orc.precision_cholesky(cov)
    g = gmm.GaussianMixture(K)
    g._w, g._mu, g._pc = (torch.as_tensor(a, device=DEV) for a in (w, mu, pc))
    g._prepare_estep()
    pcf = g._e_pc.double().cpu().numpy()
    mpf = g._e_mp.double().cpu().numpy()
    lnf = g._e_ln.double().cpu().numpy()
    X = x0.astype(np.float64)
    lp = np.stack([lnf[k] - 0.5 * ((X @ pcf[k] - mpf[k]) ** 2).sum(1) for k in range(K)], 1)
    ref = logsumexp(lp, 1)
    errs = {}
    prev = _lib.launch_opts().gmm_resp16
    try:
        for r16 in (2, 3):
            _lib.set_option("gmm_resp16", r16)
            _, lse = gmm.estep(t(x0), g._e_pc, g._e_mp, g._e_ln)
            e = lse.double().cpu().numpy() - ref
            errs[r16] = (np.sqrt((e ** 2).mean() / (ref ** 2).mean()), np.abs(e).max())
    finally:
        _lib.set_option("gmm_resp16", prev)
    print("lse rms relative / max abs error vs float64: fp32 MFMA %.3g / %.3g, bf16 parts "
          "%.3g / %.3g" % (errs[2] + errs[3]))
    assert errs[3][0] <= 1.5 * errs[2][0] and errs[3][1] <= 1.5 * errs[2][1], errs


def _c4_responsibilities(c4_rows):
    x0, _ = c4_rows
    w, mu, cov = params(6, sep=0.3)
    pc = orc.precision_cholesky(cov)
    resp = ce.gmm_resp(t(x0), *ce.gmm_resp_params(w, mu, pc, DEV)).cpu().numpy()
    g = gmm.GaussianMixture(K)
    g._w, g._mu, g._pc = (torch.as_tensor(a, device=DEV) for a in (w, mu, pc))
    g._prepare_estep()
    er, lse = gmm.estep(t(x0), g._e_pc, g._e_mp, g._e_ln)
    rows = np.random.RandomState(7).choice(len(x0), 4000, replace=False)
    ref_lr = orc.gmm_log_resp(x0[rows].astype(np.float64), w, mu, cov)
    np.testing.assert_allclose(resp[rows], np.exp(ref_lr), rtol=0, atol=2e-4)
    np.testing.assert_allclose(er.cpu().numpy()[rows], np.exp(ref_lr), rtol=0, atol=2e-4)
    np.testing.assert_allclose(resp.sum(1), 1.0, atol=1e-4)
    # lse = log sum_k w_k N(x; mu_k, S_k) (its mean is sklearn's lower bound)
    from scipy.special import logsumexp
    pc64 = pc
    ld = np.array([np.log(np.diag(pc64[k])).sum() for k in range(K)])
    X = x0[rows].astype(np.float64)
    lp = np.stack([np.log(w[k]) + ld[k] - 0.5 * D * np.log(2 * np.pi)
                   - 0.5 * ((X @ pc64[k] - mu[k] @ pc64[k]) ** 2).sum(1) for k in range(K)], 1)
    np.testing.assert_allclose(lse.cpu().numpy()[rows], logsumexp(lp, 1), rtol=2e-5, atol=2e-3)


@pytest.fixture(scope="module")
def c4_100k():
    rng = np.random.RandomState(8)
    w, mu, cov = params(9, sep=1.5)
    lab = rng.choice(K, 100_000, p=w)
    X = np.empty((100_000, D))
    for k in range(K):
        m = lab == k
        X[m] = rng.multivariate_normal(mu[k], cov[k], m.sum())
    return X.astype(np.float32), w, mu, cov


@pytest.mark.parametrize("cov", [3, 4, 5])
def test_c4_scatter_k50(c4_100k, cov):
    """M-step scatter matrices sum_i r_ik (x_i - m_k)(x_i - m_k)^T (come_gmm_scatter, the
    2-component MFMA workgroups, K = 50 = 25 pairs) vs float64 for a spread of components, both
    members of a workgroup pair included; gmm_cov_async 3 (fp32 16x16x4), 4 (bf16 parts, the
    staging inside the MFMA wavefronts: k_gmm_cov_fb3) and 5 (bf16 parts, specialised staging
    wavefronts: k_gmm_cov_bf3)."""
    from come_amd import _lib
    X, w, mu, cov_ = c4_100k
    R = np.random.RandomState(10).dirichlet(np.ones(K), len(X)).astype(np.float32)
    M = (mu + 0.1).astype(np.float32)
    prev = _lib.launch_opts().gmm_cov_async
    _lib.set_option("gmm_cov_async", cov)
    try:
        S = gmm.scatter(t(X), t(R), t(M)).cpu().numpy()
    finally:
        _lib.set_option("gmm_cov_async", prev)
    X64 = X.astype(np.float64)
    for k in (0, 1, 24, 25, 48, 49):
        Dk = X64 - M[k]
        ref = (R[:, k, None] * Dk).T @ Dk
        np.testing.assert_allclose(S[k], ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max(),
                                   err_msg="component %d" % k)


def test_c4_scatter_bf3_error_is_fp32_level(c4_100k):
    """k_gmm_cov_fb3 and k_gmm_cov_bf3 (E^T E with E = sqrt(r) (x - m) carried as three bf16
    parts) against float64 on the 100k C4 rows, all 50 components: RMS and max relative error
    within 1.5x of the fp32-MFMA scatter's (k_gmm_cov16)."""
    from come_amd import _lib
    X, w, mu, cov_ = c4_100k
    R = np.random.RandomState(10).dirichlet(np.ones(K), len(X)).astype(np.float32)
    M = (mu + 0.1).astype(np.float32)
    X64 = X.astype(np.float64)
    ref = np.stack([((R[:, k, None] * (X64 - M[k])).T @ (X64 - M[k])) for k in range(K)])
    errs = {}
    prev = _lib.launch_opts().gmm_cov_async
    try:
        for cv in (3, 4, 5):
            _lib.set_option("gmm_cov_async", cv)
            e = gmm.scatter(t(X), t(R), t(M)).double().cpu().numpy() - ref
            errs[cv] = (np.sqrt((e ** 2).mean() / (ref ** 2).mean()),
                        np.abs(e).max() / np.abs(ref).max())
    finally:
        _lib.set_option("gmm_cov_async", prev)
    print("scatter rms / max relative error vs float64: fp32 MFMA %.3g / %.3g, bf16 parts "
          "(fb3) %.3g / %.3g, (bf3) %.3g / %.3g" % (errs[3] + errs[4] + errs[5]))
    for cv in (4, 5):
        assert errs[cv][0] <= 1.5 * errs[3][0] and errs[cv][1] <= 1.5 * errs[3][1], errs


@pytest.mark.parametrize("V,K_,chunks", [(1000, 3, 7), (4133, 5, 1), (16 * 48 * 3 + 5, 2, 3),
                                          (37, 1, 4), (100_003, 7, 0)])
def test_scatter_fused_matches_bf3(V, K_, chunks):
    """k_gmm_cov_fb3 (gmm_cov_async 4 at d = 128) takes k_gmm_cov_bf3's (5) arithmetic in the same
    order -- 16-sample k-steps in sample order, the six part products per off-diagonal tile in the
    same order, zeros for rows past the chunk -- with two differences: sqrt(r) by v_sqrt_f32
    (within 1 ulp of bf3's correctly rounded sqrtf) and a diagonal tile's cross terms as U + U^T
    (U = a1 b2 + a1 b3), a different rounding of the same sum, exactly symmetric.  So the two agree
    to a few fp32 ulps of the matrix scale everywhere (a layout or tiling error would show as O(1)),
    and both match float64.  Ragged chunks (rows not a multiple of the 16-row block or of the
    staging ring), an odd K (a workgroup with one live component), a single chunk, more chunks than
    rows, and gmm.scatter's own chunking."""
    from come_amd import _lib
    rng = np.random.RandomState(V)
    X = rng.standard_normal((V, D)).astype(np.float32)
    R = rng.dirichlet(np.ones(K_), V).astype(np.float32)
    M = (rng.standard_normal((K_, D)) * 0.5).astype(np.float32)
    out = {}
    prev = _lib.launch_opts().gmm_cov_async
    try:
        for cv in (4, 5):
            _lib.set_option("gmm_cov_async", cv)
            out[cv] = gmm.scatter(t(X), t(R), t(M), chunks=chunks or None).cpu().numpy()
    finally:
        _lib.set_option("gmm_cov_async", prev)
    for k in range(K_):
        scale = np.abs(out[5][k]).max()
        np.testing.assert_allclose(out[4][k], out[5][k], rtol=0, atol=2e-6 * scale)
    assert np.array_equal(out[4], out[4].transpose(0, 2, 1))
    X64 = X.astype(np.float64)
    for k in range(K_):
        Dk = X64 - M[k]
        ref = (R[:, k, None] * Dk).T @ Dk
        np.testing.assert_allclose(out[4][k], ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max())



def test_c4_em_iterations_k50_match_sklearn(c4_100k):
    """Two EM iterations at K = 50, d = 128, V = 100k from fixed initial parameters: the GPU
    GaussianMixture (E-step + means + scatter + Cholesky) vs sklearn's GaussianMixture (:18,27)
    with the same weights_init / means_init / precisions_init, tol = 0."""
    import warnings
    from sklearn.exceptions import ConvergenceWarning
    from sklearn.mixture import GaussianMixture as SkGMM
    X, w, mu, cov = c4_100k
    rng = np.random.RandomState(11)
    w0 = np.full(K, 1.0 / K)
    mu0 = mu + rng.normal(size=mu.shape) * 0.3
    prec0 = np.stack([np.linalg.inv(c + np.eye(D) * 0.3) for c in cov])
    kw = dict(n_components=K, covariance_type="full", tol=0.0, reg_covar=1e-5, max_iter=2,
              weights_init=w0, means_init=mu0, precisions_init=prec0, init_params="random")
    sk = SkGMM(random_state=0, **kw)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", ConvergenceWarning)
        sk.fit(X.astype(np.float64))
    g = gmm.GaussianMixture(random_state=0, **kw).fit(t(X))
    assert g.n_iter_ == sk.n_iter_ == 2
    np.testing.assert_allclose(g.weights_, sk.weights_, rtol=2e-3, atol=1e-5)
    np.testing.assert_allclose(g.means_, sk.means_, rtol=2e-3, atol=2e-3)
    np.testing.assert_allclose(g.covariances_, sk.covariances_, rtol=2e-3, atol=2e-3)
    np.testing.assert_allclose(g.lower_bound_, sk.lower_bound_, rtol=1e-4)
