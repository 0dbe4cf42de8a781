"""The CPU twins of the C-ABI (include/come.h come_cpu_*, csrc/come_cpu.cpp),
called through libcome.so on the CPU -- no GPU needed:

* sequential mode bit-exact with the oracle's WAVE64 order (= the GPU kernels' order), and the
  reference's own golden vectors to tier A/B;
* Hogwild threads bit-exact with sequential on walks that share no row, and within tier C's 1%
  of the sequential held-out loss on a small power-law graph;
* community step and GMM responsibilities against the reference's golden vectors and the float64
  restatements;
* the C-ABI's argument validation.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as orc

cpu = pytest.importorskip("come_amd.cpu")

KAT_O2 = np.load(os.path.join(GOLDEN, "kat_o2.npz"))
KAT_O1 = np.load(os.path.join(GOLDEN, "kat_o1.npz"))


def tol_for(margin):
    return 1e-6 if margin >= 1e-4 else 1e-3


def rand_case(V, d, P, L, seed, T=20000):
    rng = np.random.RandomState(seed)
    table = orc.make_table(rng.randint(1, 50, V).astype(np.float64), T)
    node = rng.uniform(-1, 1, (V, d)).astype(np.float32)
    ctx = rng.uniform(-0.1, 0.1, (V, d)).astype(np.float32)
    walks = rng.randint(0, V, (P, L)).astype(np.int32)
    walks[rng.rand(P, L) < 0.03] = -1  # None entries (pyx:435-436)
    seeds = rng.randint(0, 2 ** 48, P).astype(np.uint64)
    return table, node, ctx, walks, seeds


@pytest.mark.parametrize("d,neg,w", [(128, 5, 5), (100, 10, 3), (2, 5, 2), (256, 0, 4)])
def test_o2_sequential_bit_exact_vs_oracle_wave64(d, neg, w):
    table, node, ctx, walks, seeds = rand_case(300, d, 12, 40, d + neg)
    n2, c2 = node.copy(), ctx.copy()
    pairs = cpu.sgns_o2(node, ctx, walks, seeds, w, neg, table, 0.1, 0.7, cpu.MODE_SEQUENTIAL, 1)
    ref = orc.sgns_o2(n2, c2, walks, seeds, w, neg, table, 0.1, 0.7, dot_mode=orc.DOT_WAVE64)
    assert pairs == ref
    np.testing.assert_array_equal(node, n2)
    np.testing.assert_array_equal(ctx, c2)


@pytest.mark.parametrize("d,neg", [(128, 5), (64, 10), (3, 5)])
def test_o1_sequential_bit_exact_vs_oracle_wave64(d, neg):
    rng = np.random.RandomState(d)
    V, E = 200, 300
    table = orc.make_table(rng.randint(1, 30, V).astype(np.float64), 5000)
    node = rng.uniform(-1, 1, (V, d)).astype(np.float32)
    edges = rng.randint(0, V, (E, 2)).astype(np.int32)
    seeds = rng.randint(0, 2 ** 48, E).astype(np.uint64)
    n2 = node.copy()
    pairs = cpu.sgns_o1(node, edges, seeds, neg, table, 0.2, cpu.MODE_SEQUENTIAL, 1)
    ref = orc.sgns_o1(n2, edges, seeds, neg, table, 0.2, dot_mode=orc.DOT_WAVE64)
    assert pairs == ref == 2 * E
    np.testing.assert_array_equal(node, n2)


@pytest.mark.parametrize("name", list(KAT_O2["names"]))
def test_o2_reference_golden(name):
    """The reference's own train_o2 outputs (tests/golden/make_golden.py): tier A on clean
    cases, tier B where a dot product sits within 1e-4 bucket units of an edge."""
    z, pre = KAT_O2, "o2_%s_" % name
    d, neg, w, V, L, P = [int(x) for x in z[pre + "params"]]
    lr, alpha = [float(x) for x in z[pre + "lr_alpha"]]
    node, ctx = z[pre + "node0"].copy(), z[pre + "ctx0"].copy()
    walks = np.ascontiguousarray(z[pre + "walks"], np.int32)
    seeds = np.ascontiguousarray(z[pre + "seeds"], np.uint64)
    table = np.ascontiguousarray(z[pre + "table"], np.uint32)
    cpu.sgns_o2(node, ctx, walks, seeds, w, neg, table, lr, alpha, cpu.MODE_SEQUENTIAL, 1)
    tol = tol_for(float(z[pre + "margin"]))
    np.testing.assert_allclose(node, z[pre + "node1"], rtol=0, atol=tol)
    np.testing.assert_allclose(ctx, z[pre + "ctx1"], rtol=0, atol=tol)


@pytest.mark.parametrize("name", list(KAT_O1["names"]))
def test_o1_reference_golden(name):
    z, pre = KAT_O1, "o1_%s_" % name
    d, neg, V, E = [int(x) for x in z[pre + "params"]]
    node = z[pre + "node0"].copy()
    pairs = cpu.sgns_o1(node, np.ascontiguousarray(z[pre + "edges"], np.int32),
                        np.ascontiguousarray(z[pre + "seeds"], np.uint64), neg,
                        np.ascontiguousarray(z[pre + "table"], np.uint32),
                        float(z[pre + "lr"][0]), cpu.MODE_SEQUENTIAL, 1)
    assert pairs == 2 * E
    np.testing.assert_allclose(node, z[pre + "node1"], rtol=0,
                               atol=tol_for(float(z[pre + "margin"])))


def test_o2_hogwild_threads_bit_exact_on_disjoint_walks():
    """Walks that share no row (and draw no negatives) are independent: 8 Hogwild workers must
    give the sequential result bit for bit, whatever the interleaving."""
    rng = np.random.RandomState(3)
    V, d, L = 8192, 64, 16
    node = rng.uniform(-1, 1, (V, d)).astype(np.float32)
    ctx = rng.uniform(-0.1, 0.1, (V, d)).astype(np.float32)
    walks = rng.permutation(V).reshape(V // L, L).astype(np.int32)
    seeds = np.zeros(V // L, np.uint64)
    table = np.arange(1, 10, dtype=np.uint32)
    n2, c2 = node.copy(), ctx.copy()
    p1 = cpu.sgns_o2(node, ctx, walks, seeds, 3, 0, table, 0.05, 1.0, cpu.MODE_HOGWILD, 8)
    p2 = cpu.sgns_o2(n2, c2, walks, seeds, 3, 0, table, 0.05, 1.0, cpu.MODE_SEQUENTIAL, 1)
    assert p1 == p2 == orc.sgns_o2(node.copy(), ctx.copy(), walks, seeds, 3, 0, table, 0.05,
                                   1.0)
    np.testing.assert_array_equal(node, n2)
    np.testing.assert_array_equal(ctx, c2)


def test_o2_hogwild_threads_tier_c():
    """Tier C on a small power-law graph (exact host walker): the held-out SGNS loss after a
    Hogwild pass with 8 worker threads within 1% of the sequential pass's."""
    import random
    from come_amd import graph_utils as gu
    from come_amd.graph import chung_lu
    from tierc_inputs import heldout_o2_pairs, sgns_loss
    g = chung_lu(20000, 10.0, gamma=2.5, seed=5)
    gh = gu.Graph(np.arange(1, g.V + 1), g.rowptr, g.col.astype(np.int32), g.degree,
                  np.zeros((0, 2), np.int32))
    walks = np.asarray(gu._corpus(gh, [1], 40, 0.0, [random.Random(5)], threads=1), np.int32)
    train, held = walks[:16000], walks[16000:]
    table = orc.make_table(g.degree.astype(np.float64), 1_000_000)
    rng = np.random.RandomState(1)
    node0 = rng.uniform(-1, 1, (g.V, 32)).astype(np.float32)
    seeds = rng.randint(0, 2 ** 48, len(train)).astype(np.uint64)
    ri, rp, rn = heldout_o2_pairs(held, 4, 5, table, 50000, 2)
    losses = []
    for mode, threads in ((cpu.MODE_SEQUENTIAL, 1), (cpu.MODE_HOGWILD, 8)):
        node, ctx = node0.copy(), np.zeros_like(node0)
        cpu.sgns_o2(node, ctx, train, seeds, 4, 5, table, 0.1, 1.0, mode, threads)
        losses.append(sgns_loss(node, ctx, ri, rp, rn))
    l0 = sgns_loss(node0, np.zeros_like(node0), ri, rp, rn)
    assert losses[0] < l0 - 0.3
    assert abs(losses[1] - losses[0]) / losses[0] < 0.01, losses


def test_community_grad_reference_golden():
    z = np.load(os.path.join(GOLDEN, "community.npz"))
    for name in z["names"]:
        p = name + "_"
        beta, lr = [float(x) for x in z[p + "scal"]]
        x = z[p + "x0"].copy()
        cpu.community_grad(x, z[p + "pi"], z[p + "mu"], z[p + "inv"], beta, lr,
                           int(z[p + "iters"]), threads=4)
        np.testing.assert_allclose(x, z[p + "x1"], rtol=1e-5, atol=1e-5, err_msg=name)


@pytest.mark.parametrize("d,V,K,iters", [(64, 500, 7, 3), (96, 200, 3, 2), (256, 60, 3, 2)])
def test_community_grad_vs_oracle(d, V, K, iters):
    rng = np.random.RandomState(d + V)
    x0 = rng.normal(size=(V, d)).astype(np.float32)
    A = rng.normal(size=(K, d, d)) / np.sqrt(d)
    cov = np.einsum("kij,klj->kil", A, A) + np.eye(d)[None] * 0.5
    inv = np.linalg.inv(cov.astype(np.float32)).astype(np.float32)
    mu = rng.normal(size=(K, d)).astype(np.float32)
    pi = rng.dirichlet(np.ones(K), V).astype(np.float32)
    for beta in (0.05, 40.0):  # 40: the clip at +-5 is exercised
        x = x0.copy()
        cpu.community_grad(x, pi, mu, inv, beta, 0.1, iters, threads=3)
        ref = orc.community_train(x0, pi, mu, inv, beta, 0.1, iters)
        np.testing.assert_allclose(x, ref, rtol=2e-5, atol=2e-5)


def resp_params(w, mu, pc):
    d = mu.shape[1]
    mp = np.einsum("kd,kde->ke", mu, pc)
    ln = np.log(w) + np.array([np.log(np.diag(p)).sum() for p in pc]) - 0.5 * d * np.log(2 * np.pi)
    return (np.ascontiguousarray(pc, np.float32), np.ascontiguousarray(mp, np.float32),
            np.ascontiguousarray(ln, np.float32))


def test_gmm_resp_reference_golden():
    """sklearn predict_proba outputs captured from the reference's GaussianMixture."""
    z = np.load(os.path.join(GOLDEN, "gmm_resp.npz"))
    for name in z["names"]:
        p = name + "_"
        pc = orc.precision_cholesky(z[p + "cov"])
        resp, lse = cpu.gmm_estep(np.ascontiguousarray(z[p + "X"]),
                                  *resp_params(z[p + "w"], z[p + "mu"], pc), threads=2)
        np.testing.assert_allclose(resp, z[p + "pi"], rtol=0, atol=2e-5, err_msg=name)
        np.testing.assert_allclose(resp.sum(1), 1.0, atol=1e-5)


@pytest.mark.parametrize("V,K,d", [(700, 4, 8), (300, 5, 128), (90, 3, 200)])
def test_gmm_estep_vs_float64(V, K, d):
    from scipy.special import logsumexp
    rng = np.random.RandomState(V + d)
    mu = rng.normal(size=(K, d)) * 3
    A = rng.normal(size=(K, d, d)) / np.sqrt(d)
    cov = np.einsum("kij,klj->kil", A, A) * 0.5 + np.eye(d)[None] * 0.5
    w = rng.dirichlet(np.ones(K) * 3)
    X = (mu[rng.randint(0, K, V)] + rng.normal(size=(V, d))).astype(np.float32)
    pc = orc.precision_cholesky(cov)
    resp, lse = cpu.gmm_estep(X, *resp_params(w, mu, pc), threads=4)
    ref = orc.gmm_log_resp(X.astype(np.float64), w, mu, cov)
    np.testing.assert_allclose(resp, np.exp(ref), atol=2e-4)
    lp = np.stack([np.log(w[k]) - 0.5 * (((X.astype(np.float64) - mu[k]) @ pc[k]) ** 2).sum(1)
                   + np.log(np.diag(pc[k])).sum() - 0.5 * d * np.log(2 * np.pi)
                   for k in range(K)], 1)
    np.testing.assert_allclose(lse, logsumexp(lp, 1), rtol=2e-5, atol=2e-3)


def test_argument_validation():
    from come_amd._lib import ComeError, TABLE_PACKED
    table, node, ctx, walks, seeds = rand_case(50, 8, 2, 10, 0)
    with pytest.raises(ComeError, match="threads"):
        cpu.sgns_o2(node, ctx, walks, seeds, 2, 5, table, 0.1, 1.0, cpu.MODE_HOGWILD, 0)
    with pytest.raises(ComeError, match="packed"):
        cpu.sgns_o2(node, ctx, walks, seeds, 2, 5, table, 0.1, 1.0,
                    cpu.MODE_HOGWILD | TABLE_PACKED, 2)
    with pytest.raises(ComeError, match="negative"):
        cpu.sgns_o2(node, ctx, walks, seeds, 2, 21, table, 0.1, 1.0, cpu.MODE_HOGWILD, 2)
    with pytest.raises(TypeError):
        cpu.sgns_o2(node.astype(np.float64), ctx, walks, seeds, 2, 5, table, 0.1)
    # empty batches are no-ops
    n0 = node.copy()
    assert cpu.sgns_o2(node, ctx, walks[:0], seeds[:0], 2, 5, table, 0.1) == 0
    np.testing.assert_array_equal(node, n0)


@pytest.mark.gpu
@pytest.mark.parametrize("d,neg", [(128, 5), (256, 10)])
def test_cpu_twin_equals_gpu_sequential(d, neg):
    """The CPU twin and the GPU kernel in sequential mode: the same walks, seeds and tables give
    the same tables bit for bit (both use the WAVE64 dot order)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import come_amd.training_sdg_inner as tsi
    table, node, ctx, walks, seeds = rand_case(400, d, 10, 50, d)
    dev = torch.device("cuda", 0)
    tn, tc = torch.from_numpy(node).to(dev), torch.from_numpy(ctx).to(dev)
    tsi.sgns_o2(tn, tc, torch.from_numpy(walks).to(dev),
                torch.from_numpy(seeds.view(np.int64)).to(dev), 4, neg,
                torch.from_numpy(table.view(np.int32)).to(dev), 0.1, 1.0, tsi.MODE_SEQUENTIAL)
    cpu.sgns_o2(node, ctx, walks, seeds, 4, neg, table, 0.1, 1.0, cpu.MODE_SEQUENTIAL, 1)
    np.testing.assert_array_equal(tn.cpu().numpy(), node)
    np.testing.assert_array_equal(tc.cpu().numpy(), ctx)
