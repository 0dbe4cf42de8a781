"""End-to-end ComE flow on the GPU (scripts/come_e2e.py: adsc_Karate.py:104-137 on a planted-
partition graph) against the same flow restated on the CPU with the oracle (sequential C SGNS,
sklearn GaussianMixture, numpy community step) on the same walks: statistical parity of the
outcome -- the NMI of the fitted communities against the planted blocks."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def cpu_reference_flow(g, walks_rows, dim, neg, w, lr, alpha, beta, com_iters, k, seed):
    from sklearn.mixture import GaussianMixture
    import come_amd.training_sdg_inner as tsi
    from oracle import oracle as orc
    np.random.seed(seed)
    node = np.random.uniform(-1, 1, (g.V, dim)).astype(np.float32)   # model.py:86
    ctx = np.zeros((g.V, dim), np.float32)
    table = orc.make_table(g.degree, max(10 ** 6, 100 * g.V))
    edges = g.edges.astype(np.int32)
    walks = walks_rows.astype(np.int32)

    def o1():
        orc.sgns_o1(node, edges, tsi.draw_seeds(len(edges)), neg, table, lr)

    def o2():
        orc.sgns_o2(node, ctx, walks, tsi.draw_seeds(len(walks)), w, neg, table, lr, alpha)
    o1()
    o2()
    o1()
    o2()
    gm = GaussianMixture(k, covariance_type="full", reg_covar=1e-5, n_init=3, random_state=seed)
    gm.fit(node)
    pi = gm.predict_proba(node).astype(np.float32)
    inv = np.linalg.inv(gm.covariances_.astype(np.float32)).astype(np.float32)
    node = orc.community_train(node, pi, gm.means_.astype(np.float32), inv, beta, lr, com_iters)
    return np.argmax(pi, 1)


def test_e2e_sbm_recovers_blocks_like_the_cpu_reference_flow():
    import os
    import sys
    from sklearn.metrics import normalized_mutual_info_score
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "scripts"))
    import come_e2e
    from come_amd.graph import random_walks, sbm
    blocks, size, dim = 8, 250, 64
    kw = dict(blocks=blocks, block_size=size, p_in=0.04, p_out=0.002, dim=dim, negative=5,
              window=5, walk_length=30, num_walks=4, iters=1, lr=0.025, alpha=1.0, beta=0.1,
              com_iters=5, seed=3, n_init=3)
    out = come_e2e.run(**kw, log=lambda s: None)
    assert out["o2_pairs"] > 0 and out["gmm_converged"]
    # CPU flow on the same graph and the same walks (the device walker is seeded identically)
    g = sbm(blocks, size, 0.04, 0.002, seed=3)
    walks = random_walks(g, 4, 30, seed=4, device="cuda").cpu().numpy()
    pred = cpu_reference_flow(g, walks, dim, 5, 5, 0.025, 1.0, 0.1, 5, blocks, 3)
    nmi_cpu = normalized_mutual_info_score(np.arange(g.V) // size, pred)
    print("NMI gpu %.3f cpu-reference %.3f" % (out["nmi"], nmi_cpu))
    assert out["nmi"] > 0.8
    assert out["nmi"] >= nmi_cpu - 0.05


def test_context2vec_device_walks_equal_host_walks():
    """Context2Vec.train on a CUDA id tensor (device path: no host copy) performs exactly the
    updates of the same walks given as a numpy array (deterministic mode, same seeds)."""
    from come_amd.context_embeddings import Context2Vec
    from come_amd.model import Model
    rng = np.random.RandomState(0)
    V, d = 300, 64
    walks = rng.randint(1, V + 1, (40, 25)).astype(np.int64)
    walks[5, 20:] = -1  # an early-stopped walk
    out = []
    for paths in (walks, torch.from_numpy(walks).cuda()):
        np.random.seed(1)
        m = Model((np.arange(1, V + 1), rng.randint(1, 9, V) * 0 + 3), size=d, table_size=5000,
                  k=2)
        c = Context2Vec(lr=0.05, window_size=3, negative=4, deterministic=True)
        n = c.train(m, paths=paths, total_nodes=walks.size)
        out.append((n, m.node_embedding.cpu().numpy(), m.context_embedding.cpu().numpy()))
    assert out[0][0] == out[1][0]
    np.testing.assert_array_equal(out[0][1], out[1][1])
    np.testing.assert_array_equal(out[0][2], out[1][2])
