"""Generate the golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

Run in the build container only (needs /root/reference and oracle/_ref built by
oracle/build_ref.py).  The reference is imported read-only from /root/reference; only the
resulting input/output vectors (data) are committed.  Nothing here runs on the GPU box.

Fixtures:
  kat_o2.npz      per-walk known-answer tests of train_o2 (pyx:454-509), several (d, neg, w, V)
  kat_o1.npz      per-edge known-answer tests of train_o1 (pyx:407-450)
  make_table.npz  Model.make_table (model.py:97-122) on small degree maps
  community.npz   Community2Vec.train (community_embeddings.py:61-78) on fixed GMM parameters
  gmm_resp.npz    GaussianMixture.predict_proba + fp32 inv (community_embeddings.py:34-37) for
                  fixed (weights, means, covariances)
  karate.npz      the adsc_Karate.py:104-137 flow (workers=1) on the shipped Karate graph, walks
                  generated here with a seeded uniform walker (graph_utils' walker needs
                  networkx 1.x), every phase's output recorded

Seeds: every train_o1/train_o2 call draws next_random = 2^24*randint(0,2^24)+randint(0,2^24)
from the global numpy RNG (pyx:427,477).  For KATs the generator re-seeds numpy before each call
and records the resulting next_random explicitly, so consumers pass seeds directly.
"""
import glob
import importlib.util
import os
import random
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("COME_REFERENCE", "/root/reference")

sys.path.insert(0, REPO)
from oracle import oracle as orc  # noqa: E402  (margin computation only)


def load_reference():
    so = glob.glob(os.path.join(REPO, "oracle", "_ref", "training_sdg_inner*.so"))
    if not so:
        raise SystemExit("build the reference first: python oracle/build_ref.py")
    spec = importlib.util.spec_from_file_location("training_sdg_inner", so[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.path.insert(0, REF)
    import utils  # the reference's utils package
    sys.modules["utils.training_sdg_inner"] = mod
    utils.training_sdg_inner = mod
    return mod


class V:  # stands in for utils.embedding.Vocab: the kernels read only .index (pyx:438,488)
    __slots__ = ("index",)

    def __init__(self, i):
        self.index = i


def seed_for(s):
    np.random.seed(s)
    a = np.random.randint(0, 2 ** 24)
    b = np.random.randint(0, 2 ** 24)
    return (2 ** 24) * a + b


def power_counts(rng, n):
    return np.maximum(1, (rng.pareto(1.5, n) * 3).astype(np.int64) + 1)


def ref_table(ref_model_cls, counts_by_id, T):
    """Model.make_table on a bare instance (model.py:97-122)."""
    from utils.embedding import Vocab
    m = ref_model_cls.__new__(ref_model_cls)
    m.vocab = {}
    for idx, nid in enumerate(sorted(counts_by_id)):
        v = Vocab()
        v.count = counts_by_id[nid]
        v.index = idx
        m.vocab[nid] = v
    m.vocab_size = len(m.vocab)
    m.table_size = T
    m.make_table()
    return m.table


def gen_kat_o2(ref, Model):
    cases = [
        # name, d, neg, window, V, L, nwalks, T, none_frac, ctx_scale, node_scale
        ("d2_n4_w3", 2, 4, 3, 34, 20, 6, 2000, 0.0, 0.5, 1.0),
        ("d2_n5_tinyV", 2, 5, 2, 5, 15, 4, 500, 0.0, 0.5, 1.0),
        ("d128_n5_w5", 128, 5, 5, 500, 80, 3, 20000, 0.0, 0.1, 1.0),
        ("d128_n10_smallV_none", 128, 10, 5, 60, 40, 3, 5000, 0.1, 0.1, 0.3),
        ("d256_n10_w5", 256, 10, 5, 300, 30, 2, 10000, 0.0, 0.05, 0.3),
        ("d100_n5_w2", 100, 5, 2, 200, 25, 3, 8000, 0.05, 0.1, 0.5),
        ("d64_n1_w1", 64, 1, 1, 40, 12, 3, 1000, 0.0, 0.2, 0.5),
        ("d2_ctx0_n4", 2, 4, 3, 34, 20, 3, 2000, 0.0, 0.0, 1.0),
    ]
    out = {}
    rng = np.random.RandomState(20240601)
    for ci, (name, d, neg, w, Vn, L, P, T, none_frac, cs, ns) in enumerate(cases):
        counts = power_counts(rng, Vn)
        table = ref_table(Model, {i + 1: int(c) for i, c in enumerate(counts)}, T)
        node0 = rng.uniform(-ns, ns, (Vn, d)).astype(np.float32)
        ctx0 = rng.uniform(-cs, cs, (Vn, d)).astype(np.float32) if cs > 0 else \
            np.zeros((Vn, d), np.float32)
        walks = rng.randint(0, Vn, (P, L)).astype(np.int32)
        walks[rng.uniform(size=(P, L)) < none_frac] = -1
        seeds = np.zeros(P, np.uint64)
        node, ctx = node0.copy(), ctx0.copy()
        work = np.zeros(d, np.float32)
        counts_ret = []
        for p in range(P):
            s = 1000 * ci + p
            seeds[p] = seed_for(s)
            path = [V(int(x)) if x >= 0 else None for x in walks[p]]
            np.random.seed(s)
            counts_ret.append(ref.train_o2(node, ctx, path, 0.1, neg, w, table, py_alpha=0.7,
                                           py_size=d, py_work=work))
        # margin of this case under the restatement (REF dot order)
        n2, c2 = node0.copy(), ctx0.copy()
        orc.reset_margin()
        orc.sgns_o2(n2, c2, walks, seeds, w, neg, table, 0.1, 0.7, dot_mode=orc.DOT_REF)
        margin = orc.min_margin()
        pre = "o2_%s_" % name
        out.update({pre + "node0": node0, pre + "ctx0": ctx0, pre + "walks": walks,
                    pre + "seeds": seeds, pre + "table": table, pre + "node1": node,
                    pre + "ctx1": ctx,
                    pre + "params": np.array([d, neg, w, Vn, L, P], np.int64),
                    pre + "lr_alpha": np.array([0.1, 0.7], np.float32),
                    pre + "ret": np.array(counts_ret, np.int64),
                    pre + "margin": np.array(margin)})
        print("kat_o2 %-24s margin=%.3g" % (name, margin))
    out["names"] = np.array([c[0] for c in cases])
    np.savez_compressed(os.path.join(HERE, "kat_o2.npz"), **out)


def gen_kat_o1(ref, Model):
    cases = [
        ("d2_n4", 2, 4, 34, 40, 2000, 1.0),
        ("d128_n5", 128, 5, 400, 30, 20000, 0.2),
        ("d128_n10_smallV", 128, 10, 30, 25, 3000, 0.2),
        ("d256_n5", 256, 5, 100, 10, 4000, 0.1),
        ("d100_n3_selfloop", 100, 3, 50, 15, 3000, 0.2),
    ]
    out = {}
    rng = np.random.RandomState(777)
    for ci, (name, d, neg, Vn, E, T, ns) in enumerate(cases):
        counts = power_counts(rng, Vn)
        table = ref_table(Model, {i + 1: int(c) for i, c in enumerate(counts)}, T)
        node0 = rng.uniform(-ns, ns, (Vn, d)).astype(np.float32)
        edges = rng.randint(0, Vn, (E, 2)).astype(np.int32)
        if "selfloop" in name:
            edges[3, 1] = edges[3, 0]
        seeds = np.zeros(E, np.uint64)
        node = node0.copy()
        work = np.zeros(d, np.float32)
        for e in range(E):
            s = 50000 + 1000 * ci + e
            seeds[e] = seed_for(s)
            np.random.seed(s)
            ref.train_o1(node, [V(int(edges[e, 0])), V(int(edges[e, 1]))], 0.2, neg, table,
                         py_size=d, py_work=work)
        n2 = node0.copy()
        orc.reset_margin()
        orc.sgns_o1(n2, edges, seeds, neg, table, 0.2, dot_mode=orc.DOT_REF)
        margin = orc.min_margin()
        pre = "o1_%s_" % name
        out.update({pre + "node0": node0, pre + "edges": edges, pre + "seeds": seeds,
                    pre + "table": table, pre + "node1": node,
                    pre + "params": np.array([d, neg, Vn, E], np.int64),
                    pre + "lr": np.array([0.2], np.float32),
                    pre + "margin": np.array(margin)})
        print("kat_o1 %-24s margin=%.3g" % (name, margin))
    out["names"] = np.array([c[0] for c in cases])
    np.savez_compressed(os.path.join(HERE, "kat_o1.npz"), **out)


def karate_graph():
    import networkx as nx
    adj = np.loadtxt(os.path.join(REF, "data", "karate", "karate.adjlist"), dtype=np.int64)
    G = nx.Graph()
    G.add_edges_from(adj)  # graph_utils.py:60-69 (__from_adjlist_unchecked__)
    G = G.to_undirected()
    labels = np.loadtxt(os.path.join(REF, "data", "karate", "karate_zachary.labels"),
                        dtype=np.int64)
    return G, adj, labels


def gen_make_table(Model):
    G, _, _ = karate_graph()
    deg = dict(G.degree())
    out = {}
    rng = np.random.RandomState(5)
    cases = [("karate_T100k", deg, 100000),
             ("karate_T5e6_sha", deg, 5000000),
             ("pow1000_T200k", {i + 1: int(c) for i, c in enumerate(power_counts(rng, 1000))},
              200000),
             ("uniform7_T50", {i + 1: 3 for i in range(7)}, 50),
             ("skew_T1000", {1: 1000, 2: 1, 3: 1, 4: 5000, 5: 2}, 1000)]
    import hashlib
    for name, counts, T in cases:
        tab = ref_table(Model, counts, T)
        ids = np.array(sorted(counts), np.int64)
        out[name + "_ids"] = ids
        out[name + "_counts"] = np.array([counts[i] for i in ids], np.int64)
        out[name + "_T"] = np.array(T, np.int64)
        if name.endswith("_sha"):
            out[name + "_sha256"] = np.array(hashlib.sha256(tab.tobytes()).hexdigest())
            out[name + "_bincount"] = np.bincount(tab, minlength=len(ids)).astype(np.int64)
        else:
            out[name + "_table"] = tab
        print("make_table %s T=%d max=%d" % (name, T, tab.max()))
    out["names"] = np.array([c[0] for c in cases])
    np.savez_compressed(os.path.join(HERE, "make_table.npz"), **out)


def random_spd(rng, K, d, scale=1.0):
    A = rng.normal(size=(K, d, d)) * scale / np.sqrt(d)
    return np.einsum("kij,klj->kil", A, A) + np.eye(d)[None] * 0.3


def gen_community():
    from ADSCModel.community_embeddings import Community2Vec
    out = {}
    rng = np.random.RandomState(11)
    cases = [("v300_k4_d8", 300, 4, 8, 0.01, 0.1, 5), ("v200_k3_d128", 200, 3, 128, 0.05, 0.1, 3),
             ("v100_k5_d2_clip", 100, 5, 2, 50.0, 0.1, 2)]
    for name, Vn, K, d, beta, lr, iters in cases:
        x0 = rng.normal(size=(Vn, d)).astype(np.float32)
        cov = random_spd(rng, K, d).astype(np.float32)
        inv = np.linalg.inv(cov).astype(np.float32)
        mu = rng.normal(size=(K, d)).astype(np.float32)
        pi = rng.dirichlet(np.ones(K), Vn).astype(np.float32)
        model = types.SimpleNamespace(node_embedding=x0.copy(), centroid=mu, pi=pi,
                                      inv_covariance_mat=inv, k=K,
                                      vocab={i + 1: V(i) for i in range(Vn)})
        c2v = Community2Vec.__new__(Community2Vec)
        c2v.lr = lr
        c2v.train(list(range(1, Vn + 1)), model, beta, chunksize=37, iter=iters)
        pre = name + "_"
        out.update({pre + "x0": x0, pre + "mu": mu, pre + "inv": inv, pre + "pi": pi,
                    pre + "x1": model.node_embedding,
                    pre + "scal": np.array([beta, lr], np.float64),
                    pre + "iters": np.array(iters)})
        print("community %s" % name)
    out["names"] = np.array([c[0] for c in cases])
    np.savez_compressed(os.path.join(HERE, "community.npz"), **out)


def gen_gmm_resp():
    from sklearn.mixture import GaussianMixture
    from sklearn.mixture._gaussian_mixture import _compute_precision_cholesky
    out = {}
    rng = np.random.RandomState(13)
    for name, Vn, K, d in [("v500_k4_d8", 500, 4, 8), ("v300_k6_d128", 300, 6, 128),
                           ("v64_k2_d2", 64, 2, 2)]:
        cov = random_spd(rng, K, d, 0.5)
        mu = rng.normal(size=(K, d)) * 1.5
        w = rng.dirichlet(np.ones(K) * 3)
        X = (mu[rng.randint(0, K, Vn)] + rng.normal(size=(Vn, d))).astype(np.float32)
        g = GaussianMixture(n_components=K, covariance_type="full")
        g.weights_, g.means_, g.covariances_ = w, mu, cov
        g.precisions_cholesky_ = _compute_precision_cholesky(cov, "full")
        pi = g.predict_proba(X).astype(np.float32)        # community_embeddings.py:37
        inv = np.linalg.inv(cov.astype(np.float32)).astype(np.float32)   # :36 (fp32 inv)
        pre = name + "_"
        out.update({pre + "X": X, pre + "w": w, pre + "mu": mu, pre + "cov": cov,
                    pre + "pi": pi, pre + "inv32": inv})
        print("gmm_resp %s" % name)
    out["names"] = np.array(["v500_k4_d8", "v300_k6_d128", "v64_k2_d2"])
    np.savez_compressed(os.path.join(HERE, "gmm_resp.npz"), **out)


def karate_walks(G, num_paths, length, seed):
    """Uniform truncated walks, alpha=0, starts shuffled per pass (graph_utils.py:20-46,187-192),
    written for networkx 3 (list(G.neighbors))."""
    rnd = random.Random(seed)
    nodes = list(G.nodes())
    walks = []
    for _ in range(num_paths):
        rnd.shuffle(nodes)
        for n in nodes:
            path = [n]
            while len(path) < length:
                nb = list(G.neighbors(path[-1]))
                if not nb:
                    break
                path.append(rnd.choice(nb))
            walks.append(path)
    return np.array(walks, np.int64)


def gen_karate():
    """adsc_Karate.py:104-137 with workers=1 (deterministic), Karate zachary labels (K=2)."""
    from ADSCModel.model import Model
    from ADSCModel.node_embeddings import Node2Vec
    from ADSCModel.context_embeddings import Context2Vec
    from ADSCModel.community_embeddings import Community2Vec
    G, adj, labels = karate_graph()
    walks = karate_walks(G, 10, 20, 9999999999)
    edges = np.array(G.edges())
    size, neg, ws, lr, alpha, beta, T = 2, 4, 3, 0.1, 1.0, 0.01, 5000000
    np.random.seed(42)
    model = Model(dict(G.degree()), size=size, table_size=T,
                  input_file=os.path.join("karate", "karate_zachary"),
                  path_labels=os.path.join(REF, "data"))
    rec = {"edges": edges, "walks": walks, "degree_ids": np.array(sorted(dict(G.degree())), np.int64),
           "degree_counts": np.array([d for _, d in sorted(dict(G.degree()).items())], np.int64),
           "labels": labels, "hyper": np.array([size, neg, ws, lr, alpha, beta, T], np.float64),
           "node_init": model.node_embedding.copy(), "table_bincount":
               np.bincount(model.table, minlength=model.vocab_size).astype(np.int64)}
    nl = Node2Vec(workers=1, negative=neg, lr=lr)
    cl = Context2Vec(window_size=ws, workers=1, negative=neg, lr=lr)
    cl.alpha = alpha  # context_embeddings.py:91-92 reads self.alpha (deadlock otherwise)
    cm = Community2Vec(model, reg_covar=1e-5, lr=lr)
    np.random.seed(100)
    nl.train(model, edges=edges, iter=1, chunksize=20)
    rec["after_o1_pre"] = model.node_embedding.copy()
    np.random.seed(101)
    cl.train(model, paths=iter(list(walks)), total_nodes=walks.size, alpha=alpha, chunksize=20)
    rec["after_o2_pre_node"] = model.node_embedding.copy()
    rec["after_o2_pre_ctx"] = model.context_embedding.copy()
    np.random.seed(102)
    nl.train(model, edges=edges, iter=1, chunksize=20)
    np.random.seed(103)
    cl.train(model, paths=iter(list(walks)), total_nodes=walks.size, alpha=alpha, chunksize=20)
    rec["after_loop_node"] = model.node_embedding.copy()
    rec["after_loop_ctx"] = model.context_embedding.copy()
    np.random.seed(104)
    cm.fit(model)
    rec.update({"gmm_centroid": model.centroid, "gmm_cov": model.covariance_mat,
                "gmm_inv": model.inv_covariance_mat, "gmm_pi": model.pi,
                "gmm_weights": cm.g_mixture.weights_})
    cm.train(G.nodes(), model, beta, chunksize=20, iter=5)
    rec["after_com_node"] = model.node_embedding.copy()
    np.savez_compressed(os.path.join(HERE, "karate.npz"), **rec)
    print("karate: walks %s edges %s" % (walks.shape, edges.shape))


def main():
    ref = load_reference()
    assert ref.FAST_VERSION in (0, 1)
    from ADSCModel.model import Model
    gen_kat_o2(ref, Model)
    gen_kat_o1(ref, Model)
    gen_make_table(Model)
    gen_community()
    gen_gmm_resp()
    gen_karate()


if __name__ == "__main__":
    main()
