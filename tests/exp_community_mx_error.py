"""Experiment (not collected by pytest): would the community step survive the `M_k x - M_k mu_k`
rewrite?  That form splits x once per row instead of pi_ik (x_i - mu_k) per
component, but it rounds M_k x, whose scale is |x|, where the reference's order
(community_embeddings.py:67-71) rounds M_k (x - mu_k), whose scale is |x - mu_k|.

Data as the step sees it in a ComE run: an SBM graph (50 blocks), node embeddings trained by the
sequential O1 oracle (oracle/oracle.py sgns_o1, pyx:407-437 restated), a K = 50 full-covariance
GMM fitted by sklearn (community_embeddings.py:18-27), then the same after five community steps
(oracle.community_train) and a refit -- the clustered state the VERDICT asks about.  Both forms are
evaluated in float32 (numpy sgemm: fp32 products, fp32 accumulation -- the error level of the fp32
kernel and of the bf16-part kernels) against float64 on the same float32 inputs.

    python tests/exp_community_mx_error.py [--nodes 20000] [--dim 128]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as orc  # noqa: E402


def sbm_edges(V, B, deg_in, deg_out, rng):
    blk = np.arange(V) % B
    members = [np.flatnonzero(blk == b) for b in range(B)]
    src, dst = [], []
    for v in range(V):
        m = members[blk[v]]
        src += [v] * (deg_in + deg_out)
        dst += list(rng.choice(m, deg_in)) + list(rng.randint(0, V, deg_out))
    e = np.stack([src, dst], 1)
    e = e[e[:, 0] != e[:, 1]]
    e = np.concatenate([e, e[:, ::-1]])
    return e[rng.permutation(len(e))].astype(np.int32), blk


def fit(x, K):
    from sklearn.mixture import GaussianMixture
    gm = GaussianMixture(K, covariance_type="full", reg_covar=1e-5, n_init=1, max_iter=100,
                         random_state=0).fit(x)
    inv = np.linalg.inv(gm.covariances_).astype(np.float32)
    return gm.predict_proba(x).astype(np.float32), gm.means_.astype(np.float32), inv


def errors(x, pi, mu, inv):
    """Relative errors vs float64 of the two float32 forms of g_i = sum_k pi_ik M_k (x_i - mu_k)."""
    K = mu.shape[0]
    g64 = np.zeros(x.shape, np.float64)
    gd = np.zeros(x.shape, np.float32)   # reference order: pi (x - mu), then M
    gy = np.zeros(x.shape, np.float32)   # rewrite: pi (M x), minus pi (M mu)
    c = np.stack([inv[k] @ mu[k] for k in range(K)]).astype(np.float32)
    for k in range(K):
        p = pi[:, k:k + 1]
        g64 += (p.astype(np.float64) * (x.astype(np.float64) - mu[k].astype(np.float64))) \
            @ inv[k].astype(np.float64)
        gd += (p * (x - mu[k])) @ inv[k]
        gy += p * (x @ inv[k])
    gy -= pi @ c
    out = {}
    for name, g in (("reference_order", gd), ("mx_minus_mmu", gy)):
        d = g.astype(np.float64) - g64
        out[name] = {"rms_rel": float(np.sqrt(np.mean(d ** 2)) / np.sqrt(np.mean(g64 ** 2))),
                     "max_rel": float(np.abs(d).max() / np.abs(g64).max())}
    out["ratio_rms"] = out["mx_minus_mmu"]["rms_rel"] / out["reference_order"]["rms_rel"]
    out["ratio_max"] = out["mx_minus_mmu"]["max_rel"] / out["reference_order"]["max_rel"]
    a = np.argmax(pi, 1)
    out["median_|x-mu|/|x|"] = float(np.median(np.linalg.norm(x - mu[a], axis=1)
                                               / np.linalg.norm(x, axis=1)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=20000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=50)
    ap.add_argument("--epochs", type=int, default=5)
    args = ap.parse_args()
    rng = np.random.RandomState(7)
    V, d, K = args.nodes, args.dim, args.k
    edges, _ = sbm_edges(V, K, 10, 1, rng)
    counts = np.bincount(edges[:, 0], minlength=V)
    table = orc.make_table(counts, 10_000_000)
    np.random.seed(1)
    node = np.random.uniform(-1, 1, (V, d)).astype(np.float32)  # model.py:86
    t0 = time.time()
    for _ in range(args.epochs):
        seeds = np.random.randint(0, 2 ** 31 - 1, len(edges)).astype(np.uint64)
        orc.sgns_o1(node, edges, seeds, 5, table, 0.025)
    res = {"nodes": V, "dim": d, "k": K, "edges": int(len(edges)),
           "train_s": round(time.time() - t0, 1)}
    pi, mu, inv = fit(node, K)
    res["after_o1_fit"] = errors(node, pi, mu, inv)
    node = orc.community_train(node, pi, mu, inv, 0.1, 0.025, 5)
    pi, mu, inv = fit(node, K)
    res["after_5_community_steps_and_refit"] = errors(node, pi, mu, inv)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
