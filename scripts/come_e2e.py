"""End-to-end ComE on one GPU: the adsc_Karate.py:104-137 flow on a synthetic stochastic block
model, every phase through come_amd (no reference code), with per-phase timings and the NMI of
the GMM communities against the planted blocks.

    python scripts/come_e2e.py [--blocks 100 --block-size 1000 --dim 128 ...]

Phases (reference file:line): walks (graph_utils.py:187-192 -> device walker), O1 pre-training
(node_embeddings.py:35), O2 pre-training (context_embeddings.py:41), then per outer iteration
O1 + O2 + GMM fit (community_embeddings.py:20-37, GPU EM) + community gradient
(community_embeddings.py:61-78).  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(blocks=100, block_size=1000, p_in=0.016, p_out=4.04e-5, dim=128, negative=5,
        window=5, walk_length=40, num_walks=5, iters=1, lr=0.025, alpha=1.0, beta=0.1,
        com_iters=5, seed=0, reg_covar=1e-5, n_init=3, deterministic=False, log=print):
    import torch
    from sklearn.metrics import normalized_mutual_info_score
    from come_amd.community_embeddings import Community2Vec
    from come_amd.context_embeddings import Context2Vec
    from come_amd.graph import random_walks, sbm
    from come_amd.model import Model
    from come_amd.node_embeddings import Node2Vec

    dev = torch.device("cuda", 0)
    t = {}

    def tick(name, t0):
        torch.cuda.synchronize(dev)
        t[name] = t.get(name, 0.0) + time.time() - t0

    t0 = time.time()
    g = sbm(blocks, block_size, p_in, p_out, seed=seed)
    labels = np.arange(g.V) // block_size
    t["graph_s"] = time.time() - t0
    np.random.seed(seed)
    t0 = time.time()
    model = Model(g.degree_by_id(), size=dim, table_size=max(10 ** 6, 100 * g.V), k=blocks,
                  device=dev)
    tick("model_s", t0)
    t0 = time.time()
    walks = random_walks(g, num_walks, walk_length, seed=seed + 1, device=dev)
    walks_ids = torch.where(walks >= 0, walks + 1, walks)  # rows -> node ids (ids = row + 1)
    tick("walks_s", t0)
    edges = g.edge_ids()
    nl = Node2Vec(lr=lr, negative=negative, deterministic=deterministic)
    cl = Context2Vec(lr=lr, window_size=window, negative=negative, deterministic=deterministic)
    cm = Community2Vec(model, lr=lr, reg_covar=reg_covar)
    cm.g_mixture.n_init = n_init
    pairs = 0
    t0 = time.time()
    nl.train(model, edges=edges, iter=1)
    tick("o1_s", t0)
    t0 = time.time()
    pairs += cl.train(model, paths=walks_ids, total_nodes=walks.numel(), alpha=alpha)
    tick("o2_s", t0)
    for _ in range(iters):
        t0 = time.time()
        nl.train(model, edges=edges, iter=1)
        tick("o1_s", t0)
        t0 = time.time()
        pairs += cl.train(model, paths=walks_ids, total_nodes=walks.numel(), alpha=alpha)
        tick("o2_s", t0)
        t0 = time.time()
        cm.fit(model)
        tick("gmm_fit_s", t0)
        t0 = time.time()
        cm.train(range(1, g.V + 1), model, beta, iter=com_iters)
        tick("community_s", t0)
    pred = torch.argmax(model.pi, 1).cpu().numpy()
    nmi = float(normalized_mutual_info_score(labels, pred))
    out = {"nodes": g.V, "edges": int(g.num_edges), "blocks": blocks, "dim": dim,
           "o2_pairs": int(pairs), "nmi": nmi,
           "gmm_converged": bool(getattr(cm.g_mixture, "converged_", False)),
           "timings_s": {k: round(v, 4) for k, v in t.items()}}
    log(json.dumps(out))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=100)
    ap.add_argument("--block-size", type=int, default=1000)
    ap.add_argument("--p-in", type=float, default=0.016)
    ap.add_argument("--p-out", type=float, default=4.04e-5)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--negative", type=int, default=5)
    ap.add_argument("--window", type=int, default=5)
    ap.add_argument("--walk-length", type=int, default=40)
    ap.add_argument("--num-walks", type=int, default=5)
    ap.add_argument("--iters", type=int, default=1)
    ap.add_argument("--n-init", type=int, default=3)
    args = ap.parse_args()
    run(blocks=args.blocks, block_size=args.block_size, p_in=args.p_in, p_out=args.p_out,
        dim=args.dim, negative=args.negative, window=args.window, walk_length=args.walk_length,
        num_walks=args.num_walks, iters=args.iters, n_init=args.n_init)


if __name__ == "__main__":
    main()
