"""End-to-end throughput of the product trainers as a reference user calls them, host side
included (JSON lines):

* O1: Node2Vec.train (node_embeddings.py:35-106) at C2 (SBM 100 x 1000, ~1M edges, d = 128,
  n = 5, lr 0.1) in the reference's G.edges() order, `iter` passes: wall time per pass (edge ->
  row mapping once, per-pass seeds from the global numpy RNG, pyx:427, and their upload), beside
  the seed drawing alone (native come_np_draw_seeds vs numpy's own randint).
* O2: Context2Vec.train (context_embeddings.py:41-113) at C3 (1M-node Chung-Lu, d = 128, n = 5,
  w 5, lr 0.1) on a HOST id array of 1,048,576 walks x 80 (what build_deepwalk_corpus returns):
  wall time per train() call -- id -> row mapping, seeds, upload and the launch.

    python scripts/trainers_e2e.py [--iter 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iter", type=int, default=10)
    args = ap.parse_args()
    import torch
    import come_amd.training_sdg_inner as tsi
    from come_amd.graph import sbm
    from come_amd.model import Model
    from come_amd.node_embeddings import Node2Vec
    dev = torch.device("cuda", 0)
    g = sbm(100, 1000, 0.016, 4.04e-5, seed=0)
    np.random.seed(1234)
    m = Model(g.degree_by_id(), size=128, table_size=100_000_000, k=100, device=dev)
    edges = g.edge_ids()                                                   # node ids 1..V
    edges = edges[np.lexsort((edges[:, 1], edges[:, 0]))]                  # G.edges() order
    E = len(edges)
    trainer = Node2Vec(lr=0.1, negative=5)
    trainer.train(m, edges=edges, iter=1)  # warm-up: library, hot rows, packed table
    torch.cuda.synchronize()
    t0 = time.time()
    pairs = trainer.train(m, edges=edges, iter=args.iter)
    torch.cuda.synchronize()
    wall = time.time() - t0
    t0 = time.time()
    tsi.draw_seeds(E)
    native = time.time() - t0
    t0 = time.time()
    ab = np.random.randint(0, 2 ** 24, size=2 * E).astype(np.uint64)
    _ = (ab[0::2] << np.uint64(24)) + ab[1::2]
    numpy_ms = time.time() - t0
    print(json.dumps({"trainer": "Node2Vec.train", "edges": E, "passes": args.iter,
                      "pairs": pairs,
                      "wall_s": wall, "ms_per_pass": wall / args.iter * 1e3,
                      "pair_updates_per_s_end_to_end": pairs / wall,
                      "seed_draw_ms_per_pass_native": native * 1e3,
                      "seed_draw_ms_per_pass_numpy": numpy_ms * 1e3}), flush=True)
    del m
    torch.cuda.empty_cache()

    from come_amd.context_embeddings import Context2Vec
    from come_amd.graph import chung_lu, random_walks
    g3 = chung_lu(1_000_000, 20.0, gamma=2.5, seed=1, device=dev)
    np.random.seed(1234)
    m3 = Model(g3.degree_by_id(), size=128, table_size=100_000_000, k=1, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(100)
    walks = random_walks(g3, 0, 80, seed=100, device=dev,
                         starts=torch.randperm(g3.V, generator=gen, device=dev)[:1 << 20])
    ids = torch.where(walks >= 0, walks + 1, walks).cpu().numpy()  # node ids, -1 after the end
    c2v = Context2Vec(lr=0.1, window_size=5, negative=5)
    c2v.train(m3, paths=ids[:4096], total_nodes=ids.size)  # warm-up
    torch.cuda.synchronize()
    t0 = time.time()
    pairs3 = c2v.train(m3, paths=ids, total_nodes=ids.size)
    torch.cuda.synchronize()
    wall3 = time.time() - t0
    print(json.dumps({"trainer": "Context2Vec.train", "walks": int(ids.shape[0]),
                      "pairs": pairs3, "wall_s": wall3,
                      "pair_updates_per_s_end_to_end": pairs3 / wall3}), flush=True)


if __name__ == "__main__":
    main()
