"""End-to-end O1 throughput of the product trainer (Node2Vec.train, node_embeddings.py:35-106) at
C2 (SBM 100 x 1000, ~1M edges, d = 128, n = 5, lr 0.1), the reference's G.edges() order, `iter`
passes: wall time per pass including the host side (edge -> row mapping once, per-pass seeds from
the global numpy RNG, pyx:427, and their upload), beside the kernel time per pass and the seed
drawing alone (native come_np_draw_seeds vs numpy's own randint).  One JSON line.

    python scripts/o1_train_e2e.py [--iter 10]
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
    print(json.dumps({"edges": E, "passes": args.iter, "pairs": pairs,
                      "wall_s": wall, "ms_per_pass": wall / args.iter * 1e3,
                      "pair_updates_per_s_end_to_end": pairs / wall,
                      "seed_draw_ms_per_pass_native": native * 1e3,
                      "seed_draw_ms_per_pass_numpy": numpy_ms * 1e3}))


if __name__ == "__main__":
    main()
