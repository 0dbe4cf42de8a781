"""Tier C vs training length at C3's vocabulary: held-out SGNS loss of the GPU Hogwild product
launch (come_sgns_o2_ex, automatic kernel, Context2Vec's hot-row bitmap) after W walks, against
the sequential C oracle (walks in order, one thread) after the same W walks, for growing W.
The sequential run is one pass in 8192-walk chunks (progress printed per chunk).

    python scripts/tierc_scale.py [--nodes 1000000] [--checkpoints 16384,49152,131072]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--checkpoints", default="16384,49152,131072")
    ap.add_argument("--gpu-runs", type=int, default=2)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    import come_amd.training_sdg_inner as tsi
    from come_amd.graph import chung_lu, random_walks
    from oracle import oracle as orc
    from test_gpu_tierc import sgns_loss, heldout_o2_pairs, dev

    cps = [int(x) for x in args.checkpoints.split(",")]
    W = max(cps)
    g = chung_lu(args.nodes, 20.0, gamma=2.5, seed=1)
    table = orc.make_table(g.degree.astype(np.float64), 100_000_000)
    walks = random_walks(g, 1, 80, seed=100, device="cuda")
    rng = np.random.RandomState(7)
    pick = torch.from_numpy(rng.choice(walks.shape[0], W + 20000, replace=False)).to(walks.device)
    walks = walks[pick].cpu().numpy()
    train, held = walks[:W], walks[W:]
    node0 = rng.uniform(-1, 1, (g.V, 128)).astype(np.float32)
    seeds = rng.randint(0, 2 ** 48, W, dtype=np.int64).astype(np.uint64)
    w, n, lr = 5, 5, 0.1
    ri, rp, rn = heldout_o2_pairs(held, w, n, table, 200_000, 24)
    out = {"V": g.V, "init": sgns_loss(node0, np.zeros_like(node0), ri, rp, rn), "points": []}
    tab = dev(table)
    hot = tsi.hot_rows(tab, g.V, int(tsi.DEFAULT_HOT_P * len(table)))
    gpu = {}
    for c in cps:
        ls = []
        for _ in range(args.gpu_runs):
            node, ctx = dev(node0), torch.zeros((g.V, 128), dtype=torch.float32, device="cuda")
            for s in range(0, c, 131072):
                e = min(c, s + 131072)
                tsi.sgns_o2(node, ctx, dev(train[s:e]), dev(seeds[s:e]), w, n, tab, lr, 1.0,
                            tsi.MODE_HOGWILD, hot=hot)
            torch.cuda.synchronize()
            ls.append(sgns_loss(node.cpu().numpy(), ctx.cpu().numpy(), ri, rp, rn))
        gpu[c] = ls
        print("gpu W=%d: %s" % (c, ls), flush=True)
    sn, sc = node0.copy(), np.zeros_like(node0)
    t0 = time.time()
    done = 0
    for s in range(0, W, 8192):
        e = min(W, s + 8192)
        orc.sgns_o2_hogwild(sn, sc, train[s:e], seeds[s:e], w, n, table, lr, 1.0, threads=1)
        done = e
        print("seq %d walks %.0fs" % (done, time.time() - t0), flush=True)
        if done in cps:
            l_seq = sgns_loss(sn, sc, ri, rp, rn)
            pt = {"walks": done, "seq": l_seq, "gpu": gpu[done],
                  "max_rel": max(abs(x - l_seq) / l_seq for x in gpu[done])}
            out["points"].append(pt)
            print(json.dumps(pt), flush=True)
    print(json.dumps(out))
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
