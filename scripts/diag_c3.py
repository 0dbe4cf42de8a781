"""Hogwild stability at the benchmarked shape (C3: Chung-Lu 1M nodes, T=1e8, d=128, n=5, w=5,
L=80, lr 0.1): held-out SGNS loss and the largest node / ctx row norms after ONE bench launch
(131,072 walks) of each O2 Hogwild variant, repeated, from the same initial tables.

    python scripts/diag_c3.py [--repeat 4] [--variants stream,direct]
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
    ap.add_argument("--walks", type=int, default=1 << 17)
    ap.add_argument("--repeat", type=int, default=4)
    ap.add_argument("--variants", default="stream,direct")
    ap.add_argument("--launches", type=int, default=1)
    args = ap.parse_args()
    import torch
    import come_amd.training_sdg_inner as tsi
    from come_amd.graph import chung_lu, random_walks
    from oracle import oracle as orc
    from test_gpu_tierc import sgns_loss, heldout_o2_pairs, dev

    t0 = time.time()
    g = chung_lu(args.nodes, 20.0, gamma=2.5, seed=1)
    table = orc.make_table(g.degree.astype(np.float64), 100_000_000)
    walks = random_walks(g, 1, 80, seed=100, device="cuda")
    perm = torch.randperm(walks.shape[0], generator=torch.Generator().manual_seed(5))
    walks = walks[perm.to(walks.device)]
    train = walks[:args.walks * args.launches].contiguous()
    held = walks[-20000:].cpu().numpy()
    rng = np.random.RandomState(7)
    node0 = rng.uniform(-1, 1, (g.V, 128)).astype(np.float32)
    seeds = dev(rng.randint(0, 2 ** 48, train.shape[0], dtype=np.int64).astype(np.uint64))
    ri, rp, rn = heldout_o2_pairs(held, 5, 5, table, 200_000, 24)
    l0 = sgns_loss(node0, np.zeros_like(node0), ri, rp, rn)
    tab = dev(table)
    hot = tsi.hot_rows(tab, g.V, int(tsi.DEFAULT_HOT_P * len(table)))
    hub = np.argsort(-g.degree)[:8]
    print("setup %.1fs V=%d walks=%d init loss %.4f" % (time.time() - t0, g.V, train.shape[0], l0),
          flush=True)
    opts = {"stream": {}, "direct": {"o2_kernel": 1}}
    for name in args.variants.split(","):
        for r in range(args.repeat):
            node, ctx = dev(node0), torch.zeros_like(dev(node0))
            torch.cuda.synchronize()
            t1 = time.time()
            B = args.walks
            for s in range(args.launches):
                tsi.sgns_o2(node, ctx, train[s * B:(s + 1) * B], seeds[s * B:(s + 1) * B], 5, 5,
                            tab, 0.1, 1.0, tsi.MODE_HOGWILD, opts=opts[name], hot=hot)
            torch.cuda.synchronize()
            el = time.time() - t1
            hn, hc = node.cpu().numpy(), ctx.cpu().numpy()
            nn = np.linalg.norm(hn, axis=1)
            cn = np.linalg.norm(hc, axis=1)
            out = {"loss": sgns_loss(hn, hc, ri, rp, rn), "ms": el * 1e3,
                   "max_node_norm": float(nn.max()), "argmax_node_deg": int(g.degree[nn.argmax()]),
                   "hub_node_norms": [round(float(x), 2) for x in nn[hub]],
                   "max_ctx_norm": float(cn.max()), "nodes_norm_gt_10": int((nn > 10).sum())}
            print("%s#%d %s" % (name, r, json.dumps(out)), flush=True)


if __name__ == "__main__":
    main()
