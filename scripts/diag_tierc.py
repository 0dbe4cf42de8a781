"""Diagnostic for the tier-C test (tests/test_gpu_tierc.py): held-out SGNS loss of the O2 Hogwild
kernel variants (per-call come_launch_opts) at C3's shape on 100k nodes, against the sequential
run, plus each variant's time at that size.

    python scripts/diag_tierc.py [--walks 10000] [--lr 0.1]
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
    ap.add_argument("--walks", type=int, default=10000)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--nodes", type=int, default=100000)
    ap.add_argument("--variants", default="")
    ap.add_argument("--hot-p", default="1e-3,1e-4,3e-5,1e-5,3e-6")
    ap.add_argument("--waves", default="1024", help="max_waves values for hot_p<p>_w<waves>")
    ap.add_argument("--repeat", type=int, default=1, help="runs per variant (Hogwild spread)")
    ap.add_argument("--no-oracle", action="store_true", help="skip the sequential C oracle")
    args = ap.parse_args()
    import torch
    import come_amd.training_sdg_inner as tsi
    from come_amd.graph import chung_lu, random_walks
    from oracle import oracle as orc
    from test_gpu_tierc import sgns_loss, heldout_o2_pairs, dev

    g = chung_lu(args.nodes, 20.0, gamma=2.5, seed=21)
    table = orc.make_table(g.degree.astype(np.float64), 100_000_000)
    walks = random_walks(g, 1, 80, seed=22, device="cuda").cpu().numpy()
    rng = np.random.RandomState(23)
    walks = walks[rng.permutation(len(walks))[:args.walks + 2000]]
    node0 = rng.uniform(-1, 1, (g.V, 128)).astype(np.float32)
    seeds = rng.randint(0, 2 ** 48, args.walks, dtype=np.int64).astype(np.uint64)
    train, held = walks[:args.walks], walks[args.walks:]
    w, n, lr = 5, 5, args.lr
    ri, rp, rn = heldout_o2_pairs(held, w, n, table, 200_000, 24)
    l0 = sgns_loss(node0, np.zeros_like(node0), ri, rp, rn)
    tab = dev(table)
    tw, ts = dev(train), dev(seeds)
    variants = {
        "sequential": (tsi.MODE_SEQUENTIAL, {}),
        "default": (tsi.MODE_HOGWILD, {}),
        "stream_nohot": (tsi.MODE_HOGWILD, {"_hot_p": 0.0}),
        "direct": (tsi.MODE_HOGWILD, {"o2_kernel": 1}),
        "direct_atomic": (tsi.MODE_HOGWILD, {"o2_kernel": 1, "o2_atomic_writeback": 1}),
        "direct_fresh": (tsi.MODE_HOGWILD, {"o2_kernel": 1, "o2_fresh_loads": 1}),
        "direct_fresh_atomic": (tsi.MODE_HOGWILD, {"o2_kernel": 1, "o2_fresh_loads": 1,
                                                   "o2_atomic_writeback": 1}),
        "waves1024": (tsi.MODE_HOGWILD, {"max_waves": 1024}),
    }
    for p in args.hot_p.split(","):
        variants["hot_p%s" % p] = (tsi.MODE_HOGWILD, {"_hot_p": float(p)})
        variants["direct_hot_p%s" % p] = (tsi.MODE_HOGWILD, {"o2_kernel": 1, "_hot_p": float(p)})
        variants["stream_hot_p%s" % p] = (tsi.MODE_HOGWILD, {"o2_kernel": 3, "_hot_p": float(p)})
        for mw in args.waves.split(","):
            variants["hot_p%s_w%s" % (p, mw)] = (tsi.MODE_HOGWILD, {"max_waves": int(mw),
                                                                     "_hot_p": float(p)})
    if args.variants:
        variants = {k: v for k, v in variants.items() if k in args.variants.split(",")}
    out = {"init": l0}
    if not args.no_oracle:
        sn, sc = node0.copy(), np.zeros_like(node0)
        orc.sgns_o2_hogwild(sn, sc, train, seeds, w, n, table, lr, 1.0, threads=1)
        out["oracle_seq"] = sgns_loss(sn, sc, ri, rp, rn)
        print("oracle_seq", out["oracle_seq"], flush=True)
    runs = [(name, r) for name in variants for r in range(args.repeat)]
    for name, rep in runs:
        mode, opts = variants[name]
        opts = dict(opts)
        hp = opts.pop("_hot_p", None)
        hot = None
        if hp is not None or name == "default":
            hp = hp if hp is not None else tsi.DEFAULT_HOT_P
            hot = tsi.hot_rows(tab, g.V, max(1, int(hp * len(table)))) if hp > 0 else None
        node, ctx = dev(node0), dev(np.zeros_like(node0))
        torch.cuda.synchronize()
        t0 = time.time()
        tsi.sgns_o2(node, ctx, tw, ts, w, n, tab, lr, 1.0, mode, opts=opts, hot=hot)
        torch.cuda.synchronize()
        el = time.time() - t0
        hn, hc = node.cpu().numpy(), ctx.cpu().numpy()
        fin = bool(np.isfinite(hn).all() and np.isfinite(hc).all())
        loss = sgns_loss(hn, hc, ri, rp, rn) if fin else float("nan")
        hub = int(np.argmax(g.degree))
        nhot = 0 if hot is None else int(np.unpackbits(hot.cpu().numpy().view(np.uint8)).sum())
        key = name if args.repeat == 1 else "%s#%d" % (name, rep)
        out[key] = {"loss": loss, "ms": el * 1e3, "hot_rows": nhot,
                     "hub_node_norm": float(np.linalg.norm(hn[hub])),
                     "hub_ctx_norm": float(np.linalg.norm(hc[hub])),
                     "max_ctx_norm": float(np.linalg.norm(hc, axis=1).max())}
        print(key, json.dumps(out[key]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
