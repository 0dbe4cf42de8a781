"""O1 tier C at C2's shape with and without the contended-row bitmap (float-atomic updates of hot
rows vs plain stores everywhere): held-out losses of GPU Hogwild launches against the sequential
oracle (tests/test_gpu_tierc.py's c2_shape and losses).

    python scripts/tierc_o1_hot.py --hot-p 5e-6 0 --runs 2
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import come_amd.training_sdg_inner as tsi  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from test_gpu_tierc import c2_shape, dev, log_sigmoid, sgns_loss  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hot-p", type=float, nargs="+", default=[tsi.DEFAULT_HOT_P, 0.0])
    ap.add_argument("--runs", type=int, default=2)
    args = ap.parse_args()
    g, table, train, held, node0, seeds = c2_shape.__wrapped__()
    n, lr = 5, 0.1
    rng = np.random.RandomState(32)
    neg = table[rng.randint(0, len(table), (len(held), n))].astype(np.int64)

    def losses(x):
        ref = float(-log_sigmoid(np.einsum("pd,pd->p", x[held[:, 1]].astype(np.float64),
                                           x[held[:, 0]].astype(np.float64))).sum())
        return ref, sgns_loss(x, x, held[:, 0], held[:, 1], neg)
    seq = node0.copy()
    orc.sgns_o1_hogwild(seq, train, seeds, n, table, lr, threads=1)
    l_seq = losses(seq)
    tab = dev(table)
    for hp in args.hot_p:
        hot = tsi.hot_rows(tab, g.V, int(hp * len(table))) if hp > 0 else None
        rel = []
        for _ in range(args.runs):
            node = dev(node0)
            tsi.sgns_o1(node, dev(train), dev(seeds), n, tab, lr, tsi.MODE_HOGWILD, hot=hot)
            torch.cuda.synchronize()
            l_hog = losses(node.cpu().numpy())
            rel.append([(a - b) / abs(b) for a, b in zip(l_hog, l_seq)])
        print(json.dumps({"hot_p": hp, "seq": l_seq, "rel_ref_loss_and_sgns_loss": rel}),
              flush=True)


if __name__ == "__main__":
    main()
