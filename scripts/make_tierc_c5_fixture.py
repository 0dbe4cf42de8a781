"""Generates tests/golden/tierc_c5_seq.json: the sequential C oracle's held-out SGNS loss after one
launch of walks at C5's kernel shape (d = 256, n = 10; tests/tierc_inputs.py C5), for
tests/test_gpu_tierc.py::test_o2_hogwild_c5_kernel_shape.  CPU only: every input is built on the
host (Chung-Lu graph, make_table, the exact host walker, numpy picks), so the GPU test rebuilds the
same arrays on the box and checks the digest.  The oracle runs on one core in walk order (the
reference with workers=1), progress printed per 8192-walk chunk (~15 minutes).

    python scripts/make_tierc_c5_fixture.py [--out tests/golden/tierc_c5_seq.json]
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
    from oracle import oracle as orc
    import come_amd.training_sdg_inner as tsi
    from tierc_inputs import C5, C5_HYPER, c5_inputs, sgns_loss
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "tierc_c5_seq.json"))
    args = ap.parse_args()
    t0 = time.time()
    x = c5_inputs()
    w, n, lr = C5_HYPER["window"], C5_HYPER["negative"], C5_HYPER["lr"]
    ri, rp, rn = x.heldout(w, n)
    l0 = sgns_loss(x.node0, np.zeros_like(x.node0), ri, rp, rn)
    print("inputs ready %.0fs, init loss %.6f, digest %s" % (time.time() - t0, l0, x.digest),
          flush=True)
    sn, sc = x.node0.copy(), np.zeros_like(x.node0)
    W = x.train.shape[0]
    pairs = 0
    for s in range(0, W, 8192):
        p, _ = orc.sgns_o2_hogwild(sn, sc, x.train[s:s + 8192], x.seeds[s:s + 8192], w, n,
                                   x.table, lr, 1.0, threads=1)
        pairs += p
        print("seq %d walks %.0fs" % (min(W, s + 8192), time.time() - t0), flush=True)
    assert pairs == tsi.count_o2_pairs(x.train, w)
    out = {"what": "sequential C oracle (oracle/come_oracle_mt.c, threads=1: walks in order) "
                   "held-out SGNS loss after one launch of walks at C5's kernel shape; generated "
                   "by scripts/make_tierc_c5_fixture.py from tests/tierc_inputs.py C5",
           "inputs": {k: (list(v) if isinstance(v, tuple) else v) for k, v in C5.items()},
           "walks": W, "pairs": int(pairs), "inputs_sha256": x.digest, "init_loss": l0,
           "seq_loss": sgns_loss(sn, sc, ri, rp, rn), "lr": lr, "window": w, "negative": n,
           "wall_s": time.time() - t0}
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
