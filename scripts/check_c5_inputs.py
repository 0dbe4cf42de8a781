"""Diagnose a digest mismatch between tier-C inputs built on the device and on the host
(tests/tierc_inputs.py): compares the graph (chung_lu with / without the device), the table and
the walks (device walker vs its CPU restatement) piece by piece.

    python scripts/check_c5_inputs.py [V] [train_walks]
"""
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def h(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def main():
    import torch
    from come_amd.graph import chung_lu
    from come_amd.graph_utils import device_walks
    from oracle import oracle as orc
    V = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 151_072
    dev = torch.device("cuda", 0)
    t0 = time.time()
    gd = chung_lu(V, 20.0, gamma=2.5, seed=4, device=dev)
    print("device graph %.0fs E=%d" % (time.time() - t0, gd.num_edges), flush=True)
    t0 = time.time()
    gh = chung_lu(V, 20.0, gamma=2.5, seed=4)
    print("host graph %.0fs E=%d" % (time.time() - t0, gh.num_edges), flush=True)
    for nm in ("edges", "col", "rowptr", "degree"):
        a, b = getattr(gd, nm), getattr(gh, nm)
        same = a.shape == b.shape and np.array_equal(a, b)
        print("%-7s device %s %s host %s %s  equal=%s" % (nm, a.dtype, a.shape, b.dtype, b.shape,
                                                         same), flush=True)
        if not same and a.shape == b.shape:
            d = np.nonzero(a.ravel() != b.ravel())[0]
            print("   first differences at", d[:5], a.ravel()[d[:5]], b.ravel()[d[:5]])
    rng = np.random.RandomState(43)
    starts = rng.choice(V, W, replace=False).astype(np.int32)
    wd = device_walks(torch.as_tensor(gh.rowptr, device=dev), torch.as_tensor(gh.col, device=dev),
                      torch.as_tensor(starts, device=dev), 80, alpha=0.0, seed=41).cpu().numpy()
    wh = orc.philox_walks(gh.rowptr, gh.col, starts, 80, 0.0, seed=41)
    same = np.array_equal(wd, wh)
    print("walks on the host graph: device %s host %s equal=%s" % (h(wd), h(wh), same))
    if not same:
        bad = np.nonzero((wd != wh).any(1))[0]
        print("   walks differing:", len(bad), "first", bad[:5])
        i = bad[0]
        print("   device", wd[i][:20], "\n   host  ", wh[i][:20])


if __name__ == "__main__":
    main()
