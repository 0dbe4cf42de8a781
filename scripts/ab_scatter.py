"""A/B of the GMM scatter kernel's chunk count at C4 (V = 1M, K = 50, d = 128): interleaved
rounds, HIP-event timing, one process."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from come_amd import gmm
    dev = torch.device("cuda", 0)
    V, K, d = 1_000_000, 50, 128
    rng = np.random.RandomState(2)
    x = torch.from_numpy(rng.standard_normal((V, d)).astype(np.float32)).to(dev)
    resp = torch.from_numpy(np.random.RandomState(3).dirichlet(np.ones(K), V).astype(np.float32)
                            ).to(dev)
    mu = torch.from_numpy((rng.standard_normal((K, d)) * 0.5).astype(np.float32)).to(dev)
    variants = [int(c) for c in sys.argv[1:]] or [20, 21]
    ref = gmm.scatter(x, resp, mu, chunks=variants[0])
    res = {c: [] for c in variants}
    for r in range(6):
        for c in variants:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = gmm.scatter(x, resp, mu, chunks=c)
            e.record()
            torch.cuda.synchronize()
            if r:
                res[c].append(s.elapsed_time(e))
            if r == 0:
                err = float((out - ref).abs().max() / ref.abs().max())
                print("chunks %d: max rel diff vs chunks %d = %.2e" % (c, variants[0], err))
    for c in variants:
        print("chunks %4d  grid %5d  median %.3f ms  min %.3f ms" % (
            c, c * K, float(np.median(res[c])), float(np.min(res[c]))))


if __name__ == "__main__":
    main()
