"""k_gmm_cov_async vs k_gmm_cov_mfma on the same inputs (several shapes, ragged chunks): the
async form only moves the centring from staging to the operand reads, so the scatter matrices
must be bit-identical.  Prints the max abs difference per shape; exits 1 on any mismatch."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from come_amd import _lib, gmm
    dev = torch.device("cuda", 0)
    bad = 0
    for V, K, d, chunks in [(5000, 3, 64, None), (4097, 5, 128, 7), (300, 2, 128, 1),
                            (999, 3, 128, None), (100000, 50, 128, None), (65, 4, 64, 2)]:
        rng = np.random.RandomState(V + K + d)
        x = torch.from_numpy(rng.standard_normal((V, d)).astype(np.float32)).to(dev)
        resp = torch.from_numpy(rng.dirichlet(np.ones(K), V).astype(np.float32)).to(dev)
        mu = torch.from_numpy(rng.standard_normal((K, d)).astype(np.float32)).to(dev)
        out = []
        for opt in (0, 1):
            _lib.set_option("gmm_cov_async", opt)
            out.append(gmm.scatter(x, resp, mu, chunks=chunks).cpu().numpy())
        _lib.set_option("gmm_cov_async", 1)  # the default
        diff = float(np.abs(out[0] - out[1]).max())
        print("V=%d K=%d d=%d chunks=%s: max |async - sync| = %g" % (V, K, d, chunks, diff))
        bad += diff != 0.0
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
