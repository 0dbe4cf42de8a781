"""Digest of the three C4 kernels' outputs on fixed seeded inputs (community step, E-step, M-step
scatter at d = 128): run under two builds (COME_LIB_PATH) to check that a change to their
arithmetic is bit-identical.  python scripts/c4_digest.py [V]"""
import hashlib
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))))
from come_amd import community_embeddings as ce, gmm  # noqa: E402


def main():
    V = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    K, d = 50, 128
    rng = np.random.RandomState(11)
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)  # noqa: E731
    x = rng.randn(V, d).astype(np.float32)
    mu = rng.randn(K, d).astype(np.float32)
    A = rng.randn(K, d, d).astype(np.float32) * 0.05
    cov = np.einsum("kij,klj->kil", A, A) + np.eye(d, dtype=np.float32)[None]
    inv = np.linalg.inv(cov).astype(np.float32)
    import scipy.linalg as sl
    chol = np.linalg.cholesky(cov)  # sklearn's precisions_cholesky_: upper factors
    prec = np.stack([sl.solve_triangular(c, np.eye(d), lower=True).T for c in chol]).astype(np.float32)
    pi = rng.dirichlet(np.ones(K), V).astype(np.float32)
    xs = t(x)
    ce.community_grad(xs, t(pi), t(mu), t(inv), 0.5 * K, 0.1, 1)
    mp = np.einsum("kd,kde->ke", mu, prec).astype(np.float32)
    ln = (-0.5 * d * np.log(2 * np.pi) + np.log(np.abs(np.diagonal(prec, axis1=1, axis2=2))).sum(1)
          + np.log(1.0 / K)).astype(np.float32)
    R = gmm.estep(t(x), t(prec), t(mp), t(ln))
    R = R[0] if isinstance(R, tuple) else R
    S = gmm.scatter(t(x), t(pi), t(mu))
    torch.cuda.synchronize()
    for name, v in (("community", xs), ("estep", R), ("scatter", S)):
        a = v.detach().cpu().numpy()
        print(name, a.shape, hashlib.sha256(a.tobytes()).hexdigest()[:16], float(np.abs(a).sum()))


if __name__ == "__main__":
    main()
