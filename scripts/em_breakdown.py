"""Per-piece GPU time of one GMM EM iteration at C4 (V=1M, K=50, d=128): E-step kernel, nk / means
GEMM, scatter kernel, covariance assembly, K Cholesky factorisations + triangular solves, E-step
parameter preparation (HIP events on the current stream)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from come_amd import gmm  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    V, K, d = 1_000_000, 50, 128
    rng = np.random.RandomState(2)
    X = torch.from_numpy(rng.standard_normal((V, d)).astype(np.float32)).to(dev)
    A = rng.standard_normal((K, d, d)) / np.sqrt(d)
    cov = np.einsum("kij,klj->kil", A, A) + np.eye(d)[None] * 0.5
    w = np.random.RandomState(4).dirichlet(np.ones(K))
    mu = rng.standard_normal((K, d)) * 0.5
    gm = gmm.GaussianMixture(K, reg_covar=1e-5)
    t64 = lambda a: torch.as_tensor(np.asarray(a, np.float64), device=dev)  # noqa: E731
    gm._set_params(t64(w), t64(mu), t64(cov))
    names = ["estep", "nk+means", "scatter", "cov", "set_params"]
    tot = {n: 0.0 for n in names}
    for it in range(6):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
        ev[0].record()
        resp, _ = gmm.estep(X, gm._e_pc, gm._e_mp, gm._e_ln)
        ev[1].record()
        nk = gmm.resp_sum(resp)
        sx = gmm.resp_t_x(resp, X)
        nk = nk + 1e-15
        means = sx / nk[:, None]
        ev[2].record()
        S = gmm.scatter(X, resp, means.float()).double()
        ev[3].record()
        c = S / nk[:, None, None] + 1e-5 * torch.eye(d, dtype=torch.float64, device=dev)
        ev[4].record()
        gm._set_params(nk / V, means, c)
        ev[5].record()
        torch.cuda.synchronize()
        if it >= 1:
            for i, n in enumerate(names):
                tot[n] += ev[i].elapsed_time(ev[i + 1]) / 5
    print({n: round(v, 3) for n, v in tot.items()}, "total", round(sum(tot.values()), 3))


if __name__ == "__main__":
    main()
