"""A/B of one GMM EM iteration at C4 (V = 1M, K = 50, d = 128) in one process, each arm as
GaussianMixture.fit's loop runs it (E-step, M-step, one host read of the lower bound):
  unfused -- _m_step + _set_params (torch Cholesky / triangular solve / einsum; its own sync on
             the Cholesky status),
  fused   -- _m_step_params (come_gmm_params: everything after the scatter in one launch; the
             Cholesky status read together with the lower bound).
Interleaved rounds; prints the median / min ms per iteration of each arm.

    python scripts/em_step_ab.py [--rounds 5] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import torch
    from come_amd import gmm
    dev = torch.device("cuda", 0)
    V, K, d = 1_000_000, 50, 128
    rng = np.random.RandomState(2)
    x = torch.from_numpy(rng.standard_normal((V, d)).astype(np.float32)).to(dev)
    A = rng.standard_normal((K, d, d)) / np.sqrt(d)
    cov = np.einsum("kij,klj->kil", A, A) + np.eye(d)[None] * 0.5
    mu = torch.from_numpy((rng.standard_normal((K, d)) * 0.5)).to(dev)
    w = np.random.RandomState(4).dirichlet(np.ones(K))
    gm = gmm.GaussianMixture(K, reg_covar=1e-5)
    gm._n_total = V
    t64 = lambda a: torch.as_tensor(np.asarray(a, np.float64), device=dev)  # noqa: E731
    start = (t64(w), mu.double(), t64(cov))

    def unfused():
        resp, lse = gmm.estep(x, gm._e_pc, gm._e_mp, gm._e_ln)
        gm._set_params(*gm._m_step(x, resp))
        return float(lse.double().sum())

    def fused():
        resp, lse = gmm.estep(x, gm._e_pc, gm._e_mp, gm._e_ln)
        info = gm._m_step_params(x, resp)
        lb_info = torch.stack([lse.double().sum(), (info != 0).any().double()]).cpu()
        assert lb_info[1] == 0
        return float(lb_info[0])

    res = {"unfused": [], "fused": []}
    lbs = {}
    for r in range(args.rounds + 1):
        for name, fn in (("unfused", unfused), ("fused", fused)):
            gm._set_params(*start)
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                lb = fn()
            torch.cuda.synchronize()
            if r:
                res[name].append((time.perf_counter() - t0) / args.steps * 1e3)
            lbs[name] = lb
    print(json.dumps({k: {"median_ms": round(float(np.median(v)), 4),
                          "min_ms": round(float(np.min(v)), 4)} for k, v in res.items()}))
    print(json.dumps({"lower_bound_after_steps": lbs,
                      "rel_diff": abs(lbs["fused"] - lbs["unfused"]) / abs(lbs["unfused"])}))


if __name__ == "__main__":
    main()
