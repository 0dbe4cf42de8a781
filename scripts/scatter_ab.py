"""Interleaved A/B of the GMM M-step scatter kernels at C4 (V = 1M, K = 50, d = 128) in ONE
process: each variant is a value of the launch option gmm_cov_async (3 = k_gmm_cov16 fp32,
4 = k_gmm_cov_fb3, 5 = k_gmm_cov_bf3); an alternative build goes in COME_LIB_PATH (one library
per process).
Per variant: median / min of the HIP-event time of gmm.scatter (kernel + chunk reduction) over
interleaved rounds, the max |diff| against the first variant relative to max |S|, a digest of the
output bytes (bit identity), and the RMS / max relative error against float64 on the first
`--check` components.

    python scripts/scatter_ab.py [--rounds 8] [--check 4] 4 5
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="*", type=int, default=[4, 5])
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--k", type=int, default=50)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--check", type=int, default=2, help="components checked against float64")
    args = ap.parse_args()
    import torch
    from come_amd import gmm, _lib
    dev = torch.device("cuda", 0)
    V, K, d = args.nodes, args.k, args.dim
    rng = np.random.RandomState(2)
    xh = rng.standard_normal((V, d)).astype(np.float32)
    rh = np.random.RandomState(3).dirichlet(np.ones(K), V).astype(np.float32)
    mh = (rng.standard_normal((K, d)) * 0.5).astype(np.float32)
    x, resp, mu = (torch.from_numpy(a).to(dev) for a in (xh, rh, mh))
    outs, times = {}, {v: [] for v in args.variants}
    st = torch.cuda.current_stream(dev)
    for r in range(args.rounds + 1):
        for v in args.variants:
            _lib.set_option("gmm_cov_async", v)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(st)
            out = gmm.scatter(x, resp, mu)
            e.record(st)
            torch.cuda.synchronize()
            if r:
                times[v].append(s.elapsed_time(e))
            else:
                outs[v] = out.cpu().numpy()
    _lib.set_option("gmm_cov_async", 4)
    ref64 = []
    for k in range(args.check):
        dk = xh.astype(np.float64) - mh[k].astype(np.float64)
        ref64.append((dk * rh[:, k:k + 1].astype(np.float64)).T @ dk)
    base = outs[args.variants[0]]
    for v in args.variants:
        o = outs[v]
        errs = [np.abs(o[k] - ref64[k]) / np.abs(ref64[k]).max() for k in range(args.check)]
        rel = np.concatenate([e.ravel() for e in errs])
        print(json.dumps({
            "gmm_cov_async": v, "median_ms": round(float(np.median(times[v])), 4),
            "min_ms": round(float(np.min(times[v])), 4),
            "max_rel_diff_vs_first": float(np.abs(o - base).max() / np.abs(base).max()),
            "digest": hashlib.sha256(o.tobytes()).hexdigest()[:16],
            "f64_rms_rel": float(np.sqrt(np.mean(rel ** 2))), "f64_max_rel": float(rel.max()),
            "tflops_executed": 2.0 * V * K * d * d * (10 / 16) / (np.median(times[v]) / 1e3) / 1e12}))


if __name__ == "__main__":
    main()
