"""One GMM kernel alone at C4 (V = 1M, K = 50, d = 128) for A/B builds (scripts/ab.sh
"name:COME_LIB_PATH=..."): the M-step scatter (--op scatter) or the E-step (--op estep, sklearn-
style upper-triangular precision factors).  Prints one JSON line with the average time over
--steps calls (HIP events on the launch stream; the scatter's includes its partial reduction, the
E-step's the small flag / transpose / pack launches), the executed TFLOP/s (36 of 64 16-wide
blocks) and a digest of the output bytes (bit-identity across builds).

    python scripts/gmm_ab.py [--op scatter|estep] [--steps 20] [--chunks 0]
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
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--k", type=int, default=50)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--chunks", type=int, default=0, help="0 = gmm.scatter's default")
    ap.add_argument("--op", choices=["scatter", "estep"], default="scatter")
    ap.add_argument("--opt", action="append", default=[], help="come_set_option knob, k=v")
    args = ap.parse_args()
    import torch
    from come_amd import gmm
    import come_amd.community_embeddings as ce
    from oracle import oracle as orc
    from come_amd import _lib
    for kv in args.opt:
        k, v = kv.split("=")
        _lib.set_option(k, int(v))
    dev = torch.device("cuda", 0)
    V, K, d = args.nodes, args.k, args.dim
    rng = np.random.RandomState(2)
    x = torch.from_numpy(rng.standard_normal((V, d)).astype(np.float32)).to(dev)
    mu = torch.from_numpy((rng.standard_normal((K, d)) * 0.5).astype(np.float32)).to(dev)
    resp = torch.from_numpy(np.random.RandomState(3).dirichlet(np.ones(K), V).astype(np.float32)
                            ).to(dev)
    ch = args.chunks or None
    if args.op == "estep":
        A = rng.standard_normal((K, d, d)) / np.sqrt(d)
        cov = np.einsum("kij,klj->kil", A, A) + np.eye(d)[None] * 0.5
        w = np.random.RandomState(4).dirichlet(np.ones(K))
        pc, mp, ln = ce.gmm_resp_params(w, mu.cpu().numpy().astype(np.float64),
                                        orc.precision_cholesky(cov), dev)
        call = lambda: ce.gmm_resp(x, pc, mp, ln)  # noqa: E731
    else:
        call = lambda: gmm.scatter(x, resp, mu, chunks=ch)  # noqa: E731
    for _ in range(args.warmup):
        out = call()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.steps)]
    ms = []
    for i in range(args.steps):
        ev[2 * i].record(st)
        out = call()
        ev[2 * i + 1].record(st)
    torch.cuda.synchronize()
    ms = [ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(args.steps)]
    t = float(np.mean(ms)) / 1e3
    flops = 2.0 * V * K * d * d * (36 / 64 if d == 128 else 10 / 16)
    if isinstance(out, tuple):
        out = out[0]
    dig = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"metric": args.op, "ms_per_step": t * 1e3, "value": flops / t / 1e12,
                      "unit": "TFLOP/s executed", "frac": flops / t / 157.3e12,
                      "chunks": args.chunks, "digest": dig,
                      "roofline": {"avg_kernel_ms": t * 1e3, "frac": flops / t / 157.3e12}}))


if __name__ == "__main__":
    main()
