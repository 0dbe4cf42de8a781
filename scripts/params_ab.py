"""Time come_gmm_params (k_gmm_params) at C4's shape (K = 50, d = 128) on random SPD scatter
matrices: median / min HIP-event ms per launch over `--reps` launches per round, and a digest of
prec_chol (bit identity across builds).  One library per process (COME_LIB_PATH for an
alternative build).

    python scripts/params_ab.py [--rounds 5] [--reps 50]
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import torch
    from come_amd import gmm
    dev = torch.device("cuda", 0)
    K, d = 50, 128
    rng = np.random.RandomState(5)
    A = rng.standard_normal((K, d, 3 * d))
    nk = rng.uniform(1e3, 1e5, K)
    S = np.einsum("kij,klj->kil", A, A) / (3 * d) * nk[:, None, None]
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    S_, nk_, mu_, w_ = t(S), t(nk), t(rng.standard_normal((K, d))), t(nk / nk.sum())
    out = gmm.params(S_, nk_, mu_, w_, 1e-5)
    torch.cuda.synchronize()
    assert int((out[5] != 0).sum()) == 0
    st = torch.cuda.current_stream(dev)
    times = []
    for r in range(args.rounds + 1):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(st)
        for _ in range(args.reps):
            gmm.params(S_, nk_, mu_, w_, 1e-5)
        e.record(st)
        torch.cuda.synchronize()
        if r:
            times.append(s.elapsed_time(e) / args.reps)
    print(json.dumps({"lib": os.environ.get("COME_LIB_PATH", "default"),
                      "median_ms": round(float(np.median(times)), 4),
                      "min_ms": round(float(np.min(times)), 4),
                      "pc_digest": hashlib.sha256(out[1].cpu().numpy().tobytes()).hexdigest()[:16],
                      "cov_digest": hashlib.sha256(out[0].cpu().numpy().tobytes()).hexdigest()[:16],
                      "e_mp_digest": hashlib.sha256(out[3].cpu().numpy().tobytes()).hexdigest()[:16]}))


if __name__ == "__main__":
    main()
