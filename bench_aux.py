"""Secondary benchmarks for the other hot-path rows (bench.py is the contract line for C3/O2).

  --workload c2   BASELINE configs[1]: O1 (node_embeddings) on a synthetic SBM, 100 blocks x 1000
                  nodes, ~1M edges, d=128, negative=5; a step = one Hogwild pass over all edges
                  (come_sgns_o1); metric pair-updates/s; roofline HBM, (3+n)*d*4 B per pair.
  --workload c4   BASELINE configs[3]: 1M nodes, K=50, d=128: the community-gradient pass
                  (come_community_grad, iters=1) and the GMM responsibility pass
                  (come_gmm_resp); each 2*V*K*d^2 flops; roofline = fp32 MFMA peak 157.3 TFLOP/s
                  (k_community_b16: the bf16 MFMA peak / 6, its six bf16 part products per MAC).
  --workload walks  SURVEY.md §8f row 1, the producer of C3's input: one corpus pass over the C3
                  graph (1M-node power law, every node starts one walk, length 80) on the HIP
                  walker (come_random_walks); metric walk-steps/s; roofline: the measured 1.70
                  random 128-B line reads per step against the Infinity-Cache random-gather rate
                  (8.6 TB/s; 24 algorithmic B per step reported beside it).  CPU baseline: the exact
                  CPython-stream walker (come_walks_reference, native restatement of
                  graph_utils.build_deepwalk_corpus) on host threads.
Each prints one JSON line.  CPU baselines on a bounded sample: O1 the builder's Hogwild C
restatement of train_o1 (oracle/come_oracle_mt.c; reported beside it as the reference-equivalent
rate, restatement / its calibrated speed-up over the reference's GIL-bound Node2Vec.train,
profiles/r02_cpu_calibration.json); C4 the reference's numpy Community2Vec.train loop restated in
oracle/oracle.py and sklearn predict_proba.  The reference itself never reaches the GPU box.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
HBM_PEAK_GBS = 8000.0
F32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: f32-input MFMA = f32 vector peak
BF16_MFMA_PEAK_TFLOPS = 16 * F32_MFMA_PEAK_TFLOPS  # dense bf16 MFMA (~2.5 PF), 16x the f32 rate


def log(*a):
    print("[bench_aux]", *a, file=sys.stderr, flush=True)


def timed(fn, steps, warmup):
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0), [a.elapsed_time(b) for a, b in ev]


def c2(args):
    import torch
    import come_amd.training_sdg_inner as tsi
    from come_amd.graph import sbm
    from come_amd.model import Model
    dev = torch.device("cuda", 0)
    g = sbm(100, 1000, 0.016, 4.04e-5, seed=0)
    np.random.seed(1234)
    m = Model(g.degree_by_id(), size=args.dim, table_size=args.table_size, k=100, device=dev)
    edges = torch.from_numpy(g.edges.astype(np.int32)).to(dev)
    E = edges.shape[0]
    np.random.seed(99)
    seeds = [torch.from_numpy(tsi.draw_seeds(E).view(np.int64)).to(dev)
             for _ in range(args.steps + args.warmup)]
    it = iter(range(10 ** 9))

    hot = m.hot_rows(args.hot_p)  # the product's Hogwild launch (Node2Vec.train)
    n_hot = 0 if hot is None else int(np.unpackbits(hot.cpu().numpy().view(np.uint8)).sum())

    table = m.table if args.plain_table else m.negative_table()  # the product's (packed) table

    def step():
        tsi.sgns_o1(m.node_embedding, edges, seeds[next(it) % len(seeds)], args.negative, table,
                    args.lr, tsi.MODE_HOGWILD, hot=hot)
    el, ks = timed(step, args.steps, args.warmup)
    pairs = 2 * E
    n, d = args.negative, args.dim
    bpp = (3 + n) * d * 4
    avg = float(np.mean(ks)) / 1e3
    cpu = None
    if not args.no_cpu_baseline:
        from oracle import oracle as orc
        node = m.node_embedding.cpu().numpy().copy()
        threads = orc.usable_cpus()
        try:
            o1_ratio = float(json.load(open(os.path.join(
                ROOT, "profiles", "r02_cpu_calibration.json")))["o1_ratio_restatement_over_cython"])
        except (OSError, ValueError, KeyError):
            o1_ratio = None
        np.random.seed(98)
        cs = tsi.draw_seeds(E)
        t0 = time.time()
        done = pairs_done = 0
        while time.time() - t0 < args.cpu_seconds:
            p, e = orc.sgns_o1_hogwild(node, g.edges.astype(np.int32), cs, n, m.table_host, args.lr,
                                       threads, max(0.1, args.cpu_seconds - (time.time() - t0)))
            pairs_done += p
            done += e
        cel = time.time() - t0
        cpu = {"value": pairs_done / cel, "unit": "pair-updates/s", "cores": threads,
               "kind": "port",
               "reference_equivalent_value": (pairs_done / cel / o1_ratio) if o1_ratio else None,
               "reference_equivalent_note": "value / %s = the reference's GIL-bound Node2Vec."
                                            "train rate on the same cores (calibrated ratio, "
                                            "profiles/r02_cpu_calibration.json)" % (
                                                "%.1f" % o1_ratio if o1_ratio else "n/a"),
               "sample": "builder's Hogwild C restatement of train_o1 (oracle/come_oracle_mt.c), "
                         "%d threads taking jobs of 150 edges; %d edges in %.1fs.  The "
                         "reference's Node2Vec.train is GIL-bound (one Python call per edge): "
                         "calibrated in the container, this restatement runs %s x the "
                         "reference's Cython train_o1 at 8 threads "
                         "(profiles/r02_cpu_calibration.json)" % (
                             threads, done, cel, "%.1f" % o1_ratio if o1_ratio else "n/a")}
    print(json.dumps({
        "metric": "O1 SGNS pair-updates/sec, SBM 100k nodes / 1M edges, d=128",
        "value": pairs * args.steps / el, "unit": "pair-updates/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True, "dtype": "f32", "data": "synthetic SBM (seed 0)",
        "config": {"workload": "configs[1]/C2: O1 over %d edges of a 100x1000 SBM, d=%d, "
                               "negative=%d, lr=%g" % (E, d, n, args.lr), "hot_rows": n_hot,
                   "negative_table": "uint32" if args.plain_table else "packed"},
        "roofline": {"bound": "hbm", "achieved": bpp * pairs / avg / 1e9, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": bpp * pairs / avg / 1e9 / HBM_PEAK_GBS,
                     "bytes_per_pair": bpp, "avg_kernel_ms": avg * 1e3},
        "cpu_baseline": cpu}))


def c4(args):
    """N = 1: the three kernels on all V rows.  N > 1 (torchrun, one rank per GPU):
    every rank owns V/N rows of the replicated tables; a community pass = the kernel on the rank's
    rows + one all-gather of the updated rows (RCCL), an EM iteration = local E-step + M-step with
    the sufficient statistics all-reduced (come_amd.gmm distributed=True).  value = all ranks'
    flops / max-over-ranks time (strong scaling: V is fixed)."""
    import torch
    import torch.distributed as dist
    from come_amd import community_embeddings as ce
    from come_amd.distributed import all_gather_rows, shard_range
    from oracle import oracle as orc
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.all_ranks_device0 else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
    V, K, d = args.nodes, args.k, args.dim
    lo, hi = shard_range(V, rank, world)
    rng = np.random.RandomState(2)
    x = torch.from_numpy(rng.standard_normal((V, d)).astype(np.float32)).to(dev)
    A = rng.standard_normal((K, d, d)) / np.sqrt(d)
    cov = np.einsum("kij,klj->kil", A, A) + np.eye(d)[None] * 0.5
    inv = torch.from_numpy(np.linalg.inv(cov.astype(np.float32)).astype(np.float32)).to(dev)
    mu = torch.from_numpy((rng.standard_normal((K, d)) * 0.5).astype(np.float32)).to(dev)
    pi = torch.from_numpy(np.random.RandomState(3).dirichlet(np.ones(K), V).astype(np.float32)
                          ).to(dev)
    w = np.random.RandomState(4).dirichlet(np.ones(K))
    pc, mp, ln = ce.gmm_resp_params(w, mu.cpu().numpy().astype(np.float64),
                                    orc.precision_cholesky(cov), dev)
    flops = 2.0 * V * K * d * d
    # fraction of the MFMA blocks executed on sklearn's upper-triangular precision factors: the
    # bf16-part E-step's 16-wide column tiles x 32-feature steps (k_gmm_resp_b16, 20 of 32 at
    # d = 128) or the fp32 form's 16-wide blocks (k_gmm_resp16t, 36 of 64); the scatter's
    # symmetric 32-wide (10 of 16, k_gmm_cov_bf3) / 16-wide (36 of 64, k_gmm_cov16) tiles
    from come_amd import _lib
    opts = _lib.launch_opts()
    ct = d // 32 if d in (64, 128) else 0
    tri = (ct * (ct + 1) / 2) / (ct * ct) if ct else 1.0
    ct16 = d // 16 if d in (64, 128) else 0
    tri16 = (ct16 * (ct16 + 1) / 2) / (ct16 * ct16) if ct16 else 1.0
    tri_resp = (tri16 if opts.gmm_resp16 == 2 else (ct * (ct + 1)) / (2 * ct * ct)) if ct16 \
        else 1.0
    tri_cov = (tri16 if opts.gmm_cov_async == 3 else tri) if ct16 else 1.0
    cov_kernel = {3: "k_gmm_cov16", 4: "k_gmm_cov_fb3" if d == 128 else "k_gmm_cov_bf3",
                  5: "k_gmm_cov_bf3"}[
        opts.gmm_cov_async] if ct16 else "VALU"
    comm_kernel = {2: "k_community16", 3: "k_community_b16"}[
        opts.community_async] if ct16 else "VALU"
    # k_community_b16 carries each fp32 operand as three bf16 parts and takes six part products
    # per multiply-add: its ceiling is the bf16 MFMA peak / 6, not the fp32 MFMA peak
    comm_bf3 = comm_kernel == "k_community_b16"
    comm_peak = BF16_MFMA_PEAK_TFLOPS / 6 if comm_bf3 else F32_MFMA_PEAK_TFLOPS
    resp_kernel = {2: "k_gmm_resp16t", 3: "k_gmm_resp_b16"}[
        opts.gmm_resp16] if ct16 else "VALU"
    x0 = x.clone()
    xs, pis, x0s = x[lo:hi], pi[lo:hi], x0[lo:hi]

    def community_pass():
        ce.community_grad(xs, pis, mu, inv, 0.01, 0.1, 1)
        if world > 1:
            all_gather_rows(x)
    if world > 1:  # kernel alone on the rank's rows (the exchange excluded)
        _, ks_k = timed(lambda: ce.community_grad(xs, pis, mu, inv, 0.01, 0.1, 1), args.steps,
                        args.warmup)
    el_g, ks_g = timed(community_pass, args.steps, args.warmup)
    el_r, ks_r = timed(lambda: ce.gmm_resp(x0s, pc, mp, ln), args.steps, args.warmup)
    tg, tr = float(np.mean(ks_g)) / 1e3, float(np.mean(ks_r)) / 1e3
    # one GMM EM iteration (come_amd.gmm: E-step kernel + means GEMM + scatter kernel + K
    # Cholesky factorisations), and the M-step scatter kernel alone
    from come_amd import gmm
    gm = gmm.GaussianMixture(K, reg_covar=1e-5, distributed=world > 1)
    gm._n_total = V
    t64 = lambda a: torch.as_tensor(np.asarray(a, np.float64), device=dev)  # noqa: E731
    gm._set_params(t64(w), mu.double(), t64(cov))
    resp0 = pis.contiguous()

    def em_iter():  # one iteration of GaussianMixture.fit's loop, its host read included
        resp, lse = gmm.estep(x0s, gm._e_pc, gm._e_mp, gm._e_ln)
        info = gm._m_step_params(x0s, resp)
        lb_info = torch.stack([lse.double().sum(), (info != 0).any().double()]).cpu()
        assert lb_info[1] == 0
    el_e, ks_e = timed(em_iter, args.steps, args.warmup)
    el_s, ks_s = timed(lambda: gmm.scatter(x0s, resp0, mu), args.steps, args.warmup)
    te, ts = float(np.mean(ks_e)) / 1e3, float(np.mean(ks_s)) / 1e3
    if world > 1:  # max over ranks of every per-step time
        tk = float(np.mean(ks_k)) / 1e3
        t = torch.tensor([tg, tr, te, ts, tk], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tg, tr, te, ts, tk = t.tolist()
        dist.barrier()
        if rank != 0:
            dist.destroy_process_group()
            return
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        S = 4000
        xs = x0[:S].cpu().numpy()
        t0 = time.time()
        orc.community_train(xs, pi[:S].cpu().numpy(), mu.cpu().numpy(), inv.cpu().numpy(),
                            0.01, 0.1, 1)
        cel = time.time() - t0
        blas = blas_threads()
        cpu = {"value": 2.0 * S * K * d * d / cel / 1e12, "unit": "TFLOP/s", "cores": 1,
               "kind": "port", "blas_threads": blas,
               "sample": "Community2Vec.train's numpy loop (community_embeddings.py:61-78, "
                         "restated op for op in oracle/oracle.py) on %d of the %d rows: "
                         "%.2fs -> %.0f s per full pass.  cores 1: the loop's time is numpy's "
                         "elementwise pi * inv_cov products and its stacked [150 x d x d] @ "
                         "[150 x d x 1] matmul, which numpy runs on the calling thread whatever "
                         "the BLAS pool (%s BLAS threads were available); the reference adds no "
                         "threading of its own" % (S, V, cel, cel * V / S, blas)}
        from sklearn.mixture import GaussianMixture as SkGMM
        S2 = 20000
        Xs = x0[:S2].cpu().numpy()
        sk = SkGMM(K, covariance_type="full", reg_covar=1e-5, max_iter=1, tol=0.0,
                   weights_init=w, means_init=mu.cpu().numpy().astype(np.float64),
                   precisions_init=np.linalg.inv(cov), random_state=0)
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            sk._check_parameters(Xs)
            sk._initialize_parameters(Xs, np.random.RandomState(0))
            t0 = time.time()
            lpn, lr = sk._e_step(Xs)
            sk._m_step(Xs, lr)
            sel = time.time() - t0
        cpu["gmm_em_iteration_sample"] = (
            "sklearn GaussianMixture E+M step (community_embeddings.py:27's estimator) on %d "
            "rows: %.2fs -> %.1f s per full-size iteration, its GEMMs on %s BLAS threads" % (
                S2, sel, sel * V / S2, blas))
        cpu["gmm_em_iteration_cores"] = blas
    dist_cfg = {}
    if world > 1:
        dist_cfg = {"community_kernel_only_ms": tk * 1e3,
                    "community_exchange": "all_gather_into_tensor of %d x %d fp32 rows (%s)" % (
                        V, d, args.dist_backend),
                    "em_exchange": "all-reduce of K + K d then K d^2 float64 statistics",
                    "parallelism": "row shard x%d, replicated tables" % world}
    print(json.dumps({
        "metric": "community gradient + GMM responsibilities, 1M nodes K=50 d=128",
        "value": flops / tg / 1e12, "unit": "TFLOP/s (community gradient pass)", "n_gpus": world,
        "scaling": "strong",
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": tg * 1e3,
        "higher_is_better": True, "dtype": "f32", "data": "synthetic N(0,1) rows, random SPD",
        "config": {"workload": "configs[3]/C4: V=%d K=%d d=%d" % (V, K, d),
                   "community_kernel": comm_kernel,
                   # what "f32" means for the bf16-part kernels (README)
                   "arithmetic": ("fp32 operands as three bf16 parts, six exact part products per "
                                  "multiply-add on bf16 MFMAs, fp32 accumulation; error vs "
                                  "float64 at the fp32 kernels' level (tests/test_gpu_c4.py)")
                                 if comm_bf3 else "fp32 MFMA (exact fp32 products)",
                   # E-step / scatter: 2 V K d^2 algorithmic flops, of which the kernels execute
                   # only the upper-triangular / symmetric blocks (fractions above)
                   "gmm_resp_kernel": resp_kernel, "gmm_resp_blocks_executed": tri_resp,
                   "gmm_resp_ms": tr * 1e3, "gmm_resp_tflops_effective": flops / tr / 1e12,
                   "gmm_resp_tflops_executed": flops * tri_resp / tr / 1e12,
                   "gmm_scatter_ms": ts * 1e3, "gmm_scatter_tflops_effective": flops / ts / 1e12,
                   "gmm_scatter_kernel": cov_kernel, "gmm_scatter_blocks_executed": tri_cov,
                   "gmm_scatter_tflops_executed": flops * tri_cov / ts / 1e12,
                   "gmm_em_iteration_ms": te * 1e3, **dist_cfg},
        "roofline": {"bound": "mfma", "achieved": flops / tg / 1e12 / world,
                     "peak": comm_peak, "unit": "TFLOP/s (per GPU)",
                     "peak_basis": ("bf16 MFMA peak %.1f / 6 part products per fp32 multiply-add"
                                    % BF16_MFMA_PEAK_TFLOPS) if comm_bf3 else "fp32 MFMA peak",
                     "frac": flops / tg / 1e12 / world / comm_peak,
                     "frac_of_fp32_mfma_peak": flops / tg / 1e12 / world / F32_MFMA_PEAK_TFLOPS,
                     "flops_per_pass": flops, "avg_kernel_ms": tg * 1e3},
        "cpu_baseline": cpu}))


def walks(args):
    import random
    import torch
    from come_amd import graph_utils as gu
    from come_amd.graph import chung_lu
    dev = torch.device("cuda", 0)
    g = chung_lu(args.nodes, 20.0, gamma=2.5, seed=1)
    L = 80
    rowptr = torch.from_numpy(g.rowptr).to(dev)
    col = torch.from_numpy(g.col.astype(np.int32)).to(dev)
    starts = torch.randperm(g.V, device=dev).int()
    out = torch.empty((g.V, L), dtype=torch.int32, device=dev)
    it = iter(range(10 ** 9))

    def step():
        gu.device_walks(rowptr, col, starts, L, alpha=0.0, seed=next(it), out=out)
    el, ks = timed(step, args.steps, args.warmup)
    steps_per_launch = float((out >= 0).sum().item() - g.V)  # moves (the start is not a step)
    avg = float(np.mean(ks)) / 1e3
    bps = 24  # algorithmic: rowptr pair + one col entry + the written entry
    # What bounds it: each step is a dependent chain of random 128-B line reads -- 1.70 requests
    # per step measured (profiles/r03_pmc_walks.json: rowptr line, col line, 17% L2 hits), served
    # by the Infinity Cache (rowptr + col = 88 MB at C3) -> priced against the guide's
    # Infinity-Cache random-gather rate
    req_bytes = 1.70 * 128
    ic_peak = 8600.0  # GB/s, MI355X_MICROARCH.md 'Indexed rows': 38 MB table, random rows (IC)
    cpu = None
    if not args.no_cpu_baseline:
        Gh = gu.Graph(np.arange(1, g.V + 1), g.rowptr, g.col.astype(np.int32), g.degree,
                      np.zeros((0, 2), np.int32))
        from oracle import oracle as orc
        threads = orc.usable_cpus()  # the cgroup quota (16 on the GPU box), not os.cpu_count()
        t0 = time.time()  # one full pass per stream, streams on parallel threads
        w = gu._corpus(Gh, [1] * threads, L, 0.0, [random.Random(s) for s in range(threads)],
                       threads=threads)
        cel = time.time() - t0
        moves = float((w >= 0).sum() - w.shape[0])
        cpu = {"value": moves / cel, "unit": "walk-steps/s", "cores": threads, "kind": "port",
               "sample": "exact CPython-stream walker (come_walks_reference, restating "
                         "graph_utils.build_deepwalk_corpus + __random_walk__), %d streams x one "
                         "pass of %d walks on %d host threads: %.1fs" % (threads, g.V, threads,
                                                                        cel)}
    print(json.dumps({
        "metric": "random-walk steps/sec, 1M-node power-law graph, walk length 80",
        "value": steps_per_launch * args.steps / el, "unit": "walk-steps/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True, "dtype": "int32", "data": "synthetic Chung-Lu (seed 1)",
        "config": {"workload": "walk corpus pass: V=%d, E=%d, L=%d, alpha=0" % (
            g.V, g.num_edges, L)},
        "roofline": {"bound": "infinity-cache gathers",
                     "achieved": req_bytes * steps_per_launch / avg / 1e9,
                     "peak": ic_peak, "unit": "GB/s",
                     "frac": req_bytes * steps_per_launch / avg / 1e9 / ic_peak,
                     "request_bytes_per_step": req_bytes,
                     "algorithmic_bytes_per_step": bps,
                     "algorithmic_frac_of_hbm": bps * steps_per_launch / avg / 1e9 / HBM_PEAK_GBS,
                     "avg_kernel_ms": avg * 1e3},
        "cpu_baseline": cpu}))


def blas_threads():
    """Threads of the BLAS pool numpy / scipy / sklearn run on in this process (threadpoolctl),
    None if it cannot tell."""
    try:
        from threadpoolctl import threadpool_info
        n = [i.get("num_threads") for i in threadpool_info() if i.get("user_api") == "blas"]
        return max(n) if n else None
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["c2", "c4", "walks"], required=True)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--negative", type=int, default=5)
    ap.add_argument("--table-size", type=int, default=100_000_000)
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--k", type=int, default=50)
    ap.add_argument("--lr", type=float, default=0.1)  # lr 0.1 for every config
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--hot-p", type=float, default=None,
                    help="c2: contended-row share (default training_sdg_inner.default_hot_share; "
                         "0 = no float-atomic rows)")
    ap.add_argument("--plain-table", action="store_true",
                    help="c2: draw negatives from the uint32 table instead of the product's "
                         "exact packed form (Model.negative_table)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="c4 with N > 1: nccl (= RCCL); gloo only to rehearse on one GPU")
    ap.add_argument("--all-ranks-device0", action="store_true",
                    help="rehearsal: every rank on cuda:0 (needs --dist-backend gloo)")
    ap.add_argument("--opt", action="append", default=[],
                    help="come_set_option knob, e.g. --opt o1_pipe=0 (A/B experiments)")
    args = ap.parse_args()
    if args.opt:
        from come_amd import _lib
        for kv in args.opt:
            k, v = kv.split("=")
            _lib.set_option(k, int(v))
    {"c2": c2, "c4": c4, "walks": walks}[args.workload](args)


if __name__ == "__main__":
    main()
