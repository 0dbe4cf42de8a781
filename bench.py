"""Benchmark: SGNS pair-updates/sec at d=128 on a 1M-node power-law graph (BASELINE.json metric,
configs[2] = SURVEY.md §8d C3), 1..8 MI355X, walk shard + periodic RCCL delta all-reduce.

One "step" = the product trainer (Context2Vec.train_rows) over a batch of `--walks-per-step`
random walks per rank already resident in HBM (default 1,048,576 = one corpus pass of the 1M-node
graph = the product's launch, Context2Vec.batch_walks): at N = 1 one O2 launch (come_sgns_o2,
Hogwild, one wavefront per walk); at N > 1 one launch per `--sync-walks` of the rank's walks, each
followed by the delta all-reduce of both embedding tables over RCCL (overlapped with the next
launch; the step's last exchange blocking).  The ranks train contiguous shards of ONE corpus
(weak scaling: per-rank work fixed).  Printed by rank 0: ONE JSON line (contract in the task statement), with
`roofline` (dominant kernel: achieved algorithmic HBM bytes / launch time vs the 8 TB/s peak) and,
at N = 1, `cpu_baseline` (the builder's Hogwild C restatement of the reference's CPU path, timed on
every core this process may use; its ratio to the reference's own Cython is calibrated in the
container, profiles/r02_cpu_calibration.json).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
def kernel_name(d, n):
    """The instantiation come_sgns_o2 launches for (d, negative) in Hogwild mode."""
    vec = 1 if d <= 64 else 2 if d <= 128 else 4 if d <= 256 else 8
    full = "true" if vec > 1 and d == 64 * vec else "false"
    maxn = 5 if n <= 5 else 10 if n <= 10 else 20
    return "come::k_sgns_o2_stream<%d, %s, %d>" % (vec, full, maxn)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def o2_pairs_of_lengths(lengths, w):
    """Pairs train_o2 makes on a walk of l valid leading entries (pyx:494-506)."""
    import torch
    l = lengths.long()
    full = 2 * w * l - w * (w + 1)
    small = l * (l - 1)
    return torch.where(l >= w + 1, full, small).sum()


def cpu_port_baseline(walks_np, seeds_np, node_np, ctx_np, table_np, window, neg, lr, seconds,
                      threads):
    """Time the builder's Hogwild C restatement of the reference's CPU path
    (oracle/come_oracle_mt.c: `threads` worker threads, one train_o2 walk per claim, plain racing
    row updates -- context_embeddings.py:72-102 + pyx:454-509) on this host's cores.  The
    reference itself never reaches the GPU box; the restatement's speed relative to the
    reference's Cython train_o2 driven by Python threads is measured in the container by
    scripts/calibrate_cpu.py (profiles/r02_cpu_calibration.json).  Returns (pairs/s, pairs,
    walks, seconds, isa)."""
    from oracle import oracle as orc
    t0 = time.time()
    pairs, done = orc.sgns_o2_hogwild(node_np, ctx_np, walks_np, seeds_np, window, neg, table_np,
                                      lr, 1.0, threads, seconds)
    el = time.time() - t0
    return pairs / el, pairs, done, el, int(orc.lib().oracle_mt_isa())


def secondary_rows(timeout_s=150):
    """The other hot-path rows measured on the same GPU after the timed region, each by
    bench_aux.py in a child process (one JSON line each, with its bounded CPU baseline: the O1
    Hogwild restatement for ~6 s plus its reference-equivalent rate, the reference's numpy
    community loop and one sklearn EM iteration on row samples; none for the walker):
    C2 O1 pass, C4 community pass + GMM E-step / M-step scatter / EM iteration, walker pass (CPU:
    the exact CPython-stream walker, one corpus pass per host thread), and one GPU's share of
    configs[4]/C5 (this script on the 10M-node graph at d = 256, n = 10: one 1,048,576-walk launch
    per step over full-size replicated tables, what each of C5's 8 ranks runs; CPU: the Hogwild
    restatement for 6 s over host copies of the full 20 GB of tables).  The C5 row's
    `roofline_frac` is the skip-adjusted fraction (SURVEY.md §8d's 24,576 B per pair counts every
    target row as written; at C5 most targets are skipped, so that model exceeds the bytes the
    launch must move and its fraction can pass 1 -- kept as `roofline_frac_all_targets_written`).
    Outside the timed region and never part of `value`; a failing row is reported as an error
    string."""
    import subprocess
    out = {}
    for wl in ("c2", "c4", "walks", "c5"):
        cmd = [sys.executable, os.path.join(ROOT, "bench_aux.py"), "--workload", wl,
               "--steps", "10", "--warmup", "2", "--cpu-seconds", "6"]
        if wl == "c5":
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--nodes", "10000000",
                   "--dim", "256", "--negative", "10", "--steps", "3", "--warmup", "1",
                   "--no-secondary", "--cpu-seconds", "6",
                   "--traffic-json", os.path.join(ROOT, "profiles", "traffic_c5.json")]
        t0 = time.time()
        try:
            r = subprocess.run(cmd, capture_output=True, text=True,
                               timeout=timeout_s * (2 if wl == "c5" else 1))
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            if r.returncode != 0 or not line:
                out[wl] = "error rc=%d: %s" % (r.returncode, r.stderr.strip()[-300:])
                continue
            j = json.loads(line[-1])
            row = {"metric": j["metric"], "value": j["value"], "unit": j["unit"],
                   "ms_per_step": j["ms_per_step"], "workload": j["config"]["workload"],
                   "roofline_frac": j["roofline"]["frac"], "roofline_bound": j["roofline"]["bound"],
                   "avg_kernel_ms": j["roofline"]["avg_kernel_ms"], "wall_s": time.time() - t0,
                   "cpu_baseline": j.get("cpu_baseline")}
            if wl == "c5":
                rf = j["roofline"]
                # the skip (pyx:141) leaves more targets unwritten as training proceeds: the row
                # says which launches it timed and how many target rows they wrote per pair
                row["timed_launches"] = j["config"].get("timed_launches")
                row["target_updates_per_pair"] = rf.get("target_updates_per_pair")
                row["roofline_frac"] = rf["frac_skip_adjusted"]
                row["roofline_frac_all_targets_written"] = rf["frac"]
                row["bytes_per_pair_skip_adjusted"] = rf["bytes_per_pair_skip_adjusted"]
                row["achieved_GBps_skip_adjusted"] = rf["achieved_skip_adjusted"]
                row["traffic"] = rf.get("traffic")
                if rf.get("traffic"):
                    row["traffic_GBps"] = rf["traffic"] / (rf["avg_kernel_ms"] / 1e3) / 1e9
            if wl == "c4":
                row["community_kernel"] = j["config"]["community_kernel"]
                row["arithmetic"] = j["config"].get("arithmetic")
                row["roofline_peak"] = j["roofline"]["peak"]
                row["roofline_peak_basis"] = j["roofline"].get("peak_basis")
                row["frac_of_fp32_mfma_peak"] = j["roofline"].get("frac_of_fp32_mfma_peak")
                for k in ("gmm_resp_kernel", "gmm_resp_ms", "gmm_resp_tflops_executed",
                          "gmm_scatter_ms",
                          "gmm_scatter_tflops_executed", "gmm_em_iteration_ms"):
                    row[k] = j["config"][k]
            out[wl] = row
        except subprocess.TimeoutExpired:
            out[wl] = "error: timed out after %ds" % timeout_s
    return out


def c5_multi_gpu_row(args, rank, world, timeout_s=240):
    """configs[4]/C5 at this job's N GPUs (BASELINE: 10M nodes / 100M edges, d = 256, n = 10,
    8 x MI355X): every rank starts this script as a child on the 10M-node graph -- its own
    process group (same RANK / WORLD_SIZE, MASTER_PORT + 1), the product's distributed trainer,
    1M walks per rank per step, the dense overlapped exchange of both 10.24 GB tables -- after
    the C3 timed region.  Outside `value`; rank 0 returns the child's line as a row (an error
    string if it failed or timed out), the other ranks None."""
    import subprocess
    env = dict(os.environ)
    env["MASTER_PORT"] = str(int(os.environ.get("MASTER_PORT", "29500")) + 1)
    # torch.distributed.run tells its workers to join the agent's store on MASTER_PORT; the
    # children's group has no agent, so rank 0's child hosts its own store on MASTER_PORT + 1
    env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--nodes",
           str(args.c5_nodes), "--dim", "256", "--negative", "10", "--steps", "3", "--warmup", "1",
           "--no-secondary", "--no-cpu-baseline", "--dist-backend", args.dist_backend,
           "--traffic-json", os.path.join(ROOT, "profiles", "traffic_c5.json")]
    if args.all_ranks_device0:
        cmd.append("--all-ranks-device0")
    t0 = time.time()
    try:
        # stdout carries the child's JSON line; its stderr (progress) passes through
        r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return "error: timed out after %ds" % timeout_s if rank == 0 else None
    if rank != 0:
        return None
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode != 0 or not line:
        return "error rc=%d (the child's stderr is in this job's log)" % r.returncode
    j = json.loads(line[-1])
    rf = j["roofline"]
    return {"metric": j["metric"], "value": j["value"], "unit": j["unit"], "n_gpus": j["n_gpus"],
            "ms_per_step": j["ms_per_step"], "workload": j["config"]["workload"],
            "parallelism": j["config"]["parallelism"], "scaling": j["scaling"],
            "quality": j["config"].get("quality"),
            "timed_launches": j["config"].get("timed_launches"),
            "target_updates_per_pair": rf.get("target_updates_per_pair"),
            "roofline_frac": rf["frac_skip_adjusted"],
            "roofline_frac_all_targets_written": rf["frac"],
            "avg_kernel_ms": rf["avg_kernel_ms"], "wall_s": time.time() - t0}


def multi_rank_quality(world, combine, sync_walks, d, n):
    """The held-out-loss cost of the N > 1 exchange: the trainers' multi-rank mode
    is NOT the reference's trajectory (no periodic exchange of N replicas meets tier C at lr 0.1),
    so an N > 1 line is not like-for-like with the 1-GPU parity run.  Returns the measured
    deviation of the held-out SGNS loss from the sequential oracle's for this N, combine and
    period, from the one-GPU replica simulation over C3's 4,194,304-walk fixture
    (profiles/r04_tierc_replicas_c3_4m.json, guarded by tests/test_gpu_tierc.py
    test_o2_default_period_over_4m_walks), or None where that was not measured."""
    q = {"parity": "non-parity", "heldout_loss_rel_to_sequential_oracle": None,
         "basis": None}
    src = os.path.join(ROOT, "profiles", "r04_tierc_replicas_c3_4m.json")
    try:
        pts = json.load(open(src))["points"]
    except (OSError, ValueError, KeyError):
        pts = []
    hit = [p for p in pts if p.get("world") == world and p.get("combine") == combine
           and p.get("sync_walks") == sync_walks]
    if hit and d == 128 and n == 5:
        q["heldout_loss_rel_to_sequential_oracle"] = hit[0]["rel_to_seq"]
        q["basis"] = ("C3 4,194,304-walk fixture, %d ranks simulated on one GPU, %s, %d walks per "
                      "rank between exchanges (%d exchanges): held-out SGNS loss %+.1f%% vs the "
                      "sequential oracle (lower: less SGD noise than the reference's trajectory); "
                      "profiles/r04_tierc_replicas_c3_4m.json" % (
                          world, combine, sync_walks, hit[0]["exchanges"],
                          100 * hit[0]["rel_to_seq"]))
    else:
        q["basis"] = ("not measured for d=%d, n=%d, %d ranks, %s, %d walks per exchange; at C3's "
                      "shape the same exchange trains 12-19%% below the sequential oracle's "
                      "held-out loss (DESIGN.md §6)" % (d, n, world, combine, sync_walks))
    return q


def calibration_ratio():
    try:
        c = json.load(open(os.path.join(ROOT, "profiles", "r02_cpu_calibration.json")))
        return float(c["ratio_restatement_over_cython"]), int(c["threads"])
    except (OSError, ValueError, KeyError):
        return None, None


def measure_sparse_sync(model, step, s, dev):
    """One more training step from a snapshot, then the row-sparse exchange's local passes on
    this GPU (come_delta_flags over both tables, the row compaction, come_delta_gather and
    come_delta_scatter): rows changed per table and bytes an all-reduce would move per sync,
    sparse vs dense, with HIP-event times of the passes.  The all-reduce itself
    needs N > 1 (RCCL over xGMI)."""
    import torch
    from come_amd import _lib
    from come_amd._lib import check, ptr, stream_handle
    tabs = [model.node_embedding, model.context_embedding]
    snaps = [t.clone() for t in tabs]
    step(s)
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    st = stream_handle(dev)
    ev[0].record()
    flags = []
    for t, sn in zip(tabs, snaps):
        f = torch.empty(t.shape[0], dtype=torch.uint8, device=dev)
        check(_lib.lib().come_delta_flags(ptr(t), ptr(sn), t.shape[0], t.shape[1], ptr(f), st),
              "come_delta_flags")
        flags.append(f)
    ev[1].record()
    idx = [torch.nonzero(f).view(-1) for f in flags]
    bufs = [(t.new_empty((i.numel(), t.shape[1])), t.new_empty((i.numel(), t.shape[1])))
            for t, i in zip(tabs, idx)]
    torch.cuda.synchronize(dev)
    ev[2].record()
    for t, sn, i, (ds, do) in zip(tabs, snaps, idx, bufs):
        check(_lib.lib().come_delta_gather(ptr(t), ptr(sn), ptr(i), i.numel(), t.shape[1],
                                           ptr(ds), ptr(do), st), "come_delta_gather")
        check(_lib.lib().come_delta_scatter(ptr(t), ptr(sn), ptr(i), i.numel(), t.shape[1],
                                            ptr(ds), ptr(do), st), "come_delta_scatter")
    ev[3].record()
    torch.cuda.synchronize(dev)
    rows = [int(i.numel()) for i in idx]
    d = tabs[0].shape[1]
    dense = sum(t.numel() * 4 for t in tabs)
    sparse = sum(r * d * 4 for r in rows)
    return {"rows_changed": {"node": rows[0], "context": rows[1]}, "rows_total": tabs[0].shape[0],
            "bytes_per_sync_sparse": sparse, "bytes_per_sync_dense": dense,
            "flags_ms": ev[0].elapsed_time(ev[1]), "gather_scatter_ms": ev[2].elapsed_time(ev[3]),
            "note": "one step's changes; all-reduce payload per rank; replicas per rank: dense "
                    "3 full copies (sync base + 2 exchange buffers), sparse 1 + [rows x d]"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--mean-degree", type=float, default=20.0)  # -> ~10M undirected edges
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--negative", type=int, default=5)
    ap.add_argument("--window", type=int, default=5)
    ap.add_argument("--walk-length", type=int, default=80)
    # one step = one product launch: Context2Vec.batch_walks (1 << 20) walks, i.e. one C3 corpus
    # pass (every node starts one walk).  Walks in flight are bounded by the resident wavefronts
    # (8,192), not by the batch; a smaller batch only adds launch tails (ms per 1e8 pairs at
    # 65k / 131k / 262k walks per launch: 106.3 / 104.8 / 102.1, profiles/r03_ab_batch.txt)
    ap.add_argument("--walks-per-step", type=int, default=1 << 20)
    ap.add_argument("--table-size", type=int, default=100_000_000)
    ap.add_argument("--lr", type=float, default=0.1)  # lr 0.1, alpha 1
    ap.add_argument("--sync-walks", type=int, default=None,
                    help="N>1: walks each rank trains between two delta exchanges (default "
                         "context_embeddings.DEFAULT_SYNC_WALKS)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every CPU this process may use (affinity and cgroup quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary rows (N=1: C2 / C4 / walker via bench_aux.py and one "
                         "GPU's share of C5; N>1: C5 on the job's N GPUs)")
    ap.add_argument("--c5-nodes", type=int, default=10_000_000,
                    help="N>1: nodes of the C5 secondary row's graph (configs[4]: 10M; smaller "
                         "only to rehearse the multi-process plumbing, e.g. over gloo on one GPU)")
    ap.add_argument("--combine", default="touched_mean",
                    help="N>1: delta exchange combine rule (DeltaAllReduce; DESIGN.md §6)")
    ap.add_argument("--sparse-sync", action="store_true",
                    help="N>1: exchange only the rows some rank changed (SparseDeltaAllReduce)")
    ap.add_argument("--measure-sync", action="store_true",
                    help="N=1: after the timed steps, measure the row-sparse exchange's local "
                         "passes for one step (rows changed, bytes per sync, pass times)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N>1: blocking delta all-reduce instead of overlapping it with the next "
                         "batch")
    ap.add_argument("--plain-table", action="store_true",
                    help="draw negatives from the reference's uint32 table instead of its exact "
                         "packed form (come_pack_table; the product's default, Model."
                         "negative_table)")
    ap.add_argument("--hot-p", type=float, default=None,
                    help="rows holding >= this share of the negative table are updated with "
                         "float atomics (default training_sdg_inner.default_hot_share(d); "
                         "0 = none)")
    ap.add_argument("--opt", action="append", default=[],
                    help="per-call launch option k=v (come_launch_opts field), for A/B runs")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--all-ranks-device0", action="store_true",
                    help="rehearsal: every rank on cuda:0 (needs --dist-backend gloo)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import come_amd.training_sdg_inner as tsi
    from come_amd.context_embeddings import DEFAULT_SYNC_WALKS, Context2Vec
    from come_amd.graph import chung_lu, random_walks

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("warning: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    if args.all_ranks_device0:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    # ---- workload: C3.  Same graph on every rank; ONE corpus of world x (warmup + steps) x B
    # walks (every pass a fresh permutation of the start nodes, graph_utils.py:187-192) with one
    # seed per walk, sharded contiguously over the ranks: rank r generates exactly its shard's
    # walks (the walker's Philox counter is the walk's global index) ----
    t0 = time.time()
    g = chung_lu(args.nodes, args.mean_degree, gamma=2.5, seed=1, device=dev)  # == host build
    V, d, n, w, L = g.V, args.dim, args.negative, args.window, args.walk_length
    from come_amd.model import Model
    np.random.seed(1234)
    model = Model(g.degree_by_id(), size=d, table_size=args.table_size, k=1, device=dev)
    if rank == 0:
        log("graph V=%d E=%d (%.1fs); tables %.0f MB each; negative table %.0f MB" % (
            V, g.num_edges, time.time() - t0, V * d * 4 / 1e6, args.table_size * 4 / 1e6))
    B = args.walks_per_step
    total_steps = args.warmup + args.steps
    per_rank = total_steps * B
    lo = rank * per_rank
    gen = torch.Generator(device=dev)
    gen.manual_seed(100)
    passes = (world * per_rank + V - 1) // V
    starts = torch.cat([torch.randperm(V, generator=gen, device=dev) for _ in range(passes)])
    walks_all = random_walks(g, 0, L, seed=100, device=dev,
                             starts=starts[lo:lo + per_rank], walk_offset=lo).contiguous()
    del starts
    gen.manual_seed(5678)
    seeds_all = torch.randint(0, 2 ** 48, (world * per_rank,), generator=gen, device=dev,
                              dtype=torch.int64)[lo:lo + per_rank].contiguous()
    lengths = (walks_all >= 0).sum(dim=1)
    pairs_per_step = [int(o2_pairs_of_lengths(lengths[s * B:(s + 1) * B], w))
                      for s in range(total_steps)]
    sync_walks = args.sync_walks or DEFAULT_SYNC_WALKS
    # the product's trainer (Context2Vec.train_rows = what Context2Vec.train runs after mapping
    # the corpus): one launch per batch_walks at N = 1; at N > 1 one launch per sync_walks of
    # the rank's shard, each followed by the delta exchange (overlapped with the next launch, the
    # last one blocking)
    opts = {k: int(v) for k, v in (o.split("=", 1) for o in args.opt)} or None
    hot_p = tsi.default_hot_share(d) if args.hot_p is None else args.hot_p
    learner = Context2Vec(lr=args.lr, window_size=w, negative=n, batch_walks=B,
                          distributed=world > 1, sync_walks=sync_walks,
                          sparse_sync=args.sparse_sync, overlap=not args.no_overlap,
                          hot_share=hot_p, launch_opts=opts, combine=args.combine)
    if args.plain_table:
        model.use_packed_table = False
    neg_table = model.negative_table()
    table_kind = "packed" if isinstance(neg_table, tsi.PackedTable) else "uint32"

    # target-row updates applied by the timed launches (the +-6 skip, pyx:141, leaves a target
    # row unwritten, so the bytes a launch must move depend on the data): counted in-kernel
    upd_count = torch.zeros(1, dtype=torch.int64, device=dev)
    hot = model.hot_rows(hot_p)
    n_hot = 0 if hot is None else int(np.unpackbits(hot.cpu().numpy().view(np.uint8)).sum())

    def step(s, count=False, events=None):
        learner.train_rows(model, walks_all[s * B:(s + 1) * B], seeds_all[s * B:(s + 1) * B],
                           1.0, update_count=upd_count if count else None,
                           launch_events=events)

    stream = torch.cuda.current_stream(dev)
    for s in range(args.warmup):
        step(s)
        if rank == 0:
            log("warm-up step %d of %d enqueued" % (s + 1, args.warmup))
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    if rank == 0:
        log("warm-up done (%d steps); timing %d steps" % (args.warmup, args.steps))
    ev = []
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k, count=True, events=ev)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    launches_per_step = len(ev) / args.steps

    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        pt = torch.tensor([sum(pairs_per_step[args.warmup:])], dtype=torch.float64, device=dev)
        dist.all_reduce(pt, op=dist.ReduceOp.SUM)
        total_pairs = float(pt.item())
    else:
        total_pairs = float(sum(pairs_per_step[args.warmup:]))

    assert torch.isfinite(model.node_embedding).all() and torch.isfinite(
        model.context_embedding).all(), "non-finite embedding after training"

    c5_multi = None
    if world > 1 and not args.no_secondary:
        c5_multi = c5_multi_gpu_row(args, rank, world)
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    # SURVEY.md §8d algorithmic bytes per pair: the input row read + written and the (1+n) output
    # rows read + written = 2 (2+n) d 4 (7,168 B at d=128, n=5) -- `achieved` / `frac`.  Beside
    # it, skip-adjusted: a target whose |dot| >= 6 is skipped (pyx:141) and its row is read but
    # not written, so a launch must move pairs * (3+n) d 4 (reads + the unconditional input write,
    # pyx:149) + updates * d 4, `updates` counted in-kernel (come_launch_opts.o2_update_count).
    bytes_per_pair_max = 2 * (2 + n) * d * 4
    pairs_rank_step = float(np.mean(pairs_per_step[args.warmup:]))
    updates_rank_step = float(upd_count.item()) / args.steps
    pairs_launch = pairs_rank_step / launches_per_step
    alg_bytes_step = pairs_rank_step * (3 + n) * d * 4 + updates_rank_step * d * 4
    bytes_per_pair = alg_bytes_step / pairs_rank_step
    avg_kernel_s = float(np.mean(kern_ms)) / 1e3
    achieved = pairs_launch * bytes_per_pair_max / avg_kernel_s / 1e9
    achieved_skip = pairs_launch * bytes_per_pair / avg_kernel_s / 1e9
    walks_per_launch = B if world == 1 else min(B, sync_walks)
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if (tj.get("walks_per_launch") == walks_per_launch and tj.get("dim") == d
                    and tj.get("negative") == n and tj.get("lr") == args.lr
                    and tj.get("negative_table", "uint32") == table_kind
                    and kernel_name(d, n).replace(" ", "") in
                    tj.get("kernel", "").replace(" ", "")):
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as orc
        sample = min(400_000, walks_all.shape[0])  # more than --cpu-seconds can finish
        wn = walks_all[:sample].cpu().numpy()
        sn = seeds_all[:sample].cpu().numpy().view(np.uint64)
        node_h = np.ascontiguousarray(model.node_embedding.cpu().numpy())
        ctx_h = np.ascontiguousarray(model.context_embedding.cpu().numpy())
        threads = args.cpu_threads if args.cpu_threads > 0 else orc.usable_cpus()
        rate, cp, cw, cel, isa = cpu_port_baseline(wn, sn, node_h, ctx_h, model.table_host, w, n,
                                                   args.lr, args.cpu_seconds, threads)
        ratio, rthreads = calibration_ratio()
        cpu = {"value": rate, "unit": "pair-updates/s", "cores": threads, "kind": "port",
               "nproc": orc.usable_cpus(), "visible_cpus": os.cpu_count(),
               "sample": "builder's Hogwild C restatement of the reference CPU path "
                         "(oracle/come_oracle_mt.c, %s build): %d threads taking jobs of 150 "
                         "walks, one train_o2 per walk, as Context2Vec's workers; %d walks / %d "
                         "pair-updates of this "
                         "workload (same graph, walks, seeds, tables, negative table) in %.1fs. "
                         "Calibration (profiles/r02_cpu_calibration.json, container, %s "
                         "threads): restatement / reference Cython train_o2 = %s" % (
                             "AVX2+FMA" if isa else "baseline-ISA", threads, cw, cp, cel,
                             rthreads, "%.3f" % ratio if ratio else "n/a")}

    secondary = {"c5": c5_multi} if c5_multi is not None else None
    if world == 1 and not args.no_secondary:
        log("secondary rows (bench_aux.py c2 / c4 / walks, bench.py C5 shard; outside the timed region)")
        secondary = secondary_rows()

    sync_measure = None
    if world == 1 and args.measure_sync:
        sync_measure = measure_sparse_sync(model, step, args.warmup, dev)

    value = total_pairs / elapsed
    out = {
        "metric": "SGNS pair-updates/sec at d=%d, %s-node graph" % (
            d, "1M" if V == 1_000_000 else "%gM" % (V / 1e6)),
        "value": value,
        "unit": "pair-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: Chung-Lu power-law graph (gamma 2.5) + uniform random walks, "
                "tables initialised as the reference (node U(-1,1), ctx 0)",
        "config": {
            "workload": "%s: O2 SGNS over random walks, power-law %d nodes / %d "
                        "edges, d=%d, negative=%d, window=%d, walk_length=%d, table_size=%d, lr=%g, "
                        "alpha=1" % (
                            ("configs[4]/C5 (one GPU's shard)" if world == 1
                             else "configs[4]/C5 on %d GPUs" % world) if d == 256 and n == 10
                            else "configs[2]/C3", V, g.num_edges, d, n, w, L, args.table_size,
                            args.lr),
            "walks_per_step_per_gpu": B,
            "launch_opts": opts,
            "hot_rows": {"share_threshold": hot_p, "rows": n_hot},
            "negative_table": table_kind,
            "pairs_per_step_per_gpu": pairs_rank_step,
            "walks_per_launch": walks_per_launch,
            "sync_walks_per_rank": sync_walks if world > 1 else None,
            "exchange_combine": args.combine if world > 1 else None,
            "quality": (multi_rank_quality(world, args.combine, sync_walks, d, n) if world > 1
                        else {"parity": "tier C (held-out loss within 1% of the sequential "
                                        "oracle: tests/test_gpu_tierc.py)"}),
            "timed_launches": "launches %d-%d of a fresh run (tables from the reference's init, "
                              "model.py:86-87; %d untimed warm-up launches before them)" % (
                                  int(args.warmup * launches_per_step) + 1,
                                  int((args.warmup + args.steps) * launches_per_step),
                                  int(args.warmup * launches_per_step)),
            "exchanges_per_step": (-(-B // sync_walks)) if world > 1 else 0,
            "trainer": "Context2Vec.train_rows (distributed=%s)" % (world > 1),
            "corpus": "one corpus of %d walks (%d per rank), sharded contiguously" % (
                world * per_rank, per_rank),
            "parallelism": "walk-shard dp%d + %s delta all-reduce (%s)" % (
                world, "blocking" if args.no_overlap else "overlapped",
                "RCCL" if args.dist_backend == "nccl" else args.dist_backend)
            if world > 1 else "single GPU, Hogwild over walks",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel": kernel_name(d, n),
            "bytes_per_pair": bytes_per_pair_max,
            "achieved_skip_adjusted": achieved_skip,
            "frac_skip_adjusted": achieved_skip / HBM_PEAK_GBS,
            "bytes_per_pair_skip_adjusted": bytes_per_pair,
            "pairs_per_launch": pairs_launch,
            "target_updates_per_pair": updates_rank_step / pairs_rank_step,
            "avg_kernel_ms": avg_kernel_s * 1e3,
        },
        "cpu_baseline": cpu,
    }
    if secondary is not None:
        out["secondary"] = secondary
    if sync_measure is not None:
        out["sync_measure"] = sync_measure
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
