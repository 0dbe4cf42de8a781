"""Multi-rank combine rules on the CPU (TEST INFRASTRUCTURE for DESIGN.md §6): N ranks simulated in
one process, each training its contiguous walk shard with the oracle's Hogwild C restatement
(oracle/come_oracle_mt.c, the reference's worker pool), exchanging through the product's
DeltaAllReduce (distributed.LocalReplicas stands in for RCCL) -- the same protocol as
tests/replica_sim.py on the GPU, at a size one host finishes in seconds, so combine rules can be
screened without a GPU.  Baseline: the sequential oracle (threads=1) over the same walks.

    python scripts/replicas_cpu.py [--nodes 100000] [--walks 200000] [--worlds 2,4,8]
        [--periods 25000] [--combines touched_mean,pick] [--no-overlap] [--lr 0.1]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=100_000)
    ap.add_argument("--walks", type=int, default=200_000)
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--periods", default="25000")
    ap.add_argument("--combines", default="touched_mean,pick")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    from come_amd.distributed import DeltaAllReduce, LocalReplicas, shard_walks
    from come_amd.graph import chung_lu
    from oracle import oracle as orc
    from tierc_inputs import heldout_o2_pairs, sgns_loss
    t0 = time.time()
    g = chung_lu(args.nodes, 20.0, gamma=2.5, seed=21)
    table = orc.make_table(g.degree.astype(np.float64), 10_000_000)
    rng = np.random.RandomState(5)
    held_n = 20_000
    starts = rng.randint(0, g.V, args.walks + held_n).astype(np.int32)
    walks = orc.philox_walks(g.rowptr, g.col, starts, 80, 0.0, seed=22)
    train, held = walks[:args.walks], walks[args.walks:]
    node0 = rng.uniform(-1, 1, (g.V, args.dim)).astype(np.float32)
    seeds = rng.randint(0, 2 ** 48, args.walks, dtype=np.int64).astype(np.uint64)
    w, n = 5, 5
    ri, rp, rn = heldout_o2_pairs(held, w, n, table, 100_000, 24)
    cache = "/tmp/replicas_cpu_seq_%d_%d_%d_%g.json" % (args.nodes, args.walks, args.dim, args.lr)
    if os.path.exists(cache):
        l_seq = json.load(open(cache))["seq_loss"]
    else:
        sn, sc = node0.copy(), np.zeros_like(node0)
        orc.sgns_o2_hogwild(sn, sc, train, seeds, w, n, table, args.lr, 1.0, threads=1)
        l_seq = sgns_loss(sn, sc, ri, rp, rn)
        json.dump({"seq_loss": l_seq}, open(cache, "w"))
    print("inputs + sequential oracle %.0fs: seq loss %.5f (init %.5f)" % (
        time.time() - t0, l_seq, sgns_loss(node0, np.zeros_like(node0), ri, rp, rn)), flush=True)
    out = {"nodes": g.V, "walks": args.walks, "lr": args.lr, "seq_loss": l_seq,
           "overlap": not args.no_overlap, "points": []}
    for comb in args.combines.split(","):
        cname, lr_r = comb, args.lr
        for N in [int(v) for v in args.worlds.split(",")]:
            if cname.endswith("@lrN"):
                cname, lr_r = comb[:-4], args.lr * N
            for p in [int(v) for v in args.periods.split(",")]:
                t1 = time.time()
                group = LocalReplicas(N)
                reps, exs, shards = [], [], []
                for r in range(N):
                    nd, cx = node0.copy(), np.zeros_like(node0)
                    reps.append((nd, cx))
                    exs.append(DeltaAllReduce([torch.from_numpy(nd), torch.from_numpy(cx)],
                                              comm=group.comm(r), combine=cname))
                    shards.append(shard_walks(train, seeds, r, N))
                nb = max(1, -(-max(len(s) for _, s in shards) // p))
                for b in range(nb):
                    for r in range(N):
                        ws, ss = shards[r]
                        wb, sb = ws[b * p:(b + 1) * p], ss[b * p:(b + 1) * p]
                        if len(wb):
                            orc.sgns_o2_hogwild(reps[r][0], reps[r][1], wb, sb, w, n, table,
                                                lr_r, 1.0, threads=args.threads)
                    last = b + 1 == nb
                    for e in exs:
                        e.prepare()
                    for e in exs:
                        e.start()
                    if not args.no_overlap and not last and exs[0].overlap_safe:
                        continue
                    for e in exs:
                        e.finish()
                        e.settle()
                for r in range(1, N):
                    assert np.array_equal(reps[r][0], reps[0][0])
                loss = sgns_loss(reps[0][0], reps[0][1], ri, rp, rn)
                pt = {"world": N, "combine": comb, "period": p, "exchanges": exs[0].exchanges,
                      "loss": loss, "rel_to_seq": (loss - l_seq) / l_seq,
                      "wall_s": time.time() - t1}
                out["points"].append(pt)
                print(json.dumps(pt), flush=True)
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
