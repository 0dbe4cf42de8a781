"""Tier C of the multi-GPU SGNS path (SURVEY.md §8c applied to §8e): N ranks simulated on one GPU
(tests/replica_sim.py: the product's launches, DeltaAllReduce arithmetic and overlapped protocol;
RCCL replaced by a sum over the replicas) against the sequential oracle's held-out loss after the
same walks, for N = 1, 2, 4, 8 and a range of sync periods (walks per rank between exchanges).

    python scripts/tierc_replicas.py --fixture c3_1m [--worlds 1,2,4,8] [--periods ...]
    python scripts/tierc_replicas.py --fixture c3_131k
    python scripts/tierc_replicas.py --fixture c2 [--passes 1] [--periods 0,131072,...]

c2:      configs[1]/C2 (O1): the 100k-node SBM's edges in G.edges() order (node_embeddings.py:39),
         2% held out; N ranks of Node2Vec(distributed=True) (replica_sim.train_replicas_o1), the
         sequential oracle computed here (one core, ~1 s per pass); period = edges per rank
         between exchanges (0 = one exchange per pass, Node2Vec's default)

c3_1m:   configs[2]/C3, 1,048,576 walks (tests/golden/tierc_c3_1m_seq.json, host-built inputs)
c3_131k: configs[2]/C3, 131,072 walks (tests/golden/tierc_c3_seq.json, device-walker inputs)
Writes one JSON line per point and the whole curve to --out.
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
    ap.add_argument("--fixture", choices=["c3_1m", "c3_4m", "c3_131k", "c2"], default="c3_1m")
    ap.add_argument("--passes", type=int, default=1, help="c2: passes over the edges (iter)")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--periods", default="")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--combines", default="touched_mean",
                    help="comma list of combine rules; a '@lrN' suffix trains every rank with lr "
                         "x N (e.g. mean@lrN)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    import come_amd.training_sdg_inner as tsi
    if args.fixture == "c2":
        return main_o1(args)
    from replica_sim import train_replicas
    from tierc_inputs import sgns_loss, heldout_o2_pairs, c3_1m_inputs
    t0 = time.time()
    if args.fixture in ("c3_1m", "c3_4m"):
        from tierc_inputs import c3_4m_inputs
        fx = json.load(open(os.path.join(ROOT, "tests", "golden",
                                         "tierc_%s_seq.json" % args.fixture)))
        x = c3_1m_inputs() if args.fixture == "c3_1m" else c3_4m_inputs()
        assert x.digest == fx["inputs_sha256"]
        V, table, train, held, node0, seeds = x.g.V, x.table, x.train, x.held, x.node0, x.seeds
        periods = [1 << 17, 1 << 16, 1 << 15, 1 << 14] if args.fixture == "c3_1m" else \
            [1 << 19, 1 << 18, 1 << 17, 1 << 16]
    else:
        from test_gpu_tierc import c3_vocab_inputs, C3_FIXTURE
        fx = json.load(open(C3_FIXTURE))
        g, table, train, held, node0, seeds, digest = c3_vocab_inputs(fx["walks"])
        assert digest == fx["inputs_sha256"]
        V = g.V
        periods = [1 << 14, 1 << 13, 1 << 12, 1 << 11]
    if args.periods:
        periods = [int(p) for p in args.periods.split(",")]
    w, n, lr = 5, 5, 0.1
    ri, rp, rn = heldout_o2_pairs(held, w, n, table, 200_000, 24)
    l0 = sgns_loss(node0, np.zeros_like(node0), ri, rp, rn)
    assert abs(l0 - fx["init_loss"]) < 1e-9
    print("inputs %.0fs; init %.5f seq %.5f" % (time.time() - t0, l0, fx["seq_loss"]), flush=True)
    dev = torch.device("cuda", 0)
    tab = torch.from_numpy(table.view(np.int32)).to(dev)
    hot = tsi.hot_rows(tab, V, int(tsi.DEFAULT_HOT_P * len(table)))
    packed = tsi.pack_table(tab)
    ctx0 = np.zeros_like(node0)
    out = {"fixture": args.fixture, "walks": int(train.shape[0]), "seq_loss": fx["seq_loss"],
           "init_loss": l0, "overlap": not args.no_overlap, "points": []}
    combines = args.combines.split(",")
    for comb in combines:
        for N, p in [(N, p) for N in [int(v) for v in args.worlds.split(",")] for p in periods]:
            per_rank = -(-train.shape[0] // N)
            if N == 1 and (p != periods[0] or comb != combines[0]):
                continue  # one rank: no exchange; the period only splits launches
            if p > per_rank and p != periods[0]:
                continue
            t1 = time.time()
            cname, mrows, lr_r = comb, None, lr
            if cname.endswith("@lrN"):
                cname, lr_r = cname[:-4], lr * N
            if cname.startswith("hot_"):  # hot_mean / hot_pick[:share] -- rows holding >= share
                share = float(cname.split(":")[1]) if ":" in cname else tsi.DEFAULT_HOT_P
                hb = tsi.hot_rows(tab, V, max(1, int(share * len(table))))
                bits = torch.arange(V, device=dev)
                mrows = ((hb[bits >> 5] >> (bits & 31)) & 1).bool()
                cname = cname.split(":")[0]
            st = {}
            node, ctx = train_replicas(node0, ctx0, train, seeds, N, min(p, per_rank), w, n,
                                       packed, hot, lr_r, overlap=not args.no_overlap,
                                       combine=cname,
                                       mean_rows=mrows if cname == "hot_mean" else None,
                                       pick_rows=mrows if cname == "hot_pick" else None,
                                       stats=st)
            l = sgns_loss(node.cpu().numpy(), ctx.cpu().numpy(), ri, rp, rn)
            del node, ctx
            torch.cuda.empty_cache()
            pt = {"world": N, "combine": comb, "sync_walks": min(p, per_rank),
                  "exchanges": st.get("exchanges"), "loss": l,
                  "rel_to_seq": (l - fx["seq_loss"]) / fx["seq_loss"], "wall_s": time.time() - t1}
            out["points"].append(pt)
            print(json.dumps(pt), flush=True)
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out))


def main_o1(args):
    import torch
    import come_amd.training_sdg_inner as tsi
    from come_amd.graph import sbm
    from oracle import oracle as orc
    from replica_sim import train_replicas_o1
    from tierc_inputs import log_sigmoid, sgns_loss
    t0 = time.time()
    g = sbm(100, 1000, 0.016, 4.04e-5, seed=0)   # = tests/test_gpu_tierc.py c2_shape
    rng = np.random.RandomState(31)
    e = g.edges[rng.permutation(len(g.edges))].astype(np.int32)
    k = len(e) // 50
    table = orc.make_table(g.degree.astype(np.float64), 10_000_000)
    node0 = rng.uniform(-1, 1, (g.V, 128)).astype(np.float32)
    train, held = e[k:], e[:k]
    train = train[np.lexsort((train[:, 1], train[:, 0]))]  # G.edges() order
    srng = np.random.RandomState(33)
    seeds = [srng.randint(0, 2 ** 48, len(train), dtype=np.int64).astype(np.uint64)
             for _ in range(args.passes)]
    n, lr = 5, 0.1
    neg = table[np.random.RandomState(32).randint(0, len(table), (len(held), n))].astype(np.int64)

    def losses(x):
        ref = float(-log_sigmoid(np.einsum("pd,pd->p", x[held[:, 1]].astype(np.float64),
                                           x[held[:, 0]].astype(np.float64))).sum())
        return ref, sgns_loss(x, x, held[:, 0], held[:, 1], neg)
    seq = node0.copy()
    for sd in seeds:
        orc.sgns_o1_hogwild(seq, train, sd, n, table, lr, threads=1)
    l_seq = losses(seq)
    print("inputs + oracle %.0fs; seq loss (reference / SGNS) %.2f / %.5f" % (
        time.time() - t0, l_seq[0], l_seq[1]), flush=True)
    dev = torch.device("cuda", 0)
    tab = torch.from_numpy(table.view(np.int32)).to(dev)
    hot = tsi.hot_rows(tab, g.V, int(tsi.DEFAULT_HOT_P * len(table)))
    packed = tsi.pack_table(tab)
    periods = [int(p) for p in args.periods.split(",")] if args.periods else [0]
    out = {"fixture": "c2", "edges": int(len(train)), "passes": args.passes,
           "seq_loss_reference": l_seq[0], "seq_loss_sgns": l_seq[1], "points": []}
    for comb in args.combines.split(","):
        for N in [int(v) for v in args.worlds.split(",")]:
            for p in periods:
                if N == 1 and comb != args.combines.split(",")[0]:
                    continue
                t1 = time.time()
                st = {}
                x = train_replicas_o1(node0, train, seeds, N, p or None, n, packed, hot, lr,
                                      combine=comb, stats=st)
                l = losses(x.cpu().numpy())
                pt = {"world": N, "combine": comb, "sync_edges": p or "pass",
                      "exchanges": st.get("exchanges"), "loss_reference": l[0], "loss_sgns": l[1],
                      "rel_reference": (l[0] - l_seq[0]) / l_seq[0],
                      "rel_sgns": (l[1] - l_seq[1]) / l_seq[1], "wall_s": time.time() - t1}
                out["points"].append(pt)
                print(json.dumps(pt), flush=True)
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
