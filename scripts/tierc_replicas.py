"""Tier C of the multi-GPU SGNS path (SURVEY.md §8c applied to §8e): N ranks simulated on one GPU
(tests/replica_sim.py: the product's launches, DeltaAllReduce arithmetic and overlapped protocol;
RCCL replaced by a sum over the replicas) against the sequential oracle's held-out loss after the
same walks, for N = 1, 2, 4, 8 and a range of sync periods (walks per rank between exchanges).

    python scripts/tierc_replicas.py --fixture c3_1m [--worlds 1,2,4,8] [--periods ...]
    python scripts/tierc_replicas.py --fixture c3_131k

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
    ap.add_argument("--fixture", choices=["c3_1m", "c3_4m", "c3_131k"], default="c3_1m")
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


if __name__ == "__main__":
    main()
