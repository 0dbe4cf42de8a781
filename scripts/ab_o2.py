"""Interleaved A/B timing of O2 launch variants on the bench workload (one process, R rounds x
V variants; cdna_hip_programming.md §5.4 rule 24).  Variants are come_set_option knob sets.

    python scripts/ab_o2.py --rounds 5 --variants 'default' 'o2_plain_writeback=1' ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse(v):
    if v == "default":
        return {}
    return {k: int(x) for k, x in (kv.split("=") for kv in v.split(","))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--walks", type=int, default=1 << 17)
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--negative", type=int, default=5)
    ap.add_argument("--variants", nargs="+", default=["default"])
    ap.add_argument("--warm-launches", type=int, default=2)
    ap.add_argument("--table-size", type=int, default=100_000_000)
    args = ap.parse_args()
    import torch
    import come_amd.training_sdg_inner as tsi
    from come_amd import _lib
    from come_amd.graph import chung_lu, random_walks
    from come_amd.model import Model
    dev = torch.device("cuda", 0)
    g = chung_lu(args.nodes, 20.0, gamma=2.5, seed=1)
    np.random.seed(1234)
    m = Model(g.degree_by_id(), size=args.dim, table_size=args.table_size, k=1, device=dev)
    walks = random_walks(g, 1, 80, seed=100, device=dev)[:args.walks].contiguous()
    np.random.seed(5678)
    seeds = torch.from_numpy(tsi.draw_seeds(args.walks).view(np.int64)).to(dev)
    pairs = tsi.count_o2_pairs(walks.cpu().numpy(), 5)
    keys = ["o2_kernel", "o2_blocks_per_cu", "o2_plain_writeback", "o2_waves_per_block",
            "o2_static", "o2_pair_atomics", "resident_cap"]
    packed = tsi.pack_table(m.table)  # variant key "packed=1" draws from the packed table
    # warm the tables past the all-zero context rows, then time every launch from that state
    for _ in range(args.warm_launches):
        tsi.sgns_o2(m.node_embedding, m.context_embedding, walks, seeds, 5, args.negative,
                    m.table, 0.025, 1.0, tsi.MODE_HOGWILD)
    snap = (m.node_embedding.clone(), m.context_embedding.clone())
    res = {v: [] for v in args.variants}
    for r in range(args.rounds + 1):
        for v in args.variants:
            opts = parse(v)
            for k in keys:
                _lib.set_option(k, opts.get(k, 0))
            table = packed if opts.get("packed", 0) else m.table
            m.node_embedding.copy_(snap[0])
            m.context_embedding.copy_(snap[1])
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            tsi.sgns_o2(m.node_embedding, m.context_embedding, walks, seeds, 5, args.negative,
                        table, 0.025, 1.0, tsi.MODE_HOGWILD)
            e.record()
            torch.cuda.synchronize()
            if r > 0:  # round 0 = warmup
                res[v].append(s.elapsed_time(e))
    for k in keys:
        _lib.set_option(k, 0)
    out = {}
    for v, ts in res.items():
        med = float(np.median(ts))
        out[v] = {"median_ms": med, "min_ms": float(np.min(ts)), "pairs_per_s": pairs / med * 1e3}
        print("%-40s median %8.2f ms  min %8.2f ms  %.3e pairs/s" % (v, med, min(ts),
                                                                    pairs / med * 1e3))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
