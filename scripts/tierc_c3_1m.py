"""Tier C at the bench's own launch (configs[2]/C3, one launch of 1,048,576 walks = 8.1e8 pair
updates, packed table + hot-row bitmap = the product's launch): held-out SGNS loss of the GPU
Hogwild run against the sequential oracle (C restatement, walks in order, run in chunks of 65,536
walks so progress is printed) and against the reference's own regime (the C Hogwild restatement
with 16 worker threads).  Too long for a test (~10 minutes of single-core oracle); the result is
recorded in profiles/r03_tierc_c3_1m_launch.json.  The inputs are deterministic (Chung-Lu seed 1,
make_table, the exact CPython-stream host walker with fixed seeds, RandomState(7)), so the two
halves run apart and are matched by the inputs' digest:

    python scripts/tierc_c3_1m.py --part gpu      # on the MI355X box
    python scripts/tierc_c3_1m.py --part oracle   # anywhere (~30 min of one core + Hogwild CPU)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import come_amd.training_sdg_inner as tsi  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from test_gpu_tierc import dev, heldout_o2_pairs, sgns_loss  # noqa: E402


def main():
    import argparse
    import hashlib
    import random
    from come_amd import graph_utils as gu
    from come_amd.graph import chung_lu
    ap = argparse.ArgumentParser()
    ap.add_argument("--part", choices=["gpu", "oracle"], required=True)
    args = ap.parse_args()
    t0 = time.time()
    B = 1 << 20
    g = chung_lu(1_000_000, 20.0, gamma=2.5, seed=1)
    table = orc.make_table(g.degree.astype(np.float64), 100_000_000)
    Gh = gu.Graph(np.arange(1, g.V + 1), g.rowptr, g.col.astype(np.int32), g.degree,
                  np.zeros((0, 2), np.int32))
    walks = gu._corpus(Gh, [1, 1], 80, 0.0, [random.Random(s) for s in (11, 12)], threads=2)
    walks = np.asarray(walks, np.int32)
    rng = np.random.RandomState(7)
    pick = rng.choice(walks.shape[0], B + 20000, replace=False)
    walks = walks[pick]
    train, held = walks[:B], walks[B:]
    node0 = rng.uniform(-1, 1, (g.V, 128)).astype(np.float32)
    seeds = rng.randint(0, 2 ** 48, B, dtype=np.int64).astype(np.uint64)
    w, n, lr = 5, 5, 0.1
    rows_in, rows_pos, rows_neg = heldout_o2_pairs(held, w, n, table, 200_000, 24)
    l0 = sgns_loss(node0, np.zeros_like(node0), rows_in, rows_pos, rows_neg)
    digest = hashlib.sha256(walks.tobytes() + seeds.tobytes() + node0.tobytes()[:1 << 20] +
                            table.tobytes()[:1 << 20]).hexdigest()
    print("inputs ready %.0fs, init loss %.5f, digest %s" % (time.time() - t0, l0, digest),
          flush=True)
    if args.part == "gpu":
        gpu_part(g, table, train, seeds, node0, rows_in, rows_pos, rows_neg, l0, digest, t0)
    else:
        oracle_part(table, train, seeds, node0, rows_in, rows_pos, rows_neg, l0, digest, t0)


def gpu_part(g, table, train, seeds, node0, rows_in, rows_pos, rows_neg, l0, digest, t0):
    w, n, lr = 5, 5, 0.1
    B = train.shape[0]

    tab = dev(table)
    hot = tsi.hot_rows(tab, g.V, int(tsi.DEFAULT_HOT_P * len(table)))
    packed = tsi.pack_table(tab)
    l_gpu = []
    for _ in range(2):
        node = dev(node0)
        ctx = torch.zeros_like(node)
        tsi.sgns_o2(node, ctx, dev(train), dev(seeds), w, n, packed, lr, 1.0, tsi.MODE_HOGWILD,
                    hot=hot)
        torch.cuda.synchronize()
        l_gpu.append(sgns_loss(node.cpu().numpy(), ctx.cpu().numpy(), rows_in, rows_pos,
                               rows_neg))
        print("gpu hogwild loss %.5f" % l_gpu[-1], flush=True)

    out = {"part": "gpu", "digest": digest, "walks": B, "init_loss": l0,
           "gpu_hogwild_losses": l_gpu, "wall_s": time.time() - t0}
    print(json.dumps(out), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "tierc_c3_1m_gpu.json"), "w"), indent=1)


def oracle_part(table, train, seeds, node0, rows_in, rows_pos, rows_neg, l0, digest, t0):
    w, n, lr = 5, 5, 0.1
    B = train.shape[0]
    cn, cc = node0.copy(), np.zeros_like(node0)
    threads = min(16, orc.usable_cpus())
    orc.sgns_o2_hogwild(cn, cc, train, seeds, w, n, table, lr, 1.0, threads=threads)
    l_cpu = sgns_loss(cn, cc, rows_in, rows_pos, rows_neg)
    print("cpu hogwild (%d threads) loss %.5f  %.0fs" % (threads, l_cpu, time.time() - t0),
          flush=True)

    sn, sc = node0.copy(), np.zeros_like(node0)
    C = 65536
    for s in range(0, B, C):
        orc.sgns_o2_hogwild(sn, sc, train[s:s + C].copy(), seeds[s:s + C].copy(), w, n, table,
                            lr, 1.0, threads=1)
        print("sequential oracle: %d / %d walks  %.0fs" % (s + C, B, time.time() - t0),
              flush=True)
    l_seq = sgns_loss(sn, sc, rows_in, rows_pos, rows_neg)
    out = {"part": "oracle", "digest": digest, "walks": B,
           "pairs": int(tsi.count_o2_pairs(train, w)), "init_loss": l0, "seq_loss": l_seq,
           "cpu_hogwild_loss": l_cpu, "cpu_hogwild_threads": threads,
           "cpu_hogwild_rel_to_seq": (l_cpu - l_seq) / l_seq, "wall_s": time.time() - t0}
    print(json.dumps(out), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "tierc_c3_1m_oracle.json"), "w"),
              indent=1)


if __name__ == "__main__":
    main()
