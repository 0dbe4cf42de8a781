"""Calibrate the CPU baseline: the builder's Hogwild C restatement (oracle/come_oracle_mt.c, what
bench.py times on the GPU box) against the reference's own Cython train_o2 (oracle/_ref, built from
/root/reference/utils/training_sdg_inner.pyx by oracle/build_ref.py) driven exactly as
Context2Vec.train drives it (context_embeddings.py:72-98: worker threads, one train_o2 call per walk,
GIL released inside, pyx:493).

Runs HERE only (the reference never travels to the GPU box).  Both legs get identical inputs: the
C3 workload (Chung-Lu power law, 1M nodes, mean degree 20, d=128, n=5, w=5, L=80, T=1e8, lr as
bench.py), the same walks, seeds and starting tables; each leg runs for --seconds on --threads
threads.  Writes profiles/r02_cpu_calibration.json with both rates and their ratio.

    python scripts/calibrate_cpu.py [--threads 8] [--seconds 20]
"""
import argparse
import glob
import importlib.util
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def host_walks(g, P, L, seed):
    """Uniform random walks (no restart) of length L from P random starts, rows, numpy."""
    rng = np.random.default_rng(seed)
    cur = rng.integers(0, g.V, P)
    out = np.empty((P, L), np.int32)
    out[:, 0] = cur
    alive = np.ones(P, bool)
    for s in range(1, L):
        deg = g.rowptr[cur + 1] - g.rowptr[cur]
        alive &= deg > 0
        pick = g.rowptr[cur] + (rng.random(P) * np.maximum(deg, 1)).astype(np.int64)
        cur = np.where(alive, g.col[np.minimum(pick, len(g.col) - 1)], cur)
        out[:, s] = np.where(alive, cur, -1)
    return out


def cython_leg(ref, walks, seeds, node, ctx, table, w, n, lr, seconds, threads):
    """Context2Vec-style driver of the reference's train_o2: Python worker threads, one call per
    walk (a path of Vocab objects), per-worker work buffer.  Seeds: train_o2 draws its own from
    the global numpy RNG (pyx:477), so `seeds` is unused here (same distribution)."""

    class Vocab(object):
        __slots__ = ("index",)

        def __init__(self, i):
            self.index = i

    vocab = {}

    def path_of(row):
        out = []
        for r in row:
            if r < 0:
                break
            v = vocab.get(r)
            if v is None:
                v = vocab[r] = Vocab(int(r))
            out.append(v)
        return out

    paths = [path_of(r) for r in walks]
    state = {"next": 0, "pairs": 0, "walks": 0}
    lock = threading.Lock()
    d = node.shape[1]
    deadline = [0.0]

    def pairs_of(l):
        return 2 * w * l - w * (w + 1) if l >= w + 1 else l * (l - 1)

    def worker():
        work = np.zeros(d, np.float32)
        while True:
            with lock:
                i = state["next"]
                if i >= len(paths) or time.time() > deadline[0]:
                    return
                state["next"] = i + 1
            ref.train_o2(node, ctx, paths[i], lr, n, w, table, py_alpha=1.0, py_size=d,
                         py_work=work)
            with lock:
                state["pairs"] += pairs_of(len(paths[i]))
                state["walks"] += 1

    ts = [threading.Thread(target=worker, daemon=True) for _ in range(threads)]
    t0 = time.time()
    deadline[0] = t0 + seconds
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    el = time.time() - t0
    return state["pairs"] / el, state["pairs"], state["walks"], el


def cython_o1_leg(ref, edges, node, table, n, lr, seconds, threads):
    """Node2Vec.train-style driver of the reference's train_o1 (node_embeddings.py:58-83):
    Python worker threads, one call per edge (GIL released only inside the call)."""

    class Vocab(object):
        __slots__ = ("index",)

        def __init__(self, i):
            self.index = i
    items = [[Vocab(int(u)), Vocab(int(v))] for u, v in edges]
    state = {"next": 0, "edges": 0}
    lock = threading.Lock()
    d = node.shape[1]
    deadline = [0.0]

    def worker():
        work = np.zeros(d, np.float32)
        while True:
            with lock:
                i = state["next"]
                if i >= len(items) or time.time() > deadline[0]:
                    return
                state["next"] = i + 1
            ref.train_o1(node, items[i], lr, n, table, py_size=d, py_work=work)
            with lock:
                state["edges"] += 1

    ts = [threading.Thread(target=worker, daemon=True) for _ in range(threads)]
    t0 = time.time()
    deadline[0] = t0 + seconds
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    el = time.time() - t0
    return 2 * state["edges"] / el, state["edges"], el


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--table-size", type=int, default=100_000_000)
    ap.add_argument("--walks", type=int, default=400_000)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_cpu_calibration.json"))
    args = ap.parse_args()

    from come_amd.graph import chung_lu
    from oracle import oracle as orc

    so = glob.glob(os.path.join(ROOT, "oracle", "_ref", "training_sdg_inner*.so"))
    if not so:
        sys.exit("oracle/_ref is not built (python oracle/build_ref.py)")
    spec = importlib.util.spec_from_file_location("training_sdg_inner", so[0])
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)

    d, n, w, L = 128, 5, 5, 80
    t0 = time.time()
    g = chung_lu(args.nodes, 20.0, gamma=2.5, seed=1)
    table = orc.make_table(g.degree.astype(np.float64), args.table_size)
    walks = host_walks(g, args.walks, L, seed=7)
    rng = np.random.RandomState(1234)
    node0 = rng.uniform(-1, 1, (g.V, d)).astype(np.float32)
    seeds = ((rng.randint(0, 2 ** 24, args.walks).astype(np.uint64) << np.uint64(24))
             + rng.randint(0, 2 ** 24, args.walks).astype(np.uint64))
    print("inputs ready in %.1fs: V=%d E=%d walks=%d" % (time.time() - t0, g.V, g.num_edges,
                                                           len(walks)), flush=True)

    res = {}
    for name in ("restatement", "cython"):
        for thr in sorted({1, args.threads}):
            node, ctx = node0.copy(), np.zeros_like(node0)
            if name == "cython":
                np.random.seed(1234)
                rate, pairs, done, el = cython_leg(ref, walks, seeds, node, ctx, table, w, n,
                                                   args.lr, args.seconds, thr)
            else:
                t1 = time.time()
                pairs, done = orc.sgns_o2_hogwild(node, ctx, walks, seeds, w, n, table, args.lr,
                                                  1.0, thr, args.seconds)
                el = time.time() - t1
                rate = pairs / el
            assert np.isfinite(node).all() and np.isfinite(ctx).all()
            res["%s_%dthr" % (name, thr)] = {"pairs_per_s": rate, "pairs": pairs, "walks": done,
                                             "seconds": el}
            print(name, thr, "threads: %.3e pair-updates/s (%d walks in %.1fs)" % (
                rate, done, el), flush=True)
    # O1 (C2: SBM 100 x 1000, d=128, n=5, lr 0.2)
    from come_amd.graph import sbm
    g2 = sbm(100, 1000, 0.016, 4.04e-5, seed=0)
    table2 = orc.make_table(g2.degree.astype(np.float64), args.table_size)
    edges = g2.edges.astype(np.int32)
    rng2 = np.random.RandomState(99)
    node2 = rng2.uniform(-1, 1, (g2.V, d)).astype(np.float32)
    eseeds = rng2.randint(0, 2 ** 48, len(edges), dtype=np.int64).astype(np.uint64)
    for thr in sorted({1, args.threads}):
        x = node2.copy()
        t1 = time.time()
        p, e = orc.sgns_o1_hogwild(x, edges, eseeds, 5, table2, 0.2, thr, args.seconds)
        el = time.time() - t1
        res["o1_restatement_%dthr" % thr] = {"pairs_per_s": p / el, "edges": e, "seconds": el}
        x = node2.copy()
        rate, e, el = cython_o1_leg(ref, edges, x, table2, 5, 0.2, args.seconds, thr)
        res["o1_cython_%dthr" % thr] = {"pairs_per_s": rate, "edges": e, "seconds": el}
        print("O1", thr, "threads: restatement %.3e, cython %.3e pair-updates/s" % (
            res["o1_restatement_%dthr" % thr]["pairs_per_s"], rate), flush=True)
    k = args.threads
    out = {
        "what": "Hogwild C restatement (oracle/come_oracle_mt.c, bench.py cpu_baseline) vs the "
                "reference's Cython train_o2 (oracle/_ref) driven by Python threads like "
                "Context2Vec.train, identical inputs, this container",
        "host": "container: %d CPUs (%s)" % (os.cpu_count(), open("/proc/cpuinfo").read().split(
            "model name")[1].split("\n")[0].strip(" :\t")),
        "workload": "C3: Chung-Lu 1M nodes / %d edges, d=128, negative=5, window=5, "
                    "walk_length=80, table_size=%d, lr=%g" % (g.num_edges, args.table_size,
                                                               args.lr),
        "threads": k,
        "results": res,
        "ratio_restatement_over_cython": res["restatement_%dthr" % k]["pairs_per_s"]
        / res["cython_%dthr" % k]["pairs_per_s"],
        "ratio_restatement_over_cython_1thr": res["restatement_1thr"]["pairs_per_s"]
        / res["cython_1thr"]["pairs_per_s"],
        "o1_ratio_restatement_over_cython": res["o1_restatement_%dthr" % k]["pairs_per_s"]
        / res["o1_cython_%dthr" % k]["pairs_per_s"],
        "o1_workload": "C2: SBM 100x1000 (%d edges), d=128, negative=5, lr=0.2; the reference's "
                       "Node2Vec.train is GIL-bound (one Python call per edge), the C "
                       "restatement is not" % len(edges),
        "script": "scripts/calibrate_cpu.py",
    }
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps({k2: out[k2] for k2 in ("ratio_restatement_over_cython",
                                             "ratio_restatement_over_cython_1thr",
                                             "o1_ratio_restatement_over_cython")}))


if __name__ == "__main__":
    main()
