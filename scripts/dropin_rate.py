"""Per-call drop-in throughput: come_amd.training_sdg_inner.train_o2 / train_o1 on numpy tables
(the host route: _come_pyext + libcome's host twin) against the reference's own Cython module
(oracle/_ref, built from /root/reference/utils/training_sdg_inner.pyx by oracle/build_ref.py),
both driven by the reference's worker pool (context_embeddings.py:68-104 /
node_embeddings.py:48-100: a bounded Queue of jobs of 150 walks / edges, `workers` threads, one
call per walk / edge) on identical inputs, on this container's cores.

Runs HERE only (the reference never travels to the GPU box).

    python scripts/dropin_rate.py [--seconds 10] [--threads 1,4,8]
      -> profiles/r07_dropin_rate.json
"""
import argparse
import glob
import importlib.util
import json
import os
import sys
import threading
import time
from queue import Queue

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Vocab(object):
    __slots__ = ("index",)

    def __init__(self, i):
        self.index = i


def pool(items, call, workers, seconds, chunksize=150):
    """The reference's pool; stops feeding jobs after `seconds`.  Returns (items done, elapsed)."""
    jobs = Queue(maxsize=2 * workers)
    lock = threading.Lock()
    done = [0]

    def worker():
        while True:
            job = jobs.get()
            if job is None:
                break
            for it in job:
                call(it)
            with lock:
                done[0] += len(job)

    ts = [threading.Thread(target=worker, daemon=True) for _ in range(workers)]
    t0 = time.time()
    for t in ts:
        t.start()
    for s in range(0, len(items), chunksize):
        if time.time() - t0 > seconds:
            break
        jobs.put(items[s:s + chunksize])
    for _ in ts:
        jobs.put(None)
    for t in ts:
        t.join()
    return done[0], time.time() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--threads", default="1,4,8")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r07_dropin_rate.json"))
    args = ap.parse_args()
    threads = [int(t) for t in args.threads.split(",")]

    import come_amd.training_sdg_inner as tsi
    from come_amd.graph import chung_lu, sbm
    from oracle import oracle as orc
    so = glob.glob(os.path.join(ROOT, "oracle", "_ref", "training_sdg_inner*.so"))
    if not so:
        sys.exit("oracle/_ref is not built (python oracle/build_ref.py)")
    spec = importlib.util.spec_from_file_location("training_sdg_inner", so[0])
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)

    d, n, w, L = 128, 5, 5, 80
    g = chung_lu(1_000_000, 20.0, gamma=2.5, seed=1)
    table = orc.make_table(g.degree.astype(np.float64), 100_000_000)
    rng = np.random.RandomState(7)
    starts = rng.randint(0, g.V, 200_000).astype(np.int32)
    walks = orc.philox_walks(g.rowptr, g.col, starts, L, 0.0, seed=7)
    vocab = [Vocab(i) for i in range(g.V)]
    paths = [[vocab[x] if x >= 0 else None for x in row] for row in walks]

    def pairs_of(row):
        ok = row >= 0
        tot = 0
        for i in np.nonzero(ok)[0]:
            lo, hi = max(0, i - w), min(L, i + w + 1)
            tot += int(ok[lo:hi].sum()) - 1
        return tot
    pairs_per_walk = np.mean([pairs_of(r) for r in walks[:2000]])
    node0 = rng.uniform(-1, 1, (g.V, d)).astype(np.float32)
    res = {}
    for thr in threads:
        for name, mod in (("reference_cython", ref), ("come_host_route", tsi)):
            node, ctx = node0.copy(), np.zeros_like(node0)
            tl = threading.local()  # py_work is per worker (context_embeddings.py:81)

            def work():
                if not hasattr(tl, "w"):
                    tl.w = np.zeros(d, np.float32)
                return tl.w
            np.random.seed(1)
            k, el = pool(paths, lambda p: mod.train_o2(node, ctx, p, 0.1, n, w, table,
                                                       py_alpha=1.0, py_size=d, py_work=work()),
                         thr, args.seconds)
            res["o2_%s_%dthr" % (name, thr)] = {"pairs_per_s": k * pairs_per_walk / el,
                                                "walks": k, "seconds": el}
            print("O2 %-17s %d thr: %.3e pair-updates/s" % (name, thr, k * pairs_per_walk / el),
                  flush=True)
    g2 = sbm(100, 1000, 0.016, 4.04e-5, seed=0)
    table2 = orc.make_table(g2.degree.astype(np.float64), 100_000_000)
    vocab2 = [Vocab(i) for i in range(g2.V)]
    edges = [[vocab2[u], vocab2[v]] for u, v in g2.edges]
    node2 = rng.uniform(-1, 1, (g2.V, d)).astype(np.float32)
    for thr in threads:
        for name, mod in (("reference_cython", ref), ("come_host_route", tsi)):
            x = node2.copy()
            tl = threading.local()  # py_work is per worker (node_embeddings.py:69)

            def work():
                if not hasattr(tl, "w"):
                    tl.w = np.zeros(d, np.float32)
                return tl.w
            np.random.seed(2)
            k, el = pool(edges, lambda e: mod.train_o1(x, e, 0.2, n, table2, py_size=d,
                                                       py_work=work()), thr, args.seconds)
            res["o1_%s_%dthr" % (name, thr)] = {"pairs_per_s": 2 * k / el, "edges": k,
                                                "seconds": el}
            print("O1 %-17s %d thr: %.3e pair-updates/s" % (name, thr, 2 * k / el), flush=True)
    out = {
        "what": "per-call drop-ins on numpy tables (host route) vs the reference's Cython "
                "train_o2/train_o1, both under the reference's worker pool, identical inputs",
        "host": "container: %d CPUs (%s)" % (os.cpu_count(), open("/proc/cpuinfo").read().split(
            "model name")[1].split("\n")[0].strip(" :\t")),
        "o2_workload": "C3: Chung-Lu 1M nodes, d=128, n=5, w=5, L=80, T=1e8, lr 0.1; %.1f pair "
                       "updates per walk" % pairs_per_walk,
        "o1_workload": "C2: SBM 100x1000 (%d edges), d=128, n=5, T=1e8, lr 0.2" % len(edges),
        "results": res,
        "ratio_ours_over_reference": {
            k.replace("come_host_route_", ""): res[k]["pairs_per_s"] /
            res[k.replace("come_host_route", "reference_cython")]["pairs_per_s"]
            for k in res if "come_host_route" in k},
        "script": "scripts/dropin_rate.py",
    }
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out["ratio_ours_over_reference"]))


if __name__ == "__main__":
    main()
