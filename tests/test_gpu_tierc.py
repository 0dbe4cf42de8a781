"""Tier C: statistical parity of the Hogwild PRODUCT mode -- the mode bench.py
measures -- against the sequential oracle, at the benchmarked shapes.

Hogwild on the GPU has thousands of walks (edges) in flight, hub rows held by many wavefronts at
once and plain-store negative-row updates across 8 non-coherent XCD L2s; the reference's Hogwild
has `workers` threads.  Neither is reproducible bit for bit, so the bar is the one SURVEY.md §8c
sets: the held-out SGNS loss  -sum log sigma(u.c+) - sum_k log sigma(-u.c_k)  of the Hogwild
result within 1% of the sequential oracle's, plus -- for O1 -- the reference's own loss
(node_embeddings.py:26-31, -sum log sigma(u.v) over edges) within 1%, and the Karate NMI against
karate_zachary.labels within the oracle's seed range (0.48-0.73).

The sequential oracle here is the C restatement with one worker thread (oracle/come_oracle_mt.c:
walks in order = the reference with workers=1; pinned to the reference's own golden vectors by
tests/test_oracle_golden.py) -- the plain C oracle is 3x slower at d=128 and would need minutes.
Each test also reports the spread between two sequential runs that differ only in walk order,
the natural size of an ordering effect.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import oracle as orc

import come_amd.training_sdg_inner as tsi

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def dev(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).to(DEV)


from tierc_inputs import heldout_o2_pairs, log_sigmoid, sgns_loss  # noqa: E402,F401


@pytest.fixture(scope="module")
def c3_shape():
    """C3's shape at 100k nodes: Chung-Lu power law (gamma 2.5, mean degree 20: hubs of degree
    ~10^3), d=128, n=5, w=5, L=80, T=1e8 (the headline table size), lr 0.1;
    10,000 training walks (7.7e6 pair updates) from the device walker, 2,000 held-out walks."""
    from come_amd.graph import chung_lu, random_walks
    g = chung_lu(100_000, 20.0, gamma=2.5, seed=21)
    table = orc.make_table(g.degree.astype(np.float64), 100_000_000)
    walks = random_walks(g, 1, 80, seed=22, device="cuda").cpu().numpy()
    rng = np.random.RandomState(23)
    walks = walks[rng.permutation(len(walks))[:12_000]]
    node0 = rng.uniform(-1, 1, (g.V, 128)).astype(np.float32)
    seeds = rng.randint(0, 2 ** 48, 10_000, dtype=np.int64).astype(np.uint64)
    return g, table, walks[:10_000], walks[10_000:], node0, seeds


def o2_tierc(g, table, train, held, node0, seeds, runs=3, cpu=True):
    """Held-out loss of `runs` GPU Hogwild launches (the product's launch: Context2Vec.train's
    hot-row bitmap, the automatic kernel choice) against the sequential oracle, the same walks
    reversed (the ordering effect alone) and the reference's regime (Hogwild C threads)."""
    w, n, lr = 5, 5, 0.1
    rows_in, rows_pos, rows_neg = heldout_o2_pairs(held, w, n, table, 200_000, 24)
    ctx0 = np.zeros_like(node0)
    l0 = sgns_loss(node0, ctx0, rows_in, rows_pos, rows_neg)
    tab, tw, ts = dev(table), dev(train), dev(seeds)
    hot = tsi.hot_rows(tab, g.V, int(tsi.DEFAULT_HOT_P * len(table)))
    l_hog = []
    for _ in range(runs):  # Hogwild is not reproducible: every launch must pass, not one
        node, ctx = dev(node0), dev(ctx0)
        tsi.sgns_o2(node, ctx, tw, ts, w, n, tab, lr, 1.0, tsi.MODE_HOGWILD, hot=hot)
        torch.cuda.synchronize()
        hn, hc = node.cpu().numpy(), ctx.cpu().numpy()
        assert np.isfinite(hn).all() and np.isfinite(hc).all()
        l_hog.append(sgns_loss(hn, hc, rows_in, rows_pos, rows_neg))
    sn, sc = node0.copy(), ctx0.copy()
    pairs, done = orc.sgns_o2_hogwild(sn, sc, train, seeds, w, n, table, lr, 1.0, threads=1)
    assert done == len(train)
    l_seq = sgns_loss(sn, sc, rows_in, rows_pos, rows_neg)
    rn, rc = node0.copy(), ctx0.copy()
    orc.sgns_o2_hogwild(rn, rc, train[::-1].copy(), seeds[::-1].copy(), w, n, table, lr, 1.0,
                        threads=1)
    l_rev = sgns_loss(rn, rc, rows_in, rows_pos, rows_neg)
    l_cpu = float("nan")
    if cpu:
        cn, cc = node0.copy(), ctx0.copy()
        orc.sgns_o2_hogwild(cn, cc, train, seeds, w, n, table, lr, 1.0,
                            threads=min(16, orc.usable_cpus()))
        l_cpu = sgns_loss(cn, cc, rows_in, rows_pos, rows_neg)
    rel = [abs(x - l_seq) / l_seq for x in l_hog]
    print("O2 held-out loss (V=%d, %d walks, %d pairs): init %.5f  seq %.5f  reversed %.5f  "
          "cpu-hogwild %.5f  gpu-hogwild %s  max |gpu-seq|/seq %.5f  |rev-seq|/seq %.5f" % (
              g.V, len(train), pairs, l0, l_seq, l_rev, l_cpu,
              " ".join("%.5f" % x for x in l_hog), max(rel), abs(l_rev - l_seq) / l_seq))
    assert l_seq < l0 - 0.05  # training moved the loss: the comparison is not vacuous
    assert max(rel) < 0.01, (l_hog, l_seq)  # SURVEY.md §8c tier C, every launch


def test_o2_hogwild_heldout_loss_matches_sequential_oracle(c3_shape):
    """100k nodes, 10k walks in one launch: every walk in flight at once, the most contended
    regime (the automatic choice runs the direct kernel here, come_sgns_o2_ex)."""
    o2_tierc(*c3_shape)


C3_FIXTURE = os.path.join(GOLDEN, "tierc_c3_seq.json")


def c3_vocab_inputs(walks_n=131_072):
    """The benchmarked shape (configs[2]/C3): Chung-Lu 1M nodes (gamma 2.5, mean degree 20,
    bench.py's seed), T = 1e8, d=128, n=5, w=5, L=80, lr 0.1, and ONE bench launch of training
    walks (131,072, from the device walker); 20,000 held-out walks."""
    import hashlib
    from come_amd.graph import chung_lu, random_walks
    g = chung_lu(1_000_000, 20.0, gamma=2.5, seed=1)
    table = orc.make_table(g.degree.astype(np.float64), 100_000_000)
    walks = random_walks(g, 1, 80, seed=100, device="cuda")
    rng = np.random.RandomState(7)
    pick = torch.from_numpy(rng.choice(walks.shape[0], walks_n + 20000, replace=False))
    walks = walks[pick.to(walks.device)].cpu().numpy()
    node0 = rng.uniform(-1, 1, (g.V, 128)).astype(np.float32)
    seeds = rng.randint(0, 2 ** 48, walks_n, dtype=np.int64).astype(np.uint64)
    digest = hashlib.sha256(walks.tobytes() + table.tobytes()[:1 << 20]).hexdigest()
    return g, table, walks[:walks_n], walks[walks_n:], node0, seeds, digest


def test_o2_hogwild_heldout_loss_at_benchmarked_shape():
    """Tier C at C3 itself: one launch (131,072 walks, 1.0e8 pair updates; the bench and the
    product launch 1,048,576 walks of the same kernel at the same concurrency) of the product's
    Hogwild path (streaming kernel, hot-row bitmap, packed negative table) against the sequential oracle's held-out loss after the same
    walks.  The oracle run takes ~3 minutes on one core, so its result is a committed fixture
    (tests/golden/tierc_c3_seq.json, scripts/make_tierc_fixture.py: the same inputs, sequential C
    oracle in walk order); the inputs' digest must match it.  Measured (profiles/
    r02_tierc_vs_walks_c3_vocab.json): the gap is 2.2% after 16k walks, 0.6% after 49k and
    < 0.1% after this launch -- the GPU's thousands of walks in flight act like a large minibatch
    early on, and the effect fades as training proceeds."""
    import json
    fx = json.load(open(C3_FIXTURE))
    g, table, train, held, node0, seeds, digest = c3_vocab_inputs(fx["walks"])
    assert digest == fx["inputs_sha256"], "inputs differ from the fixture's (walker / graph changed)"
    w, n, lr = 5, 5, 0.1
    rows_in, rows_pos, rows_neg = heldout_o2_pairs(held, w, n, table, 200_000, 24)
    l0 = sgns_loss(node0, np.zeros_like(node0), rows_in, rows_pos, rows_neg)
    assert abs(l0 - fx["init_loss"]) < 1e-9
    tab = dev(table)
    hot = tsi.hot_rows(tab, g.V, int(tsi.DEFAULT_HOT_P * len(table)))
    packed = tsi.pack_table(tab)  # the product's negative table (Model.negative_table)
    assert packed is not None
    l_hog = []
    for _ in range(2):
        node = dev(node0)
        ctx = torch.zeros_like(node)
        tsi.sgns_o2(node, ctx, dev(train), dev(seeds), w, n, packed, lr, 1.0, tsi.MODE_HOGWILD,
                    hot=hot)
        torch.cuda.synchronize()
        l_hog.append(sgns_loss(node.cpu().numpy(), ctx.cpu().numpy(), rows_in, rows_pos,
                               rows_neg))
    rel = [abs(x - fx["seq_loss"]) / fx["seq_loss"] for x in l_hog]
    print("C3 held-out loss: init %.5f  seq (fixture) %.5f  gpu-hogwild %s  max rel %.5f" % (
        l0, fx["seq_loss"], " ".join("%.5f" % x for x in l_hog), max(rel)))
    assert fx["seq_loss"] < l0 - 0.5
    assert max(rel) < 0.01, (l_hog, fx["seq_loss"])  # SURVEY.md §8c tier C


def test_o2_update_count_matches_oracle(c3_shape):
    """The in-kernel target-update counter (come_launch_opts.o2_update_count, what bench.py's
    algorithmic bytes are computed from) equals the oracle's count in SEQUENTIAL mode (same
    arithmetic, same order); in Hogwild mode it is within 5% of it (other skips happen when
    other walks' updates interleave)."""
    g, table, train, held, node0, seeds = c3_shape
    w, n, lr = 5, 5, 0.1
    few, fs = train[:300], seeds[:300]
    counts = []
    tab = dev(table)
    hot = tsi.hot_rows(tab, g.V, int(tsi.DEFAULT_HOT_P * len(table)))
    for mode in (tsi.MODE_SEQUENTIAL, tsi.MODE_HOGWILD):
        cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
        node, ctx = dev(node0), dev(np.zeros_like(node0))
        tsi.sgns_o2(node, ctx, dev(few), dev(fs), w, n, tab, lr, 1.0, mode,
                    update_count=cnt, hot=hot)
        torch.cuda.synchronize()
        counts.append(int(cnt.item()))
    sn, sc = node0.copy(), np.zeros_like(node0)
    orc.reset_updates()
    pairs = orc.sgns_o2(sn, sc, few, fs, w, n, table, lr, 1.0, dot_mode=orc.DOT_WAVE64)
    ref = orc.updates()
    print("target updates: oracle %d, sequential %d, hogwild %d, max %d" % (
        ref, counts[0], counts[1], pairs * (1 + n)))
    assert counts[0] == ref and 0 < ref <= pairs * (1 + n)
    assert abs(counts[1] - ref) < 0.05 * ref


@pytest.fixture(scope="module")
def c2_shape():
    """C2: SBM 100 blocks x 1,000 nodes, p_in 0.016, p_out 4.04e-5 (~1M edges), d=128, n=5;
    2% of the edges held out."""
    from come_amd.graph import sbm
    g = sbm(100, 1000, 0.016, 4.04e-5, seed=0)
    rng = np.random.RandomState(31)
    e = g.edges[rng.permutation(len(g.edges))].astype(np.int32)
    k = len(e) // 50
    table = orc.make_table(g.degree.astype(np.float64), 10_000_000)
    node0 = rng.uniform(-1, 1, (g.V, 128)).astype(np.float32)
    seeds = rng.randint(0, 2 ** 48, len(e) - k, dtype=np.int64).astype(np.uint64)
    return g, table, e[k:], e[:k], node0, seeds


def test_o1_hogwild_heldout_loss_matches_sequential_oracle(c2_shape):
    g, table, train, held, node0, seeds = c2_shape
    n, lr = 5, 0.1
    rng = np.random.RandomState(32)
    neg = table[rng.randint(0, len(table), (len(held), n))].astype(np.int64)

    def losses(x):
        ref = float(-log_sigmoid(np.einsum("pd,pd->p", x[held[:, 1]].astype(np.float64),
                                           x[held[:, 0]].astype(np.float64))).sum())
        return ref, sgns_loss(x, x, held[:, 0], held[:, 1], neg)

    l0 = losses(node0)
    node = dev(node0)
    tab = dev(table)
    hot = tsi.hot_rows(tab, g.V, int(tsi.DEFAULT_HOT_P * len(table)))
    tsi.sgns_o1(node, dev(train), dev(seeds), n, tab, lr, tsi.MODE_HOGWILD, hot=hot)
    torch.cuda.synchronize()
    hog = node.cpu().numpy()
    assert np.isfinite(hog).all()
    l_hog = losses(hog)
    seq = node0.copy()
    orc.sgns_o1_hogwild(seq, train, seeds, n, table, lr, threads=1)
    l_seq = losses(seq)
    rev = node0.copy()
    orc.sgns_o1_hogwild(rev, train[::-1].copy(), seeds[::-1].copy(), n, table, lr, threads=1)
    l_rev = losses(rev)
    print("O1 held-out loss (reference :26-31 / SGNS): init %.1f / %.5f  seq %.1f / %.5f  "
          "reversed %.1f / %.5f  gpu-hogwild %.1f / %.5f" % (l0 + l_seq + l_rev + l_hog))
    assert l_seq[1] < l0[1] - 0.05
    for a, b in zip(l_hog, l_seq):
        assert abs(a - b) / abs(b) < 0.01, (l_hog, l_seq)  # SURVEY.md §8c tier C


def test_o1_hogwild_in_reference_edge_order(c2_shape):
    """O1 tier C in the reference's own edge order (np.array(G.edges()), node_embeddings.py:39:
    grouped by the first endpoint, so consecutive edges share their input row) at the product
    default o1_chunk = -1 (k_sgns_o1_runs, one contiguous chunk per wavefront: the edges in flight
    spread over the whole list), against the sequential oracle on the same order: held-out losses
    within 1%.  Measured r04q: -1 +0.23%; the per-edge kernel (o1_chunk 0, the
    wavefronts in flight on ~24k consecutive edges sharing a few hundred input rows) +1.59%, and
    o1_chunk 16 +1.52% -- both outside tier C in this order, which is why -1 is the default."""
    from come_amd import _lib
    g, table, train, held, node0, seeds = c2_shape
    train = train[np.lexsort((train[:, 1], train[:, 0]))]  # G.edges() order of the kept edges
    n, lr = 5, 0.1
    rng = np.random.RandomState(32)
    neg = table[rng.randint(0, len(table), (len(held), n))].astype(np.int64)

    def losses(x):
        ref = float(-log_sigmoid(np.einsum("pd,pd->p", x[held[:, 1]].astype(np.float64),
                                           x[held[:, 0]].astype(np.float64))).sum())
        return ref, sgns_loss(x, x, held[:, 0], held[:, 1], neg)

    node = dev(node0)
    tab = dev(table)
    hot = tsi.hot_rows(tab, g.V, int(tsi.DEFAULT_HOT_P * len(table)))
    chunk = _lib.launch_opts().o1_chunk
    assert chunk == -1
    tsi.sgns_o1(node, dev(train), dev(seeds), n, tab, lr, tsi.MODE_HOGWILD, hot=hot)
    torch.cuda.synchronize()
    hog = node.cpu().numpy()
    assert np.isfinite(hog).all()
    l_hog = losses(hog)
    seq = node0.copy()
    orc.sgns_o1_hogwild(seq, train, seeds, n, table, lr, threads=1)
    l_seq = losses(seq)
    print("O1 G.edges() order, chunk %d: held-out loss (reference :26-31 / SGNS) seq %.1f / %.5f "
          "gpu-hogwild %.1f / %.5f" % ((chunk,) + l_seq + l_hog))
    for a, b in zip(l_hog, l_seq):
        assert abs(a - b) / abs(b) < 0.01, (l_hog, l_seq)  # SURVEY.md §8c tier C


def test_hot_rows_bitmap_matches_table_counts():
    """come_hot_rows: bit r set iff row r holds >= min_count slots (numpy bincount), on a
    make_table table (long uniform runs) and on an unsorted table (per-lane counting)."""
    rng = np.random.RandomState(41)
    V = 5000
    for table in (orc.make_table(rng.randint(1, 1000, V), 2_000_000),
                  rng.randint(0, V, 300_000).astype(np.uint32)):
        cnt = np.bincount(table, minlength=V)
        for mc in (1, 50, 400, 10 ** 9):
            bits = tsi.hot_rows(dev(table), V, mc).cpu().numpy().view(np.uint32)
            got = ((bits[np.arange(V) >> 5] >> (np.arange(V) & 31)) & 1).astype(bool)
            np.testing.assert_array_equal(got, cnt >= mc)


def karate_flow(seed, gpu, distributed=False):
    """adsc_Karate.py:104-137 (+ the final fit of :148) on the shipped Karate graph and the walks
    the reference's own walker produced (tests/golden/karate.npz): pre-train O1 + O2, then one
    loop of O1, O2, GMM fit (sklearn, unseeded: global numpy RNG), community step x5, GMM fit.
    gpu=True: come_amd trainers in Hogwild mode (distributed=True: the multi-GPU trainers over the
    initialised process group, their default exchange); gpu=False: the oracle (sequential C SGNS,
    numpy community step).  Returns argmax of the responsibilities per node row."""
    from sklearn.mixture import GaussianMixture
    z = np.load(os.path.join(GOLDEN, "karate.npz"))
    size, neg, ws, lr, alpha, beta, T = z["hyper"]
    size, neg, ws, T = int(size), int(neg), int(ws), int(T)
    lr, alpha, beta = float(lr), float(alpha), float(beta)
    np.random.seed(seed)
    if gpu:
        from come_amd.community_embeddings import Community2Vec
        from come_amd.context_embeddings import Context2Vec
        from come_amd.model import Model
        from come_amd.node_embeddings import Node2Vec
        model = Model((z["degree_ids"], z["degree_counts"]), size=size, table_size=T, k=2,
                      device=DEV)
        nl = Node2Vec(workers=1, negative=neg, lr=lr, distributed=distributed)
        cl = Context2Vec(window_size=ws, workers=1, negative=neg, lr=lr, distributed=distributed)
        cm = Community2Vec(model, reg_covar=1e-5, lr=lr, gmm_backend="sklearn")
        for _ in range(2):
            nl.train(model, edges=z["edges"], iter=1, chunksize=20)
            cl.train(model, paths=z["walks"], total_nodes=z["walks"].size, alpha=alpha,
                     chunksize=20)
        cm.fit(model)
        cm.train(list(z["degree_ids"]), model, beta, chunksize=20, iter=5)
        cm.fit(model)
        return torch.argmax(model.pi, 1).cpu().numpy()
    node = np.random.uniform(-1, 1, (34, size)).astype(np.float32)  # model.py:86
    ctx = np.zeros_like(node)
    table = orc.make_table(z["degree_counts"], T)
    edges = (z["edges"] - 1).astype(np.int32)
    walks = (z["walks"] - 1).astype(np.int32)
    for _ in range(2):
        orc.sgns_o1(node, edges, tsi.draw_seeds(len(edges)), neg, table, lr)
        orc.sgns_o2(node, ctx, walks, tsi.draw_seeds(len(walks)), ws, neg, table, lr, alpha)

    def fit(x):
        gm = GaussianMixture(2, covariance_type="full", reg_covar=1e-5, n_init=10)
        gm.fit(x)
        inv = np.linalg.inv(gm.covariances_.astype(np.float32))
        return gm.predict_proba(x).astype(np.float32), gm.means_.astype(np.float32), inv
    pi, mu, inv = fit(node)
    node = orc.community_train(node, pi, mu, inv, beta, lr, 5, chunksize=20)
    return np.argmax(fit(node)[0], 1)


def test_karate_nmi_hogwild_within_reference_range():
    """Karate NMI vs karate_zachary.labels over 10 seeds: the Hogwild GPU flow's mean lies in
    the reference's measured seed range 0.48-0.73 and within 0.1 of the
    sequential oracle flow's mean on the same seeds."""
    from sklearn.metrics import normalized_mutual_info_score
    z = np.load(os.path.join(GOLDEN, "karate.npz"))
    labels = z["labels"][np.argsort(z["labels"][:, 0]), 1]
    seeds = range(10)
    gpu = [normalized_mutual_info_score(labels, karate_flow(s, True)) for s in seeds]
    cpu = [normalized_mutual_info_score(labels, karate_flow(s, False)) for s in seeds]
    print("Karate NMI gpu-hogwild %s mean %.3f | oracle %s mean %.3f" % (
        np.round(gpu, 3), np.mean(gpu), np.round(cpu, 3), np.mean(cpu)))
    assert 0.48 <= np.mean(gpu) <= 0.73, gpu
    assert abs(np.mean(gpu) - np.mean(cpu)) <= 0.1, (gpu, cpu)


def _karate_ranks_worker(rank, world, port, out_dir, seeds):
    """One rank of the multi-GPU Karate flow: `world` processes on cuda:0 over gloo (RCCL needs one
    GPU per rank; the trainers' exchange arithmetic is the same)."""
    import torch.distributed as dist
    from sklearn.metrics import normalized_mutual_info_score
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z = np.load(os.path.join(GOLDEN, "karate.npz"))
    labels = z["labels"][np.argsort(z["labels"][:, 0]), 1]
    nmi = [normalized_mutual_info_score(labels, karate_flow(s, True, distributed=True))
           for s in seeds]
    np.save(os.path.join(out_dir, "nmi%d.npy" % rank), np.array(nmi))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_karate_nmi_multi_rank_not_below_reference_range(tmp_path, world):
    """The reference's own quality check (adsc_Karate.py:104-148: NMI of the community assignment
    vs karate_zachary.labels) under N-replica training: `world` ranks (processes on one GPU, gloo)
    run the Karate flow with Context2Vec / Node2Vec(distributed=True) and the default exchange;
    asserted: over 10 seeds the mean NMI is NOT BELOW the bottom of the reference's seed range
    0.48-0.73, and the replicas agree (every rank computes the same assignments).
    Not asserted: that it stays inside the range -- it does at 2 ranks (mean 0.683) but lands
    ABOVE it at 4 (0.745, r05e: the replicas' mean carries less SGD noise than the reference's
    Hogwild), which is why distributed training is documented as non-parity."""
    import socket
    import torch.multiprocessing as mp
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    seeds = list(range(10))
    mp.spawn(_karate_ranks_worker, args=(world, port, str(tmp_path), seeds), nprocs=world,
             join=True)
    nmi = [np.load(str(tmp_path / ("nmi%d.npy" % r))) for r in range(world)]
    for r in range(1, world):
        np.testing.assert_array_equal(nmi[r], nmi[0])
    print("Karate NMI, %d ranks: %s mean %.3f" % (world, np.round(nmi[0], 3), nmi[0].mean()))
    assert nmi[0].mean() >= 0.48, nmi[0]


# ---- configs[4]/C5 (d = 256, n = 10) -----------------------------------------------------------

def c5_launch_losses(x, fx, runs=2):
    """Held-out losses of `runs` product launches (streaming kernel k_sgns_o2_stream<4, true, 10>,
    hot-row bitmap, packed table) over the inputs `x`, compared against fixture `fx`."""
    from tierc_inputs import C5_HYPER, compact_loss
    assert x.digest == fx["inputs_sha256"], "inputs differ from the fixture's"
    w, n, lr = C5_HYPER["window"], C5_HYPER["negative"], C5_HYPER["lr"]
    ri, rp, rn = x.heldout(w, n)
    l0 = None
    tab = dev(x.table)
    # the product's contended rows for this row width (Model.hot_rows: default_hot_share(d))
    hot = tsi.hot_rows(tab, x.g.V, int(tsi.default_hot_share(x.node0.shape[1]) * len(x.table)))
    packed = tsi.pack_table(tab)
    assert packed is not None
    walks, seeds = dev(x.train), dev(x.seeds)
    node0 = torch.from_numpy(x.node0)
    l_hog = []
    for _ in range(runs):
        node = node0.to(DEV)
        ctx = torch.zeros_like(node)
        if l0 is None:
            l0 = compact_loss(node, ctx, ri, rp, rn)
            assert abs(l0 - fx["init_loss"]) < 1e-9
        tsi.sgns_o2(node, ctx, walks, seeds, w, n, packed, lr, 1.0, tsi.MODE_HOGWILD, hot=hot)
        torch.cuda.synchronize()
        l_hog.append(compact_loss(node, ctx, ri, rp, rn))
        del node, ctx
        torch.cuda.empty_cache()
    rel = [(v - fx["seq_loss"]) / fx["seq_loss"] for v in l_hog]
    print("V=%d: held-out loss init %.5f  seq (fixture) %.5f  gpu-hogwild %s  rel %s" % (
        x.g.V, l0, fx["seq_loss"], " ".join("%.5f" % v for v in l_hog),
        " ".join("%+.5f" % r for r in rel)))
    assert fx["seq_loss"] < l0 - 0.5
    return rel


def test_o2_hogwild_c5():
    """Tier C at configs[4]/C5 itself: Chung-Lu 10M nodes / ~100M edges (seed 4), d = 256,
    n = 10, T = 1e8, lr 0.1, ONE launch of 131,072 walks (1.0e8 pair updates, device-walker
    stream from distinct random starts) of the product's Hogwild path: held-out loss of two
    launches within 1% of the sequential oracle's, a committed fixture (tests/golden/
    tierc_c5_seq.json, scripts/make_tierc_fixture_host.py c5: the same inputs built on the host
    with the walker's CPU restatement; tests/tierc_inputs.py C5, matched by digest).  The 10
    GB tables never leave the device whole (tierc_inputs.compact_loss)."""
    import json
    from tierc_inputs import c5_inputs
    fx = json.load(open(os.path.join(GOLDEN, "tierc_c5_seq.json")))
    rel = c5_launch_losses(c5_inputs(device=DEV), fx)
    assert max(abs(r) for r in rel) < 0.01, rel  # SURVEY.md §8c tier C


def test_o2_hogwild_c5_kernel_on_1m_nodes():
    """Tier C for C5's kernel on a 1M-node graph of C5's generator, where rows hold 10x the table
    share they hold at C5's 10M nodes (the top row 5.0e-4 vs 1.6e-4): held-out loss of two product
    launches within 1% of the sequential oracle's (tests/golden/tierc_c5_1m_seq.json).  Until
    round 5 this failed at -1.8% (the test then only guarded -2.5% .. +1%): rows between 8e-7 and
    5e-6 of the table were written with plain stores, and on this graph each of their updates races
    0.1-0.2 others in flight, so enough updates were lost to damp the SGD noise below the
    reference's.  The product now makes them contended rows at d > 128 (default_hot_share:
    -0.40%, profiles/r06_hot_share.txt)."""
    import json
    from tierc_inputs import c5_1m_inputs
    fx = json.load(open(os.path.join(GOLDEN, "tierc_c5_1m_seq.json")))
    rel = c5_launch_losses(c5_1m_inputs(), fx)
    assert max(abs(r) for r in rel) < 0.01, rel  # SURVEY.md §8c tier C


# ---- the multi-GPU path: N ranks' delta-sum training --------------------------

@pytest.fixture(scope="module")
def c3_1m():
    import json
    from tierc_inputs import c3_1m_inputs
    fx = json.load(open(os.path.join(GOLDEN, "tierc_c3_1m_seq.json")))
    x = c3_1m_inputs()
    assert x.digest == fx["inputs_sha256"], "inputs differ from the fixture's"
    ri, rp, rn = x.heldout(5, 5)
    assert abs(sgns_loss(x.node0, np.zeros_like(x.node0), ri, rp, rn) - fx["init_loss"]) < 1e-9
    tab = dev(x.table)
    hot = tsi.hot_rows(tab, x.g.V, int(tsi.DEFAULT_HOT_P * len(x.table)))
    return fx, x, (ri, rp, rn), tsi.pack_table(tab), hot


def test_o2_hogwild_at_the_bench_launch(c3_1m):
    """Tier C at the bench's own launch: ONE Hogwild launch of 1,048,576 walks (8.07e8 pair
    updates, the product's Context2Vec.batch_walks) on C3's graph, against the committed
    sequential-oracle fixture of the same walks (tests/golden/tierc_c3_1m_seq.json, 41 minutes of
    one core): within 1%."""
    fx, x, (ri, rp, rn), packed, hot = c3_1m
    node = torch.from_numpy(x.node0).to(DEV)
    ctx = torch.zeros_like(node)
    tsi.sgns_o2(node, ctx, dev(x.train), dev(x.seeds), 5, 5, packed, 0.1, 1.0, tsi.MODE_HOGWILD,
                hot=hot)
    torch.cuda.synchronize()
    loss = sgns_loss(node.cpu().numpy(), ctx.cpu().numpy(), ri, rp, rn)
    del node, ctx
    torch.cuda.empty_cache()
    rel = (loss - fx["seq_loss"]) / fx["seq_loss"]
    print("C3 bench launch (1,048,576 walks): held-out loss %.5f vs seq %.5f (rel %+.5f)" % (
        loss, fx["seq_loss"], rel))
    assert abs(rel) < 0.01, (loss, fx["seq_loss"])


# Held-out loss of the trainers' multi-rank exchange (touched_mean) relative to the sequential
# oracle, measured with >= 4 exchanges per rank (profiles/r05_tierc_replicas_*):
# -13..-17% at 2-8 ranks.  Two-sided bands around those values: the exchange must keep training
# BELOW the reference's noise floor by about this much -- a drift either way fails.
TOUCHED_MEAN_BAND = (-0.21, -0.09)


@pytest.mark.parametrize("world", [8, 4, 2])
def test_o2_multi_rank_exchange_regression_band(c3_1m, world):
    """`world` ranks simulated on one GPU (tests/replica_sim.py: each rank its own replica and
    contiguous walk shard, the product's launches, DeltaAllReduce's fused passes, the trainers'
    default touched_mean combine and overlapped protocol, RCCL replaced by a sum over the
    replicas) over the C3 bench launch's 1,048,576 walks with 32,768 walks per rank between
    exchanges: 16 / 8 / 4 exchanges per rank at 2 / 4 / 8 ranks.

    NOT tier C, and no periodic exchange is (the full sweep): summing the ranks'
    deltas diverges (held-out loss 6-100 vs the oracle's 2.56); keeping one rank's delta per row
    ("pick") matches the SGD noise floor but keeps 1/N of the shared rows' progress (+1 / +5 /
    +10% at 2 / 4 / 8 ranks) and diverges when overlapped; averaging (touched_mean, the trainers'
    default) trains to a LOWER held-out loss (-13..-17%: the mean of N replicas carries less SGD
    noise).  Asserted: the default stays in that two-sided band (TOUCHED_MEAN_BAND)."""
    from replica_sim import train_replicas
    fx, x, (ri, rp, rn), packed, hot = c3_1m
    st = {}
    node, ctx = train_replicas(x.node0, np.zeros_like(x.node0), x.train, x.seeds, world,
                               1 << 15, 5, 5, packed, hot, 0.1, stats=st)
    loss = sgns_loss(node.cpu().numpy(), ctx.cpu().numpy(), ri, rp, rn)
    del node, ctx
    torch.cuda.empty_cache()
    rel = (loss - fx["seq_loss"]) / fx["seq_loss"]
    print("C3 1M walks, %d ranks, %d exchanges (touched_mean): held-out loss %.5f vs seq %.5f "
          "(rel %+.5f)" % (world, st["exchanges"], loss, fx["seq_loss"], rel))
    assert st["exchanges"] >= 4
    assert np.isfinite(loss) and TOUCHED_MEAN_BAND[0] < rel < TOUCHED_MEAN_BAND[1], \
        (loss, fx["seq_loss"])


# ranks -> (exchanges per rank, band) at the default period over the 4M-walk fixture: 2 ranks make
# 4 exchanges (measured -12.4%, r05); 8 ranks -- the C5 topology -- make ONE (their whole shard is
# one period; measured -19.4% in round 3, profiles/r04_tierc_replicas_c3_4m.json), a band of its own
# around that (the trainers' default period at 8 ranks had no quality test).
DEFAULT_PERIOD_CASES = {2: (4, TOUCHED_MEAN_BAND), 8: (1, (-0.25, -0.12))}


@pytest.mark.parametrize("world", [2, 8])
def test_o2_default_period_over_4m_walks(world):
    """The multi-GPU default period (context_embeddings.DEFAULT_SYNC_WALKS = 524,288 walks per rank
    between exchanges, overlapped, touched_mean) over the 4,194,304 walks of the C3_4M fixture
    (tests/golden/tierc_c3_4m_seq.json: the sequential oracle, ~3 h of one core) on 2 ranks (4
    exchanges per rank, the 1M-walk band) and 8 ranks (1 exchange: DEFAULT_PERIOD_CASES)."""
    import json
    from come_amd.context_embeddings import DEFAULT_SYNC_WALKS
    from replica_sim import train_replicas
    from tierc_inputs import c3_4m_inputs
    fx = json.load(open(os.path.join(GOLDEN, "tierc_c3_4m_seq.json")))
    x = c3_4m_inputs()
    assert x.digest == fx["inputs_sha256"], "inputs differ from the fixture's"
    ri, rp, rn = x.heldout(5, 5)
    tab = dev(x.table)
    hot = tsi.hot_rows(tab, x.g.V, int(tsi.DEFAULT_HOT_P * len(x.table)))
    st = {}
    node, ctx = train_replicas(x.node0, np.zeros_like(x.node0), x.train, x.seeds, world,
                               DEFAULT_SYNC_WALKS, 5, 5, tsi.pack_table(tab), hot, 0.1, stats=st)
    loss = sgns_loss(node.cpu().numpy(), ctx.cpu().numpy(), ri, rp, rn)
    del node, ctx
    torch.cuda.empty_cache()
    rel = (loss - fx["seq_loss"]) / fx["seq_loss"]
    print("C3 4M walks, %d ranks x %d walks per exchange, %d exchanges: held-out loss %.5f vs seq "
          "%.5f (rel %+.5f)" % (world, DEFAULT_SYNC_WALKS, st["exchanges"], loss, fx["seq_loss"],
                                rel))
    exchanges, band = DEFAULT_PERIOD_CASES[world]
    assert st["exchanges"] == exchanges
    assert np.isfinite(loss) and band[0] < rel < band[1], (loss, fx["seq_loss"])


@pytest.fixture(scope="module")
def c2_reference_order(c2_shape):
    """C2 in the reference's own edge order (np.array(G.edges()), node_embeddings.py:39) with 4
    passes' worth of per-edge seeds (Node2Vec.train(iter=4)) and the sequential oracle's held-out
    losses after them (one core, ~1 s per pass)."""
    g, table, train, held, node0, _ = c2_shape
    train = train[np.lexsort((train[:, 1], train[:, 0]))]
    srng = np.random.RandomState(33)
    seeds = [srng.randint(0, 2 ** 48, len(train), dtype=np.int64).astype(np.uint64)
             for _ in range(4)]
    neg = table[np.random.RandomState(32).randint(0, len(table), (len(held), 5))].astype(np.int64)

    def losses(x):
        ref = float(-log_sigmoid(np.einsum("pd,pd->p", x[held[:, 1]].astype(np.float64),
                                           x[held[:, 0]].astype(np.float64))).sum())
        return ref, sgns_loss(x, x, held[:, 0], held[:, 1], neg)
    seq = node0.copy()
    for sd in seeds:
        orc.sgns_o1_hogwild(seq, train, sd, 5, table, 0.1, threads=1)
    tab = dev(table)
    hot = tsi.hot_rows(tab, g.V, int(tsi.DEFAULT_HOT_P * len(table)))
    return g, train, node0, seeds, tsi.pack_table(tab), hot, losses, losses(seq)


# |held-out loss / sequential oracle's - 1| of Node2Vec(distributed=True)'s exchange (touched_mean,
# one per pass) after 4 passes, measured (profiles/r05_tierc_replicas_c2_4pass.json): reference
# loss / SGNS loss -1.4 / -2.0% at 2 ranks, +0.5 / -0.5% at 4, +3.1 / +1.9% at 8 -- tier C (1%) at 4
# ranks only; the bands guard the measured values.
O1_MULTI_RANK_BAND = {2: 0.03, 4: 0.01, 8: 0.045}


@pytest.mark.parametrize("world", [2, 4, 8])
def test_o1_multi_rank_exchange_tier_c(c2_reference_order, world):
    """Multi-GPU O1 (Node2Vec(distributed=True), node_embeddings.py:35-106): `world` ranks
    simulated on one GPU (tests/replica_sim.train_replicas_o1: each rank its contiguous shard of
    every pass, the product's launch, one blocking exchange per pass with the trainers' default
    combine, RCCL replaced by a sum over the replicas), 4 passes = 4 exchanges, in the reference's
    G.edges() order: both held-out losses (the reference's :26-31 and SGNS) within
    O1_MULTI_RANK_BAND of the sequential oracle's, either side (tier C's 1% at 4 ranks)."""
    from come_amd.node_embeddings import Node2Vec
    from replica_sim import train_replicas_o1
    g, train, node0, seeds, packed, hot, losses, l_seq = c2_reference_order
    st = {}
    x = train_replicas_o1(node0, train, seeds, world, None, 5, packed, hot, 0.1,
                          combine=Node2Vec().combine, stats=st)
    l = losses(x.cpu().numpy())
    rel = [(a - b) / b for a, b in zip(l, l_seq)]
    print("O1 %d ranks, %d exchanges: held-out (reference / SGNS) %.1f / %.5f vs seq %.1f / %.5f "
          "(rel %+.4f / %+.4f)" % ((world, st["exchanges"]) + l + l_seq + tuple(rel)))
    assert st["exchanges"] == 4
    assert max(abs(r) for r in rel) < O1_MULTI_RANK_BAND[world], (l, l_seq)

