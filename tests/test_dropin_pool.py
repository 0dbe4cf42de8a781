"""The per-call drop-ins (training_sdg_inner.train_o2 / train_o1, pyx:407-509) under the
reference's own worker pool: `workers` Python threads lifting jobs of `chunksize` walks (edges) off
a bounded queue and calling the drop-in once per walk (edge) on shared tables, exactly as
Context2Vec.train (ADSCModel/context_embeddings.py:68-109) and Node2Vec.train
(ADSCModel/node_embeddings.py:48-100) drive the Cython module.

Concurrent calls are Hogwild, so the bar is tier C: the held-out SGNS loss after
one pass of the pool within 1% of the sequential oracle's (oracle/come_oracle_mt.c, threads=1) on
the same walks.  Routes (training_sdg_inner "per-call drop-ins"):
  * host    -- numpy tables, the reference's case: libcome's host twin through _come_pyext, GIL
               released per call (CPU; runs in the CPU suite);
  * device  -- CUDA tensor tables: one sequential-mode kernel launch per call (GPU);
  * locked  -- numpy tables forced down the device route (set_numpy_route("device")): device
               mirrors, upload -> launch -> writeback serialised by the route's lock (GPU).
Each test also checks the drop-in's return values (the non-None counts) summed over the pool.
"""
import threading
from queue import Queue

import numpy as np
import pytest

from oracle import oracle as orc
from tierc_inputs import heldout_o2_pairs, log_sigmoid, sgns_loss

import come_amd.training_sdg_inner as tsi

WORKERS, CHUNK = 4, 150  # 4 workers; the trainers' chunksize default (context_embeddings.py:41)
ROUTES = ["host", pytest.param("device", marks=pytest.mark.gpu),
          pytest.param("locked", marks=pytest.mark.gpu)]


class Vocab(object):
    """utils/embedding.py Vocab: the drop-ins read only .index."""
    __slots__ = ("index",)

    def __init__(self, i):
        self.index = i


def run_pool(items, call, workers=WORKERS, chunksize=CHUNK):
    """context_embeddings.py:68-104: a Queue of at most 2*workers jobs, `workers` threads each
    summing call(item) over its job under a shared lock; returns the summed counts."""
    jobs = Queue(maxsize=2 * workers)
    lock = threading.Lock()
    count = [0]
    errors = []

    def worker_train():
        while True:
            job = jobs.get()
            if job is None:
                break
            try:
                n = sum(call(it) for it in job)
            except Exception as e:  # surfaced below: a worker exception must fail the test
                errors.append(e)
                n = 0
            with lock:
                count[0] += n

    threads = [threading.Thread(target=worker_train, daemon=True) for _ in range(workers)]
    for t in threads:
        t.start()
    for s in range(0, len(items), chunksize):
        jobs.put(items[s:s + chunksize])
    for _ in threads:
        jobs.put(None)
    for t in threads:
        t.join()
    assert not errors, errors[0]
    return count[0]


def _tables(route, *arrays):
    """The tables as the route takes them, and a function returning them as numpy."""
    if route in ("host", "locked"):
        return arrays, lambda t: t
    import torch
    dev = torch.device("cuda", 0)
    out = []
    for a in arrays:
        a = np.ascontiguousarray(a)
        if a.dtype == np.uint32:
            a = a.view(np.int32)
        out.append(torch.from_numpy(a).to(dev))
    return out, lambda t: t.cpu().numpy()


@pytest.fixture(scope="module")
def o2_shape():
    """C3's shape at 100k nodes (Chung-Lu gamma 2.5, mean degree 20, d=128, n=5, w=5, L=80,
    lr 0.1), a 1e7-slot table; 10,000 training walks (~7.7e6 pair updates) and 2,000 held out,
    from the device walker's CPU restatement."""
    from come_amd.graph import chung_lu
    g = chung_lu(100_000, 20.0, gamma=2.5, seed=21)
    table = orc.make_table(g.degree.astype(np.float64), 10_000_000)
    rng = np.random.RandomState(23)
    starts = rng.choice(g.V, 12_000, replace=False).astype(np.int32)
    walks = orc.philox_walks(g.rowptr, g.col, starts, 80, 0.0, seed=22)
    node0 = rng.uniform(-1, 1, (g.V, 128)).astype(np.float32)
    seeds = rng.randint(0, 2 ** 48, 10_000, dtype=np.int64).astype(np.uint64)
    return g, table, walks[:10_000], walks[10_000:], node0, seeds


@pytest.mark.parametrize("route", ROUTES)
def test_o2_dropin_under_reference_worker_pool(o2_shape, route):
    g, table, train, held, node0, seeds = o2_shape
    w, n, lr = 5, 5, 0.1
    rows_in, rows_pos, rows_neg = heldout_o2_pairs(held, w, n, table, 200_000, 24)
    ctx0 = np.zeros_like(node0)
    l0 = sgns_loss(node0, ctx0, rows_in, rows_pos, rows_neg)
    vocab = [Vocab(i) for i in range(g.V)]
    paths = [[vocab[x] if x >= 0 else None for x in row] for row in train]
    (node, ctx, tab), host = _tables(route, node0.copy(), ctx0.copy(), table)
    prev = tsi.set_numpy_route("device" if route == "locked" else "host")
    try:
        np.random.seed(5)
        count = run_pool(paths, lambda p: tsi.train_o2(node, ctx, p, lr, n, w, tab, py_alpha=1.0,
                                                       py_size=128, py_work=None))
    finally:
        tsi.set_numpy_route(prev)
    assert count == int((train >= 0).sum())
    hn, hc = host(node), host(ctx)
    assert np.isfinite(hn).all() and np.isfinite(hc).all()
    l_pool = sgns_loss(hn, hc, rows_in, rows_pos, rows_neg)
    sn, sc = node0.copy(), ctx0.copy()
    orc.sgns_o2_hogwild(sn, sc, train, seeds, w, n, table, lr, 1.0, threads=1)
    l_seq = sgns_loss(sn, sc, rows_in, rows_pos, rows_neg)
    print("O2 pool (%s, %d workers): init %.5f  seq %.5f  pool %.5f  rel %.5f" % (
        route, WORKERS, l0, l_seq, l_pool, (l_pool - l_seq) / l_seq))
    assert l_seq < l0 - 0.05
    assert abs(l_pool - l_seq) / l_seq < 0.01, (l_pool, l_seq)  # SURVEY.md §8c tier C


@pytest.fixture(scope="module")
def o1_shape():
    return o1_inputs()


def o1_inputs():
    """C2's generator at 10 blocks x 500 nodes (p_in 0.03: ~37k edges), d=128, n=5, lr 0.1, the
    reference's init (model.py:86: uniform(-1, 1)); 5% of the edges held out, the rest shuffled."""
    from come_amd.graph import sbm
    g = sbm(10, 500, 0.03, 4.04e-5, seed=3)
    rng = np.random.RandomState(31)
    e = g.edges[rng.permutation(len(g.edges))].astype(np.int32)
    k = len(e) // 20
    table = orc.make_table(g.degree.astype(np.float64), 10_000_000)
    node0 = rng.uniform(-1, 1, (g.V, 128)).astype(np.float32)
    return g, table, e[k:], e[:k], node0


@pytest.mark.parametrize("route", ROUTES)
def test_o1_dropin_under_reference_worker_pool(o1_shape, route):
    """Tier C for O1 against the sequential oracle fed the pool's own seed stream (the global
    RNG from the same seed, in call order).  O1 from the reference's init at lr 0.1 is chaotic at
    this size: two sequential runs that differ only in their seed stream land up to a few percent
    apart on the reference's loss (node_embeddings.py:26-31), so the bar is 1% or twice that
    measured seed spread, whichever is larger, and the spread is printed beside the result."""
    g, table, train, held, node0 = o1_shape
    n, lr = 5, 0.1
    rng = np.random.RandomState(32)
    neg = table[rng.randint(0, len(table), (len(held), n))].astype(np.int64)

    def losses(x):  # node_embeddings.py:26-31 over the held-out edges, and the SGNS loss
        ref = float(-log_sigmoid(np.einsum("pd,pd->p", x[held[:, 1]].astype(np.float64),
                                           x[held[:, 0]].astype(np.float64))).sum())
        return ref, sgns_loss(x, x, held[:, 0], held[:, 1], neg)

    l0 = losses(node0)
    vocab = [Vocab(i) for i in range(g.V)]
    items = [[vocab[u], vocab[v]] for u, v in train]
    (node, tab), host = _tables(route, node0.copy(), table)
    prev = tsi.set_numpy_route("device" if route == "locked" else "host")
    try:
        np.random.seed(6)
        count = run_pool(items, lambda e: tsi.train_o1(node, e, lr, n, tab, py_size=128))
    finally:
        tsi.set_numpy_route(prev)
    assert count == 2 * len(items)
    x = host(node)
    assert np.isfinite(x).all()
    l_pool = losses(x)
    seqs = []
    for seed in (6, 60):
        np.random.seed(seed)
        sd = tsi.draw_seeds(len(train))
        s = node0.copy()
        orc.sgns_o1_hogwild(s, train, sd, n, table, lr, threads=1)
        seqs.append(losses(s))
    l_seq = seqs[0]
    spread = [abs(a - b) / abs(b) for a, b in zip(seqs[1], seqs[0])]
    print("O1 pool (%s, %d workers): init %.1f / %.5f  seq %.1f / %.5f  pool %.1f / %.5f  "
          "seed spread %.4f / %.4f" % ((route, WORKERS) + l0 + l_seq + l_pool + tuple(spread)))
    assert l_seq[1] < l0[1] - 0.05
    for a, b, sp in zip(l_pool, l_seq, spread):
        assert abs(a - b) / abs(b) < max(0.01, 2 * sp), (l_pool, l_seq, spread)  # tier C


@pytest.mark.gpu
def test_locked_route_pool_equals_its_serial_replay(o2_shape):
    """No lost updates on the device route with numpy tables: under the worker pool, the route's
    lock makes every call's upload -> launch -> writeback atomic, so the pool's result must equal
    -- bit for bit -- the host twin run sequentially over the calls in the order they took the
    lock, with the seeds they drew (the sequential kernel and the twin agree bit for bit).  Hub
    rows appear in nearly every call, so a single interleaved upload or writeback would show."""
    import threading as th
    from come_amd import cpu
    g, table, train, held, node0, seeds = o2_shape
    w, n, lr = 5, 5, 0.1
    train = train[:1500]
    vocab = [Vocab(i) for i in range(g.V)]
    paths = [[vocab[x] if x >= 0 else None for x in row] for row in train]
    log = []
    orig = tsi._device_o2

    def logged(node, ctx, rows, nr, *rest):
        log.append((rows.copy(), nr))  # runs under the route's lock: execution order
        return orig(node, ctx, rows, nr, *rest)
    node, ctx = node0.copy(), np.zeros_like(node0)
    prev = tsi.set_numpy_route("device")
    tsi._device_o2 = logged
    try:
        np.random.seed(5)
        run_pool(paths, lambda p: tsi.train_o2(node, ctx, p, lr, n, w, table))
    finally:
        tsi._device_o2 = orig
        tsi.set_numpy_route(prev)
    assert len(log) == len(train) and isinstance(tsi._DEVICE_LOCK, type(th.Lock()))
    rn, rc = node0.copy(), np.zeros_like(node0)
    walks = np.stack([r for r, _ in log]).astype(np.int32)
    sd = np.array([s for _, s in log], np.uint64)
    cpu.sgns_o2(rn, rc, walks, sd, w, n, table, lr, 1.0, cpu.MODE_SEQUENTIAL, threads=1)
    np.testing.assert_array_equal(node, rn)
    np.testing.assert_array_equal(ctx, rc)


def test_host_route_matches_sequential_twin_bit_for_bit():
    """One thread: the host route (seeds from the global RNG, per call) equals the host twin run
    in sequential mode on the same seeds -- the route adds nothing but the call protocol."""
    rng = np.random.RandomState(8)
    V, d, T = 3000, 128, 50_000
    table = orc.make_table(rng.randint(1, 40, V), T)
    node0 = rng.uniform(-0.5, 0.5, (V, d)).astype(np.float32)
    ctx0 = rng.uniform(-0.1, 0.1, (V, d)).astype(np.float32)
    walks = rng.randint(0, V, (40, 60)).astype(np.int32)
    walks[3, 10:] = -1
    walks[7, 5] = -1
    vocab = [Vocab(i) for i in range(V)]
    a_n, a_c = node0.copy(), ctx0.copy()
    np.random.seed(9)
    for row in walks:
        tsi.train_o2(a_n, a_c, [vocab[x] if x >= 0 else None for x in row], 0.1, 5, 5, table)
    np.random.seed(9)
    seeds = tsi.draw_seeds(len(walks))
    from come_amd import cpu
    b_n, b_c = node0.copy(), ctx0.copy()
    cpu.sgns_o2(b_n, b_c, walks, seeds, 5, 5, table, 0.1, 1.0, cpu.MODE_SEQUENTIAL, threads=1)
    np.testing.assert_array_equal(a_n, b_n)
    np.testing.assert_array_equal(a_c, b_c)
    edges = rng.randint(0, V, (200, 2)).astype(np.int32)
    a = node0.copy()
    np.random.seed(10)
    for u, v in edges:
        assert tsi.train_o1(a, [vocab[u], vocab[v]], 0.2, 5, table) == 2
    np.random.seed(10)
    eseeds = tsi.draw_seeds(len(edges))
    b = node0.copy()
    cpu.sgns_o1(b, edges, eseeds, 5, table, 0.2, cpu.MODE_SEQUENTIAL, threads=1)
    np.testing.assert_array_equal(a, b)


def test_host_route_argument_errors():
    """Wrong dtypes raise TypeError naming the argument (the reference would read garbage); a
    non-uint32 integer table is converted (the RNG is drawn once either way)."""
    V, d = 50, 8
    node = np.zeros((V, d), np.float32)
    ctx = np.zeros((V, d), np.float32)
    path = [Vocab(i) for i in range(10)]
    with pytest.raises(TypeError, match="py_node_embedding"):
        tsi.train_o2(node.astype(np.float64), ctx, path, 0.1, 2, 2, np.arange(V, dtype=np.uint32))
    with pytest.raises(TypeError):
        tsi.train_o2(node[:, ::2], ctx[:, ::2], path, 0.1, 2, 2, np.arange(V, dtype=np.uint32))
    np.random.seed(1)
    tsi.train_o2(node, ctx, path, 0.1, 2, 2, np.arange(V, dtype=np.int64))
    after_int64 = np.random.randint(0, 1 << 30)
    np.random.seed(1)
    n2, c2 = np.zeros_like(node), np.zeros_like(ctx)
    tsi.train_o2(n2, c2, path, 0.1, 2, 2, np.arange(V, dtype=np.uint32))
    assert np.random.randint(0, 1 << 30) == after_int64
    np.testing.assert_array_equal(node, n2)
    assert tsi.train_o2(node, ctx, [], 0.1, 2, 2, np.arange(V, dtype=np.uint32)) == 0
    assert tsi.train_o2(node, ctx, [None, Vocab(1), None], 0.1, 2, 2,
                        np.arange(V, dtype=np.uint32)) == 1
