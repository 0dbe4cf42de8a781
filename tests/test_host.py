"""Host-side logic of the product package (no GPU): the native make_table, pair counting, seed
drawing, walk -> row conversion, Model construction, text IO, sharding."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as orc

import come_amd.training_sdg_inner as tsi
from come_amd import _lib, io_utils
from come_amd.distributed import shard_range, shard_walks
from come_amd.model import Model


def native_make_table(counts_by_row, T, power=0.75):
    c = np.zeros(len(counts_by_row) + 1, np.float64)
    c[1:] = counts_by_row
    out = np.zeros(int(T), np.uint32)
    _lib.check(_lib.lib().come_make_table(_lib.ptr(c), len(counts_by_row), _lib.ptr(out), int(T),
                                         power), "make_table")
    return out


@pytest.mark.parametrize("seed,V,T", [(0, 2, 10), (1, 3, 7), (2, 10, 1000), (3, 1000, 100000),
                                      (4, 5000, 12345), (5, 50, 49), (6, 3000, 3000),
                                      (7, 200, 1)])
def test_native_make_table_equals_literal_loop(seed, V, T):
    rng = np.random.RandomState(seed)
    counts = np.maximum(1, (rng.pareto(1.2, V) * 5).astype(np.int64))
    np.testing.assert_array_equal(native_make_table(counts, T), orc.make_table(counts, T))


def test_native_make_table_golden():
    import hashlib
    z = np.load(os.path.join(GOLDEN, "make_table.npz"))
    for name in z["names"]:
        t = native_make_table(z[name + "_counts"], int(z[name + "_T"]))
        if name + "_table" in z:
            np.testing.assert_array_equal(t, z[name + "_table"])
        else:
            assert hashlib.sha256(t.tobytes()).hexdigest() == str(z[name + "_sha256"])


def test_native_make_table_clamp_heavy_tail():
    counts = np.array([1] * 5 + [10 ** 6])  # last id carries almost all mass -> clamp to V-1
    np.testing.assert_array_equal(native_make_table(counts, 5000), orc.make_table(counts, 5000))


def test_exp_table_native_equals_oracle():
    np.testing.assert_array_equal(tsi.exp_table(), orc.exp_table())
    assert tsi.init() == tsi.FAST_VERSION == 0


def test_count_pairs():
    rng = np.random.RandomState(0)
    for L, w in [(80, 5), (20, 3), (3, 5), (1, 2), (10, 0)]:
        walks = rng.randint(0, 50, (7, L)).astype(np.int32)
        n = tsi.count_o2_pairs(walks, w)
        if L >= w + 1:
            assert n == 7 * (2 * w * L - w * (w + 1))
        node = np.zeros((50, 4), np.float32)
        ctx = np.zeros((50, 4), np.float32)
        assert n == orc.sgns_o2(node, ctx, walks, np.zeros(7, np.uint64), w, 0,
                                np.zeros(1, np.uint32), 0.1, 1.0)
    walks[:, ::3] = -1
    node = np.zeros((50, 4), np.float32)
    assert tsi.count_o2_pairs(walks, 2) == orc.sgns_o2(
        node, node.copy(), walks, np.zeros(7, np.uint64), 2, 0, np.zeros(1, np.uint32), 0.1, 1.0)


def test_draw_seeds_matches_per_call_draws():
    """pyx:427/477: two np.random.randint(0, 2**24) draws per call, in call order."""
    np.random.seed(77)
    fast = tsi.draw_seeds(1000)
    np.random.seed(77)
    slow = [(2 ** 24) * np.random.randint(0, 2 ** 24) + np.random.randint(0, 2 ** 24)
            for _ in range(1000)]
    np.testing.assert_array_equal(fast, np.array(slow, np.uint64))
    assert (fast < 2 ** 48).all()


def karate_model(**kw):
    z = np.load(os.path.join(GOLDEN, "karate.npz"))
    deg = dict(zip(z["degree_ids"].tolist(), z["degree_counts"].tolist()))
    np.random.seed(42)
    return Model(deg, size=2, table_size=int(z["hyper"][6]), k=2, device="cpu", **kw), z


def test_model_matches_reference_init():
    m, z = karate_model()
    np.testing.assert_array_equal(m.node_embedding.numpy(), z["node_init"])
    np.testing.assert_array_equal(np.bincount(m.table_host, minlength=34), z["table_bincount"])
    assert m.vocab[1].index == 0 and m.vocab[34].index == 33
    assert (m.context_embedding.numpy() == 0).all()
    assert tuple(m.pi.shape) == (34, 2) and tuple(m.inv_covariance_mat.shape) == (2, 2, 2)


def test_walks_to_rows_drops_oov_and_pads():
    from come_amd.embedding import walks_to_rows
    m, _ = karate_model()
    rows = walks_to_rows(m, [[1, 2, 99, 3], [34], [0, 5]])
    np.testing.assert_array_equal(rows, [[0, 1, 2], [33, -1, -1], [4, -1, -1]])
    arr = np.array([[1, 2, 3], [4, 5, 6]])
    np.testing.assert_array_equal(walks_to_rows(m, arr), arr - 1)


def test_down_sampling_draw_count():
    from come_amd.embedding import walks_to_rows
    m, _ = karate_model(down_sampling=0.005)
    p = m.sample_probability_rows()
    walk = np.arange(1, 35)
    low = int((p < 1).sum())
    assert 0 < low < 34
    np.random.seed(5)
    walks_to_rows(m, [walk])
    after = np.random.random_sample()
    np.random.seed(5)
    np.random.random_sample(low)
    assert np.random.random_sample() == after


def test_save_load_roundtrip(tmp_path):
    m, _ = karate_model()
    m.save(str(tmp_path), "karate")
    m2 = Model.load_model(str(tmp_path), "karate", device="cpu")
    np.testing.assert_array_equal(m2.node_embedding.numpy(), m.node_embedding.numpy())
    np.testing.assert_array_equal(m2.table_host, m.table_host)
    assert m2.vocab[34].index == 33


def test_io_roundtrip(tmp_path):
    x = np.random.RandomState(1).randn(5, 3).astype(np.float32)
    io_utils.save_embedding(x, "e", path=str(tmp_path))
    lines = open(os.path.join(str(tmp_path), "e.txt")).read().splitlines()
    assert lines[0].split("\t")[0] == "1" and len(lines) == 5
    np.testing.assert_allclose(io_utils.load_embedding("e", path=str(tmp_path)), x, rtol=1e-6)
    io_utils.save_ground_true("lab", [1, 2, 2], path=str(tmp_path))
    os.rename(os.path.join(str(tmp_path), "lab.txt"), os.path.join(str(tmp_path), "lab.labels"))
    labels, k = io_utils.load_ground_true(path=str(tmp_path), file_name="lab")
    assert labels == [1, 2, 2] and k == 2


def test_o1_edges_down_sampled_like_prepare_sentences():
    """Node2Vec's edge rows go through the reference's down-sampling draw (prepare_sentences,
    embedding.py:126-136): one draw per endpoint with sample_probability < 1, edge by edge; an
    edge that loses an endpoint is skipped (the reference reads an uninitialised index there)."""
    from come_amd.node_embeddings import Node2Vec
    m, z = karate_model(down_sampling=0.005)
    edges = z["edges"]
    p = m.sample_probability_rows()
    rows = edges - 1
    draws = int((p[rows] < 1).sum())
    np.random.seed(9)
    got = Node2Vec(negative=4)._edge_rows(m, edges)
    after = np.random.random_sample()
    np.random.seed(9)
    keep = np.ones(rows.shape, bool)
    for e in range(len(rows)):
        for k in range(2):
            if p[rows[e, k]] < 1:
                keep[e, k] = p[rows[e, k]] >= np.random.random_sample()
    assert np.random.random_sample() == after and draws > 0
    expect = np.where(keep.all(1)[:, None], rows, -1)
    np.testing.assert_array_equal(got, expect)
    m0, _ = karate_model()
    np.testing.assert_array_equal(Node2Vec(negative=4)._edge_rows(m0, edges), rows)


@pytest.mark.parametrize("n,world", [(10, 3), (7, 8), (0, 2), (100, 1), (1001, 8)])
def test_shard_range_partitions(n, world):
    seen = []
    for r in range(world):
        lo, hi = shard_range(n, r, world)
        seen.extend(range(lo, hi))
    assert seen == list(range(n))
    w, s = shard_walks(np.arange(n * 2).reshape(n, 2), np.arange(n), world - 1, world)
    assert len(w) == len(s)


def test_graph_generators():
    from come_amd.graph import CSRGraph, chung_lu, sbm
    g = chung_lu(2000, 10, seed=1)
    assert g.V == 2000 and g.num_edges > 5000
    assert g.rowptr[-1] == 2 * g.num_edges and g.degree.max() > 5 * g.degree.mean()
    s = sbm(4, 100, 0.1, 0.001, seed=0)
    assert s.V == 400 and s.num_edges > 0
    ids, deg = s.degree_by_id()
    assert ids[0] == 1 and deg.sum() == 2 * s.num_edges
    g2, ids = CSRGraph.from_adjlist(os.path.join(GOLDEN, "..", "..", "tests", "golden",
                                                 "karate.adjlist")) \
        if os.path.exists(os.path.join(GOLDEN, "karate.adjlist")) else (None, None)
    if g2 is not None:
        assert g2.V == 34 and g2.num_edges == 78


def test_community_train_unknown_node_raises_keyerror():
    """community_embeddings.py:64 looks nodes up with model.vocab[x]: an unknown id raises."""
    from come_amd.community_embeddings import Community2Vec
    m, _ = karate_model()
    cm = Community2Vec.__new__(Community2Vec)
    cm.lr, cm.distributed, cm.group = 0.1, False, None
    with pytest.raises(KeyError):
        cm.train([1, 2, 999], m, 0.01)


@pytest.mark.parametrize("V,K,d", [(1000, 7, 5), (100, 3, 4), (256 * 3 + 17, 50, 9), (256, 2, 3)])
def test_gmm_split_k_sums_equal_float64_reference(V, K, d):
    """gmm.resp_t_x / resp_sum (the M-step's means numerator and nk as chunked sums added in
    float64, gmm.py) equal the float64 products within fp32 partial-sum error, for V not a
    multiple of the chunk count and V below it."""
    import torch
    from come_amd import gmm
    rng = np.random.RandomState(V + K)
    resp = torch.from_numpy(rng.dirichlet(np.ones(K), V).astype(np.float32))
    X = torch.from_numpy(rng.normal(size=(V, d)).astype(np.float32))
    ref_sx = resp.double().t() @ X.double()
    ref_nk = resp.double().sum(0)
    sx, nk = gmm.resp_t_x(resp, X), gmm.resp_sum(resp)
    assert sx.dtype == torch.float64 and nk.dtype == torch.float64
    np.testing.assert_allclose(sx.numpy(), ref_sx.numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(nk.numpy(), ref_nk.numpy(), rtol=1e-6, atol=1e-6)


def test_chung_lu_device_path_equals_numpy():
    """chung_lu(device=...) builds the graph with torch 1-D sort / unique / gathers
    (CSRGraph.from_device_pairs); on any device it must equal the numpy construction exactly.
    Run here on torch's CPU device (the GPU run of the same code: scripts/check_c5_inputs.py)."""
    import torch
    from come_amd.graph import chung_lu
    for V, deg in ((3000, 8.0), (40000, 20.0)):
        a = chung_lu(V, deg, seed=4)
        b = chung_lu(V, deg, seed=4, device=torch.device("cpu"))
        for n in ("edges", "col", "rowptr", "degree"):
            np.testing.assert_array_equal(getattr(a, n), getattr(b, n), err_msg=n)


@pytest.mark.parametrize("V,K,d", [(1_000_000, 50, 128), (1_000_000, 7, 128), (100_000, 50, 128),
                                   (1_000_000, 50, 64), (5000, 3, 64), (1000, 3, 128),
                                   (2_000_000, 200, 128), (999, 3, 96)])
def test_scatter_chunks_fill_whole_rounds(V, K, d):
    """gmm.scatter's default chunk count: the MFMA grid ((K / components per workgroup) x chunks,
    two workgroups per CU) makes at most 8 whole rounds of the 2 x 256 slots, the partials stay
    within 512 MB and no chunk is smaller than 64 rows."""
    from come_amd.gmm import scatter_chunks
    c = scatter_chunks(V, K, d, 256)
    assert 1 <= c <= max(1, -(-V // 64))
    assert c * K * d * d <= max(128 << 20, K * d * d)
    if d in (64, 128):
        groups = -(-K // (2 if d == 128 else 4))
        assert groups * c <= 8 * 512
        if V >= 64 * 8 * 512:  # rows enough for every slot: whole rounds, within one group
            assert (groups * c) % 512 > 512 - groups or (groups * c) % 512 == 0
    if (V, K, d) == (1_000_000, 50, 128):
        assert c == 163  # = the measured C4 grid (7.96 rounds, profiles/r05_ab_gmm_diag.txt)


def test_default_hot_share_by_row_width():
    """The contended-row share the product uses (training_sdg_inner.default_hot_share) is the
    one the library derives the bitmap with (come.h COME_DEFAULT_HOT_SHARE / _WIDE): 5e-6 up to
    d = 128, 8e-7 above (profiles/r06_hot_share.txt)."""
    import re
    import come_amd.training_sdg_inner as tsi
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(root, "include", "come.h")).read()
    narrow = float(re.search(r"#define COME_DEFAULT_HOT_SHARE\s+(\S+)", hdr).group(1))
    wide = float(re.search(r"#define COME_DEFAULT_HOT_SHARE_WIDE\s+(\S+)", hdr).group(1))
    assert [tsi.default_hot_share(d) for d in (2, 64, 128)] == [narrow] * 3 == [5e-6] * 3
    assert [tsi.default_hot_share(d) for d in (129, 256, 512)] == [wide] * 3 == [8e-7] * 3


@pytest.mark.parametrize("seed", [0, 1234, 2 ** 31 + 7])
def test_draw_seeds_is_numpy_stream(seed):
    """draw_seeds (native come_np_draw_seeds) == the reference's per-call seeding, pyx:427/477
    (2^24 * randint(0, 2^24) + randint(0, 2^24) from the GLOBAL numpy RNG, call after call): the
    same values and the global RNG left exactly where numpy's own draws leave it, across the
    624-word regeneration boundary and with a cached Gaussian pending."""
    def reference(n):
        out = np.empty(n, np.uint64)
        for i in range(n):  # the reference's per-call expression, pyx:477
            out[i] = (2 ** 24) * np.random.randint(0, 2 ** 24) + np.random.randint(0, 2 ** 24)
        return out
    for n in (0, 1, 311, 312, 313, 2000):
        np.random.seed(seed)
        np.random.random(5)
        np.random.standard_normal()  # leaves a cached Gaussian in the legacy state
        got, after = tsi.draw_seeds(n), np.random.random(4)
        gauss = np.random.standard_normal()
        np.random.seed(seed)
        np.random.random(5)
        np.random.standard_normal()
        want, after_ref = reference(n), np.random.random(4)
        assert np.array_equal(got, want), n
        assert np.array_equal(after, after_ref) and gauss == np.random.standard_normal(), n
