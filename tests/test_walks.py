"""Walk producer and text formats -- CPU tests.

* graph build order, corpus walks, walk files: the native path (come_amd.graph_utils over
  libcome.so) against tests/golden/walks.npz, produced by the reference's own graph_utils
  (make_golden_walks.py), bit for bit;
* the oracle's pure-Python restatement pinned against the same fixture;
* native vs oracle on random graphs (restart, self-loops, duplicates, sparse ids);
* the restated CPython random stream (seed, random(), _randbelow) against CPython itself;
* save_embedding byte-for-byte against the reference's str(np.float32) formatting.
"""
import ctypes
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN
from come_amd import _lib, graph_utils as gu, io_utils
from oracle import oracle as orc

W = np.load(os.path.join(GOLDEN, "walks.npz"))


def pad(walks, L):
    a = np.full((len(walks), L), -1, np.int64)
    for i, w in enumerate(walks):
        a[i, :len(w)] = w
    return a


@pytest.mark.parametrize("case", ["karate", "messy"])
def test_graph_order_matches_reference(case):
    G = gu.Graph.from_edges(W[case + "_edges_in"])
    assert np.array_equal(G.node_ids, W[case + "_nodes"])
    assert np.array_equal(G.edges(), W[case + "_edges"])
    assert np.array_equal(G.degree_arr, W[case + "_degree"])
    assert G.number_of_edges() == len(W[case + "_edges"])
    adj = orc.nx_graph(W[case + "_edges_in"])
    for n in list(adj)[:20]:
        assert G.neighbors(n) == list(adj[n])


@pytest.mark.parametrize("case,paths,L,alpha,seed", [
    ("karate", 10, 20, 0.0, 9999999999), ("karate_a03", 2, 15, 0.3, 4242),
    ("messy", 3, 25, 0.1, 7)])
def test_corpus_matches_reference(case, paths, L, alpha, seed):
    g = "messy" if case == "messy" else "karate"
    G = gu.Graph.from_edges(W[g + "_edges_in"])
    adj = orc.nx_graph(W[g + "_edges_in"])
    if g == "karate":  # load_adjacencylist(path, True): to_undirected() reorders adjacencies
        G, adj = G.to_undirected(), orc.nx_to_undirected(adj)
    rnd = random.Random(seed)
    walks = gu.build_deepwalk_corpus(G, paths, L, alpha=alpha, rand=rnd)
    assert np.array_equal(walks, W[case + "_walks"])
    # the caller's Random continues exactly where the reference leaves it
    assert np.array_equal(np.array(rnd.getstate()[1], np.uint32), W[case + "_state"])
    # oracle pinned on the same fixture
    rnd2 = random.Random(seed)
    ow = orc.deepwalk_corpus(adj, paths, L, alpha, rnd2)
    assert np.array_equal(pad(ow, L), W[case + "_walks"])


@pytest.mark.parametrize("workers", [1, 4])
def test_walk_files_match_reference(tmp_path, workers):
    G = gu.Graph.from_edges(W["karate_edges_in"]).to_undirected()
    files = gu.write_walks_to_disk(G, str(tmp_path / "karate.walks"), num_paths=10,
                                   path_length=20, alpha=0, rand=random.Random(9999999999),
                                   num_workers=workers)
    assert [gu.count_lines(f) for f in files] == list(W["karate_files_w%d_count" % workers])
    assert np.array_equal(gu.read_walk_files(files), W["karate_files_w%d" % workers])
    it = list(gu.combine_files_iter(files))
    assert np.array_equal(pad(it, 20), W["karate_files_w%d" % workers])
    c = gu.count_textfiles(files)
    ids, n = np.unique(W["karate_files_w%d" % workers], return_counts=True)
    assert c == dict(zip(ids.tolist(), n.tolist()))


def test_load_adjacencylist(tmp_path):
    e = W["messy_edges_in"]
    f = tmp_path / "g.adjlist"
    with open(f, "w") as fh:
        fh.write("# comment line\n")
        for i, (u, v) in enumerate(e):
            fh.write("%d %d\n" % (u, v) if i % 3 else "%d\t%d\r\n" % (u, v))
    G = gu.load_adjacencylist(str(f), False)
    assert np.array_equal(G.node_ids, W["messy_nodes"])
    assert np.array_equal(G.edges(), W["messy_edges"])
    Gu = gu.load_adjacencylist(str(f), True)
    und = orc.nx_to_undirected(orc.nx_graph(e))
    assert np.array_equal(Gu.edges(), W["messy_edges"])
    for n in und:
        assert Gu.neighbors(n) == list(und[n])
    with open(f, "a") as fh:
        fh.write("1 2 3\n")
    with pytest.raises(ValueError):
        gu.load_adjacencylist(str(f))
    with open(f, "a") as fh:
        fh.write("1 x\n")
    with pytest.raises(_lib.ComeError):
        gu.load_adjacencylist(str(f))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_native_walker_vs_oracle_random_graphs(seed):
    rng = np.random.RandomState(seed)
    n = rng.randint(5, 200)
    ids = rng.choice(np.arange(1, 10 ** 6), n, replace=False)
    e = ids[rng.randint(0, n, (rng.randint(n, 4 * n), 2))]
    m = rng.rand(len(e)) < 0.05
    e[m, 1] = e[m, 0]  # self-loops
    G = gu.Graph.from_edges(e)
    adj = orc.nx_graph(e)
    if seed == 1:
        G, adj = G.to_undirected(), orc.nx_to_undirected(adj)
    assert G.node_ids.tolist() == list(adj)
    assert G.edges().tolist() == [list(x) for x in orc.nx_edges(adj)]
    assert G.degree_arr.tolist() == orc.nx_degree(adj)
    alpha = [0.0, 0.25, 1.0][seed]
    L = rng.randint(1, 40)
    r1, r2 = random.Random(seed * 31 + 5), random.Random(seed * 31 + 5)
    walks = gu.build_deepwalk_corpus(G, 2, L, alpha=alpha, rand=r1)
    ow = orc.deepwalk_corpus(adj, 2, L, alpha, r2)
    assert np.array_equal(walks, pad(ow, L))
    assert r1.getstate() == r2.getstate()


def test_emit_rows_and_multi_stream_threads():
    G = gu.Graph.from_edges(W["messy_edges_in"])
    emit = np.argsort(np.argsort(G.node_ids)).astype(np.int32)  # Vocab.index = rank of the id
    rs = [random.Random(s) for s in (1, 2, 3)]
    rs2 = [random.Random(s) for s in (1, 2, 3)]
    a = gu._corpus(G, [1, 2, 1], 12, 0.2, rs, threads=3, emit=emit)
    b = gu._corpus(G, [1, 2, 1], 12, 0.2, rs2, threads=1)
    bb = np.where(b >= 0, emit[np.maximum(b, 0)], -1)
    assert np.array_equal(a, bb)
    assert [r.getstate() for r in rs] == [r.getstate() for r in rs2]


def test_pyrandom_restatement_matches_cpython():
    L = _lib.lib()
    st = np.zeros(625, np.uint32)
    for seed in (0, 1, 9999999999, 2 ** 31, 2 ** 64 - 1):
        assert L.come_pyrandom_seed(seed, _lib.ptr(st)) == 0
        assert st.tolist() == list(random.Random(seed).getstate()[1])
    r = random.Random(123)
    st = np.array(r.getstate()[1], np.uint32)
    out = np.zeros(500)
    assert L.come_pyrandom_draw(_lib.ptr(st), 0, 0, 500, _lib.ptr(out)) == 0
    assert out.tolist() == [r.random() for _ in range(500)]
    for n in (1, 2, 3, 5, 64, 1000, 2 ** 31 + 1, 2 ** 32):
        assert L.come_pyrandom_draw(_lib.ptr(st), 1, n, 500, _lib.ptr(out)) == 0
        assert out.tolist() == [float(r._randbelow(n)) for _ in range(500)]
    assert st.tolist() == list(r.getstate()[1])


def test_float32_text_matches_numpy_str():
    L = _lib.lib()
    rng = np.random.RandomState(5)
    xs = np.concatenate([rng.randint(0, 2 ** 32, 20000, dtype=np.uint64).astype(np.uint32)
                         .view(np.float32),
                         np.float32([0, -0.0, 1, 1e-4, 1e16, 0.1, -2.5, np.inf, -np.inf, np.nan,
                                     3.4e38, 1e-45, 123456789, 1e-5])]).astype(np.float32)
    buf = ctypes.create_string_buffer(48)
    for x in xs:
        L.come_format_f32(float(x), buf)
        assert buf.value.decode() == str(np.float32(x)), x


def test_save_embedding_matches_reference_format(tmp_path):
    rng = np.random.RandomState(3)
    emb = (rng.randn(50, 7) * 10.0 ** rng.randint(-6, 6, (50, 7))).astype(np.float32)
    io_utils.save_embedding(emb, "sub/emb", path=str(tmp_path))
    got = open(tmp_path / "sub" / "emb.txt").read()
    # IO_utils.py:58-62 verbatim semantics
    want = "".join(str(i + 1) + "\t" + " ".join(str(v) for v in row) + "\n"
                   for i, row in enumerate(emb))
    assert got == want
    back = io_utils.load_embedding("sub/emb", path=str(tmp_path))
    assert np.array_equal(back, emb)
