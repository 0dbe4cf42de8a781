"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  Tier A (clean cases): <= 1e-6 abs; cases whose dot products lie
within 1e-5 of a sigmoid-bucket edge (margin, in bucket units) may flip a bucket vs OpenBLAS'
summation order: tier B, <= 1e-3 abs."""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as orc

KAT_O2 = np.load(os.path.join(GOLDEN, "kat_o2.npz"))
KAT_O1 = np.load(os.path.join(GOLDEN, "kat_o1.npz"))


def tol_for(margin):
    return 1e-6 if margin >= 1e-4 else 1e-3


@pytest.mark.parametrize("name", list(KAT_O2["names"]))
@pytest.mark.parametrize("mode", [orc.DOT_REF, orc.DOT_WAVE64])
def test_o2_kat(name, mode):
    z, pre = KAT_O2, "o2_%s_" % name
    d, neg, w, V, L, P = [int(x) for x in z[pre + "params"]]
    lr, alpha = [float(x) for x in z[pre + "lr_alpha"]]
    node, ctx = z[pre + "node0"].copy(), z[pre + "ctx0"].copy()
    pairs = orc.sgns_o2(node, ctx, z[pre + "walks"], z[pre + "seeds"], w, neg, z[pre + "table"],
                        lr, alpha, dot_mode=mode)
    assert pairs > 0
    tol = tol_for(float(z[pre + "margin"]))
    np.testing.assert_allclose(node, z[pre + "node1"], rtol=0, atol=tol)
    np.testing.assert_allclose(ctx, z[pre + "ctx1"], rtol=0, atol=tol)
    # train_o2's return value: non-None entries per walk (pyx:483-490)
    np.testing.assert_array_equal((z[pre + "walks"] >= 0).sum(1), z[pre + "ret"])


def test_o2_kat_mostly_bit_exact():
    """The restatement reproduces the reference BIT FOR BIT on every clean case."""
    exact = 0
    for name in KAT_O2["names"]:
        pre = "o2_%s_" % name
        d, neg, w, V, L, P = [int(x) for x in KAT_O2[pre + "params"]]
        node, ctx = KAT_O2[pre + "node0"].copy(), KAT_O2[pre + "ctx0"].copy()
        orc.sgns_o2(node, ctx, KAT_O2[pre + "walks"], KAT_O2[pre + "seeds"], w, neg,
                    KAT_O2[pre + "table"], *[float(x) for x in KAT_O2[pre + "lr_alpha"]])
        exact += np.array_equal(node, KAT_O2[pre + "node1"]) and \
            np.array_equal(ctx, KAT_O2[pre + "ctx1"])
    assert exact >= len(KAT_O2["names"]) - 1


@pytest.mark.parametrize("name", list(KAT_O1["names"]))
def test_o1_kat(name):
    z, pre = KAT_O1, "o1_%s_" % name
    d, neg, V, E = [int(x) for x in z[pre + "params"]]
    node = z[pre + "node0"].copy()
    pairs = orc.sgns_o1(node, z[pre + "edges"], z[pre + "seeds"], neg, z[pre + "table"],
                        float(z[pre + "lr"][0]))
    assert pairs == 2 * E
    np.testing.assert_allclose(node, z[pre + "node1"], rtol=0,
                               atol=tol_for(float(z[pre + "margin"])))


def test_make_table_golden():
    z = np.load(os.path.join(GOLDEN, "make_table.npz"))
    for name in z["names"]:
        counts = z[name + "_counts"]
        ids = z[name + "_ids"]
        assert (ids == np.arange(1, len(ids) + 1)).all()
        t = orc.make_table(counts, int(z[name + "_T"]))
        if name + "_table" in z:
            np.testing.assert_array_equal(t, z[name + "_table"])
        else:
            assert hashlib.sha256(t.tobytes()).hexdigest() == str(z[name + "_sha256"])


def test_make_table_quirks():
    """model.py:112 starts at node id 1 (row 0 never drawn) and clamps at V-1."""
    t = orc.make_table(np.array([5, 1, 1, 1, 9]), 1000)
    assert t.min() >= 1 and t.max() <= 4
    assert (np.diff(t.astype(np.int64)) >= 0).all()
    assert np.bincount(t, minlength=5)[0] == 0


def test_exp_table_formula():
    e = orc.exp_table()
    assert e.dtype == np.float32 and e.shape == (1000,)
    assert (np.diff(e) >= 0).all()
    assert abs(float(e[500]) - 0.5) < 1e-6
    # pyx:533 stores e/(e+1) of a float-rounded exp
    i = np.arange(1000)
    ex = np.exp(((i.astype(np.float32) / np.float32(1000)).astype(np.float64) * 2.0 - 1.0) * 6.0)
    ex = ex.astype(np.float32).astype(np.float64)
    np.testing.assert_array_equal(e, (ex / (ex + 1.0)).astype(np.float32))


def test_lcg_matches_reference_constants():
    s = 12345
    for _ in range(10):
        s2 = orc.lcg_next(s)
        assert s2 == (s * 25214903917 + 11) & ((1 << 48) - 1)
        s = s2


def test_community_golden():
    z = np.load(os.path.join(GOLDEN, "community.npz"))
    for name in z["names"]:
        p = name + "_"
        beta, lr = [float(x) for x in z[p + "scal"]]
        x1 = orc.community_train(z[p + "x0"], z[p + "pi"], z[p + "mu"], z[p + "inv"], beta, lr,
                                 int(z[p + "iters"]), chunksize=37)
        np.testing.assert_array_equal(x1, z[p + "x1"])


def test_gmm_resp_golden():
    z = np.load(os.path.join(GOLDEN, "gmm_resp.npz"))
    for name in z["names"]:
        p = name + "_"
        pi = orc.gmm_predict_proba(z[p + "X"], z[p + "w"], z[p + "mu"], z[p + "cov"])
        np.testing.assert_allclose(pi.astype(np.float32), z[p + "pi"], rtol=0, atol=1e-6)
        np.testing.assert_array_equal(np.linalg.inv(z[p + "cov"].astype(np.float32)),
                                      z[p + "inv32"])


def test_karate_flow_oracle():
    """adsc_Karate.py:104-137 (workers=1) replayed with the oracle: tier B."""
    z = np.load(os.path.join(GOLDEN, "karate.npz"))
    size, neg, ws, lr, alpha, beta, T = z["hyper"]
    neg, ws, T = int(neg), int(ws), int(T)
    table = orc.make_table(z["degree_counts"], T)
    np.testing.assert_array_equal(np.bincount(table, minlength=34), z["table_bincount"])
    node = z["node_init"].copy()
    ctx = np.zeros_like(node)
    edges = z["edges"] - 1
    walks = (z["walks"] - 1).astype(np.int32)

    def seeds(s, n):
        np.random.seed(s)
        ab = np.random.randint(0, 2 ** 24, size=2 * n).astype(np.uint64)
        return (ab[0::2] << np.uint64(24)) + ab[1::2]

    orc.sgns_o1(node, edges, seeds(100, len(edges)), neg, table, float(lr))
    np.testing.assert_allclose(node, z["after_o1_pre"], atol=1e-3)
    orc.sgns_o2(node, ctx, walks, seeds(101, len(walks)), ws, neg, table, float(lr), float(alpha))
    np.testing.assert_allclose(node, z["after_o2_pre_node"], atol=1e-3)
    np.testing.assert_allclose(ctx, z["after_o2_pre_ctx"], atol=1e-3)
    orc.sgns_o1(node, edges, seeds(102, len(edges)), neg, table, float(lr))
    orc.sgns_o2(node, ctx, walks, seeds(103, len(walks)), ws, neg, table, float(lr), float(alpha))
    np.testing.assert_allclose(node, z["after_loop_node"], atol=1e-3)
    np.testing.assert_allclose(ctx, z["after_loop_ctx"], atol=1e-3)
    x = orc.community_train(z["after_loop_node"], z["gmm_pi"], z["gmm_centroid"], z["gmm_inv"],
                            float(beta), float(lr), 5, chunksize=20)
    np.testing.assert_allclose(x, z["after_com_node"], atol=1e-6)


# ---- the Hogwild CPU restatement (oracle/come_oracle_mt.c; bench.py's cpu_baseline) ----------

@pytest.mark.parametrize("name", list(KAT_O2["names"]))
def test_o2_hogwild_restatement_one_thread_matches_golden(name):
    """One worker thread = walks in order (workers=1): the reference's own output, up to the
    8-wide dot product's summation order (tier B)."""
    z, pre = KAT_O2, "o2_%s_" % name
    d, neg, w, V, L, P = [int(x) for x in z[pre + "params"]]
    lr, alpha = [float(x) for x in z[pre + "lr_alpha"]]
    node, ctx = z[pre + "node0"].copy(), z[pre + "ctx0"].copy()
    pairs, done = orc.sgns_o2_hogwild(node, ctx, z[pre + "walks"], z[pre + "seeds"], w, neg,
                                      z[pre + "table"], lr, alpha, threads=1)
    assert done == P and pairs == orc.sgns_o2(node.copy(), ctx.copy(), z[pre + "walks"],
                                              z[pre + "seeds"], w, neg, z[pre + "table"], lr,
                                              alpha)
    np.testing.assert_allclose(node, z[pre + "node1"], rtol=0, atol=1e-3)
    np.testing.assert_allclose(ctx, z[pre + "ctx1"], rtol=0, atol=1e-3)


@pytest.mark.parametrize("name", list(KAT_O1["names"]))
def test_o1_hogwild_restatement_one_thread_matches_golden(name):
    z, pre = KAT_O1, "o1_%s_" % name
    d, neg, V, E = [int(x) for x in z[pre + "params"]]
    node = z[pre + "node0"].copy()
    pairs, done = orc.sgns_o1_hogwild(node, z[pre + "edges"], z[pre + "seeds"], neg,
                                      z[pre + "table"], float(z[pre + "lr"][0]), threads=1)
    assert pairs == 2 * E and done == E
    np.testing.assert_allclose(node, z[pre + "node1"], rtol=0, atol=1e-3)


def test_o2_hogwild_restatement_threads_disjoint_rows_exact():
    """Walks that share no row cannot race when they draw no negatives (n = 0), so 8 threads give
    exactly the 1-thread result."""
    rng = np.random.RandomState(3)
    V, d, P, L = 4000, 64, 64, 20
    walks = np.arange(P * L, dtype=np.int32).reshape(P, L)  # every row distinct
    table = np.arange(P * L, V, dtype=np.uint32)            # negatives outside the walks
    seeds = rng.randint(0, 2 ** 48, P).astype(np.uint64)
    node0 = rng.uniform(-1, 1, (V, d)).astype(np.float32)
    outs = []
    for thr in (1, 8):
        node, ctx = node0.copy(), np.zeros_like(node0)
        pairs, done = orc.sgns_o2_hogwild(node, ctx, walks, seeds, 3, 0, table, 0.1, 1.0, thr)
        assert done == P
        outs.append((node, ctx))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])


def test_o2_hogwild_restatement_deadline_and_threads():
    """max_seconds stops the claiming early; every walk is processed once otherwise."""
    rng = np.random.RandomState(4)
    V, d, P, L = 2000, 32, 400, 30
    walks = rng.randint(0, V, (P, L)).astype(np.int32)
    seeds = rng.randint(0, 2 ** 48, P).astype(np.uint64)
    table = orc.make_table(rng.randint(1, 20, V), 10000)
    node, ctx = rng.uniform(-1, 1, (V, d)).astype(np.float32), np.zeros((V, d), np.float32)
    pairs, done = orc.sgns_o2_hogwild(node, ctx, walks, seeds, 5, 5, table, 0.05, 1.0, 4)
    assert done == P and pairs == P * (2 * 5 * L - 5 * 6)
    assert np.isfinite(node).all() and np.isfinite(ctx).all()
    assert orc.usable_cpus() >= 1
