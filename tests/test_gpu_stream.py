"""Deterministic coverage of the product's Hogwild O2 kernel (k_sgns_o2_stream) including its
negative-row path (pyx:128-149): repeated negatives within a pair (a later draw sees the updated
row, pyx:147), negatives repeated across consecutive pairs (prefetched copies of a row the current
pair writes), negatives equal to later positives of the same walk (the held cold positive and its
prefetched copy), draws equal to the positive (skipped, pyx:135), non-temporal negative loads.

Bars:
  * one wavefront (max_waves=1), no contended rows: walks run in order, so the launch must equal
    the sequential oracle (WAVE64 dot order) BIT FOR BIT even when every row is shared;
  * 256 walks in flight that share no row -- walk rows, positives and every negative draw are
    private to a walk (seeds chosen so no two walks draw the same table slot, slots mapped to the
    walk's own rows and a private pool) -- BIT FOR BIT as well;
  * contended rows (float-atomic deltas instead of fma write-backs) on one wavefront: tier B,
    <= 1e-3 abs, most elements within 1e-5;
  * the library-derived contended-row bitmap (hot="auto" / hot_rows == NULL, plain and packed
    table) equals the explicit come_hot_rows bitmap at DEFAULT_HOT_P.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

import come_amd.training_sdg_inner as tsi

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
LCG_MUL, LCG_ADD, MASK48 = np.uint64(25214903917), np.uint64(11), np.uint64((1 << 48) - 1)


def dev(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).to(DEV)


def lcg_slots(seeds, count, T):
    """Table slots of `count` consecutive draws from each seed (pyx:133-134, Appendix A2/A4)."""
    nr = np.asarray(seeds, np.uint64).copy()
    out = np.empty((len(nr), count), np.int64)
    with np.errstate(over="ignore"):
        for k in range(count):
            out[:, k] = ((nr >> np.uint64(16)) % np.uint64(T)).astype(np.int64)
            nr = (nr * LCG_MUL + LCG_ADD) & MASK48
    return out


def run(node0, ctx0, walks, seeds, w, n, table, lr, mode, hot, opts=None):
    node, ctx = dev(node0), dev(ctx0)
    tsi.sgns_o2(node, ctx, dev(walks), dev(seeds), w, n, table, lr, 1.0, mode, opts=opts,
                hot=hot)
    torch.cuda.synchronize()
    return node.cpu().numpy(), ctx.cpu().numpy()


def oracle(node0, ctx0, walks, seeds, w, n, table, lr):
    n_ref, c_ref = node0.copy(), ctx0.copy()
    orc.sgns_o2(n_ref, c_ref, walks, seeds, w, n, table, lr, 1.0, dot_mode=orc.DOT_WAVE64)
    return n_ref, c_ref


@pytest.mark.parametrize("d,n", [(128, 5), (128, 10), (256, 10), (64, 20)])
@pytest.mark.parametrize("kernel", [3, 1])  # streaming (the product's), direct
def test_one_wavefront_bit_exact_with_shared_rows(d, n, kernel):
    """60 rows, 12 walks of 40, w = 5: negatives repeat inside pairs, across consecutive pairs
    and hit positives of the same walk all the time."""
    rng = np.random.RandomState(d + n + kernel)
    V, P, L, w = 60, 12, 40, 5
    table = orc.make_table(rng.randint(1, 40, V), 997)
    node0 = rng.uniform(-1, 1, (V, d)).astype(np.float32)
    ctx0 = rng.uniform(-0.3, 0.3, (V, d)).astype(np.float32)
    walks = rng.randint(0, V, (P, L)).astype(np.int32)
    walks[3, 30:] = -1
    seeds = rng.randint(0, 2 ** 48, P, dtype=np.int64).astype(np.uint64)
    got = run(node0, ctx0, walks, seeds, w, n, dev(table), 0.05, tsi.MODE_HOGWILD, None,
              opts={"o2_kernel": kernel, "max_waves": 1})
    ref = oracle(node0, ctx0, walks, seeds, w, n, table, 0.05)
    np.testing.assert_array_equal(got[0], ref[0])
    np.testing.assert_array_equal(got[1], ref[1])


def disjoint_case(P, L, w, n, d, pool, T, seed):
    """P walks whose rows, positives and negative draws are private: walk p owns rows
    [p B, (p + 1) B), B = L + pool; its walk positions repeat rows of the first L/2 of them; its
    draws hit slots no other walk draws (seeds re-drawn until so), mapped to its own walk rows or
    its pool (so a draw can equal the current positive, a later positive, or repeat)."""
    rng = np.random.RandomState(seed)
    B = L + pool
    V = P * B
    walks = (np.arange(P)[:, None] * B + rng.randint(0, L // 2, (P, L))).astype(np.int32)
    draws = tsi.count_o2_pairs(walks[:1], w) * n
    seeds = rng.randint(0, 2 ** 48, P, dtype=np.int64).astype(np.uint64)
    slots = lcg_slots(seeds, draws, T)
    owner = np.full(T, -1, np.int64)
    for p in range(P):
        for _ in range(200):
            s = np.unique(slots[p])
            if (owner[s] < 0).all():
                owner[s] = p
                break
            seeds[p] = np.uint64(rng.randint(0, 2 ** 48, dtype=np.int64))
            slots[p] = lcg_slots(seeds[p:p + 1], draws, T)[0]
        else:
            raise AssertionError("could not place walk %d" % p)
    table = np.zeros(T, np.uint32)
    for p in range(P):
        cand = np.concatenate([np.unique(walks[p]), p * B + L + np.arange(pool)])
        table[slots[p]] = rng.choice(cand, draws)
    node0 = rng.uniform(-1, 1, (V, d)).astype(np.float32)
    ctx0 = rng.uniform(-0.3, 0.3, (V, d)).astype(np.float32)
    return node0, ctx0, walks, seeds, table


@pytest.mark.parametrize("d,n", [(128, 5), (128, 10), (256, 5), (256, 10)])
def test_disjoint_walks_in_flight_bit_exact(d, n):
    """256 walks in flight (forced streaming kernel, no contended rows), each with repeated
    negatives from a private pool of 6 rows: equal to the sequential oracle bit for bit."""
    P, L, w = 256, 12, 2
    node0, ctx0, walks, seeds, table = disjoint_case(P, L, w, n, d, pool=6, T=(1 << 26) - 5,
                                                     seed=d * 10 + n)
    got = run(node0, ctx0, walks, seeds, w, n, dev(table), 0.05, tsi.MODE_HOGWILD, None,
              opts={"o2_kernel": 3})
    ref = oracle(node0, ctx0, walks, seeds, w, n, table, 0.05)
    assert not np.array_equal(ref[1], ctx0)  # negatives moved rows
    np.testing.assert_array_equal(got[0], ref[0])
    np.testing.assert_array_equal(got[1], ref[1])


@pytest.mark.parametrize("hot_kind", ["all", "table_share"])
def test_one_wavefront_contended_rows_tier_b(hot_kind):
    """Hot rows are updated by float-atomic deltas (row + g*in, rounded twice, instead of fma):
    one wavefront against the sequential oracle within tier B."""
    rng = np.random.RandomState(5)
    V, P, L, w, n, d = 80, 10, 30, 5, 5, 128
    table = orc.make_table(rng.randint(1, 200, V), 20011)
    node0 = rng.uniform(-1, 1, (V, d)).astype(np.float32)
    ctx0 = rng.uniform(-0.3, 0.3, (V, d)).astype(np.float32)
    walks = rng.randint(0, V, (P, L)).astype(np.int32)
    seeds = rng.randint(0, 2 ** 48, P, dtype=np.int64).astype(np.uint64)
    if hot_kind == "all":
        hot = torch.full(((V + 31) // 32,), -1, dtype=torch.int32, device=DEV)
    else:
        hot = tsi.hot_rows(dev(table), V, int(0.015 * len(table)))
        nh = int(np.unpackbits(hot.cpu().numpy().view(np.uint8)).sum())
        assert 0 < nh < V
    got = run(node0, ctx0, walks, seeds, w, n, dev(table), 0.05, tsi.MODE_HOGWILD, hot,
              opts={"o2_kernel": 3, "max_waves": 1})
    ref = oracle(node0, ctx0, walks, seeds, w, n, table, 0.05)
    for a, b in zip(got, ref):
        diff = np.abs(a - b)
        assert diff.max() <= 1e-3, diff.max()                    # tier B
        assert np.mean(diff <= 1e-5) > 0.95, np.mean(diff <= 1e-5)


@pytest.mark.parametrize("d", [128, 256])
def test_derived_hot_bitmap_matches_explicit(d):
    """hot="auto" (the C-ABI's hot_rows == NULL: libcome derives the bitmap, plain or packed
    table) trains exactly like the explicit come_hot_rows bitmap at default_hot_share(d) (5e-6 up
    to d = 128, 8e-7 above), and differs from hot=None (COME_HOT_NONE) -- disjoint walks, so every
    run is deterministic."""
    rng = np.random.RandomState(9)
    V, L, w, n, T = 1 << 19, 16, 3, 0, 10_000_000  # share 5e-6 = 50 slots: hubs hot
    counts = rng.zipf(1.6, V).clip(1, 10 ** 6)
    table = orc.make_table(counts, T)
    node0 = rng.uniform(-1, 1, (V, d)).astype(np.float32)
    ctx0 = rng.uniform(-0.3, 0.3, (V, d)).astype(np.float32)
    walks = rng.permutation(V).reshape(V // L, L).astype(np.int32)
    seeds = rng.randint(0, 2 ** 48, V // L, dtype=np.int64).astype(np.uint64)
    tab = dev(table)
    packed = tsi.pack_table(tab)
    explicit = tsi.hot_rows(tab, V, max(1, int(tsi.default_hot_share(d) * T)))
    nh = int(np.unpackbits(explicit.cpu().numpy().view(np.uint8)).sum())
    assert 10 < nh < V // 2, nh
    opts = {"o2_kernel": 3}
    ref = run(node0, ctx0, walks, seeds, w, n, tab, 0.1, tsi.MODE_HOGWILD, explicit, opts)
    for t in (tab, packed):
        got = run(node0, ctx0, walks, seeds, w, n, t, 0.1, tsi.MODE_HOGWILD, "auto", opts)
        np.testing.assert_array_equal(got[0], ref[0])
        np.testing.assert_array_equal(got[1], ref[1])
    cold = run(node0, ctx0, walks, seeds, w, n, tab, 0.1, tsi.MODE_HOGWILD, None, opts)
    assert not np.array_equal(cold[1], ref[1])


def test_hot_bitmap_validation():
    node = torch.zeros((100, 64), dtype=torch.float32, device=DEV)
    walks = torch.zeros((1, 4), dtype=torch.int32, device=DEV)
    seeds = torch.zeros(1, dtype=torch.int64, device=DEV)
    tab = torch.zeros(10, dtype=torch.int32, device=DEV)
    with pytest.raises(ValueError):
        tsi.sgns_o2(node, node.clone(), walks, seeds, 2, 1, tab, 0.1, 1.0, tsi.MODE_HOGWILD,
                    hot=torch.zeros(3, dtype=torch.int32, device=DEV))  # needs 4 words
    with pytest.raises(TypeError):
        tsi.sgns_o2(node, node.clone(), walks, seeds, 2, 1, tab, 0.1, 1.0, tsi.MODE_HOGWILD,
                    hot=torch.zeros(4, dtype=torch.int64, device=DEV))
