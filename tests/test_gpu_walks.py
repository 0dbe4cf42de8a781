"""HIP walker (come_random_walks) on the GPU: every step is an edge of the graph or a restart to
the walk's start (graph_utils.py:36-45), walks do not depend on how they are split over launches,
and the step distribution is the reference walker's (uniform neighbour, restart with probability
alpha) -- a statistical parity test, since the device stream is Philox, not CPython's MT19937
(the exact stream is the host path, tests/test_walks.py)."""
import numpy as np
import pytest

from come_amd import graph_utils as gu
from come_amd.graph import chung_lu

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def csr(g, d):
    return (torch.from_numpy(g.rowptr).to(d), torch.from_numpy(g.col.astype(np.int32)).to(d))


@pytest.mark.parametrize("alpha", [0.0, 0.3])
def test_steps_are_edges_or_restarts(alpha):
    d = dev()
    g = chung_lu(3000, 8.0, seed=3)
    rowptr, col = csr(g, d)
    starts = torch.randperm(g.V, device=d).int()
    w = gu.device_walks(rowptr, col, starts, 40, alpha=alpha, seed=11).cpu().numpy()
    assert w.shape == (g.V, 40)
    assert np.array_equal(w[:, 0], starts.cpu().numpy())
    edges = set(map(tuple, np.stack([np.repeat(np.arange(g.V), np.diff(g.rowptr)), g.col], 1)
                    .tolist()))
    deg = np.diff(g.rowptr)
    for r in range(0, g.V, 7):
        row = w[r]
        n = int((row >= 0).sum())
        assert (row[n:] == -1).all()
        if n < 40:  # stopped early: only at a node without neighbours
            assert deg[row[n - 1]] == 0
        for t in range(1, n):
            a, b = int(row[t - 1]), int(row[t])
            assert (a, b) in edges or (alpha > 0 and b == row[0]), (r, t, a, b)


def test_launch_shape_independent_and_emit():
    d = dev()
    g = chung_lu(5000, 6.0, seed=4)
    rowptr, col = csr(g, d)
    starts = torch.randint(0, g.V, (10000,), device=d, dtype=torch.int32)
    full = gu.device_walks(rowptr, col, starts, 25, alpha=0.1, seed=99)
    a = gu.device_walks(rowptr, col, starts[:3333].contiguous(), 25, alpha=0.1, seed=99)
    b = gu.device_walks(rowptr, col, starts[3333:].contiguous(), 25, alpha=0.1, seed=99,
                        walk_offset=3333)
    assert torch.equal(full, torch.cat([a, b]))
    other = gu.device_walks(rowptr, col, starts, 25, alpha=0.1, seed=100)
    assert not torch.equal(full, other)
    emit = (torch.arange(g.V, device=d, dtype=torch.int32) * 3 + 1).contiguous()
    e = gu.device_walks(rowptr, col, starts, 25, alpha=0.1, seed=99, emit=emit)
    assert torch.equal(e, torch.where(full >= 0, full * 3 + 1, full))


def test_neighbour_choice_uniform_and_restart_rate():
    """Chi-square of first-step choices at a hub (uniform over its neighbours) and the restart
    rate out of a leaf (alpha)."""
    d = dev()
    hub_deg = 12
    edges = [(0, i) for i in range(1, hub_deg + 1)] + [(1, 2)]
    G = gu.Graph.from_edges(np.array(edges) + 1)  # ids 1.., positions in first-appearance order
    rowptr, col = (torch.from_numpy(G.rowptr).to(d), torch.from_numpy(G.col).to(d))
    P = 1 << 20
    starts = torch.zeros(P, dtype=torch.int32, device=d)
    w = gu.device_walks(rowptr, col, starts, 2, alpha=0.0, seed=5).cpu().numpy()
    counts = np.bincount(w[:, 1], minlength=hub_deg + 1)[1:]
    exp = P / hub_deg
    chi2 = ((counts - exp) ** 2 / exp).sum()
    assert chi2 < 40.0, (chi2, counts)  # 11 dof: p ~ 1e-4
    leaf = 5  # position 5 = node id 6, only neighbour: the hub
    starts = torch.full((P,), leaf, dtype=torch.int32, device=d)
    w = gu.device_walks(rowptr, col, starts, 2, alpha=0.3, seed=6).cpu().numpy()
    rate = (w[:, 1] == leaf).mean()
    assert abs(rate - 0.3) < 5 * np.sqrt(0.3 * 0.7 / P), rate
    assert set(np.unique(w[:, 1])) <= {0, leaf}


def test_matches_reference_walker_distribution():
    """Transition frequencies of device walks vs the exact reference walker on Karate (host,
    CPython stream), both from every node: total-variation distance per source node small."""
    import os
    import random
    from conftest import GOLDEN
    W = np.load(os.path.join(GOLDEN, "walks.npz"))
    G = gu.Graph.from_edges(W["karate_edges_in"]).to_undirected()
    d = dev()
    V = G.number_of_nodes()
    ref = gu._corpus(G, [400], 20, 0.2, [random.Random(1)])
    starts = torch.arange(V, device=d, dtype=torch.int32).repeat(400)
    rowptr, col = (torch.from_numpy(G.rowptr).to(d), torch.from_numpy(G.col).to(d))
    gw = gu.device_walks(rowptr, col, starts, 20, alpha=0.2, seed=3).cpu().numpy()

    def trans(w):
        m = np.zeros((V, V + 1))
        a, b = w[:, :-1].ravel(), w[:, 1:].ravel()
        restart = b == np.repeat(w[:, :1], w.shape[1] - 1, 1).ravel()
        np.add.at(m, (a[~restart], b[~restart]), 1)
        np.add.at(m, (a[restart], np.full(restart.sum(), V)), 1)
        return m / m.sum(1, keepdims=True)
    tv = 0.5 * np.abs(trans(ref) - trans(gw)).sum(1)
    assert tv.max() < 0.05, tv


@pytest.mark.parametrize("P,L", [(1, 1), (255, 17), (257, 80), (10000, 33), (3000, 16)])
def test_staged_output_matches_direct_stores(P, L):
    """k_random_walks_staged (LDS-staged, coalesced row segments) vs k_random_walks (one store
    per lane per step): the same Philox counters, so the walks must be identical -- including
    invalid starts, dead ends (a node without neighbours), emit and ragged P / L."""
    from come_amd import _lib
    d = dev()
    g = chung_lu(2000, 5.0, seed=P + L)
    rowptr = np.concatenate([g.rowptr, [g.rowptr[-1]] * 3])  # 3 isolated nodes at the end
    V = len(rowptr) - 1
    rowptr_t = torch.from_numpy(rowptr).to(d)
    col = torch.from_numpy(g.col.astype(np.int32)).to(d)
    rng = np.random.RandomState(P)
    s = rng.randint(0, V, P).astype(np.int32)
    s[::7] = V - 1 - (np.arange(len(s[::7])) % 3)  # isolated: walk ends after one step
    s[::11] = -1  # not a node: an empty walk
    starts = torch.from_numpy(s).to(d)
    emit = (torch.arange(V, device=d, dtype=torch.int32) * 5 + 2).contiguous()
    try:
        for kw in ({}, {"emit": emit}):
            out = []
            for opt in (0, 1, 2, 3):  # direct, then 16-, 8- and 32-step LDS slices
                _lib.set_option("walk_staged", opt)
                out.append(gu.device_walks(rowptr_t, col, starts, L, alpha=0.15, seed=7,
                                           walk_offset=5, **kw))
            for o in out[1:]:
                assert torch.equal(out[0], o), (P, L, kw.keys())
            w = out[1].cpu().numpy()
            assert (w[::11] == -1).all()
    finally:
        _lib.set_option("walk_staged", 1)  # the default


@pytest.mark.parametrize("alpha,L,offset", [(0.0, 80, 0), (0.15, 33, 5_000_000_123), (1.0, 7, 5)])
def test_device_walker_bit_exact_vs_cpu_restatement(alpha, L, offset):
    """come_random_walks (k_random_walks_staged) against its CPU restatement
    (oracle/come_oracle_walks.c: the same Philox-4x32-10 counters, restart and neighbour picks):
    identical walks, incl. dead ends (isolated nodes), invalid starts, the restart path, a walk
    offset beyond 2^32 (the counter's high word) and the emit map."""
    import torch
    from come_amd.graph import chung_lu
    from come_amd.graph_utils import device_walks
    from oracle import oracle as orc
    g = chung_lu(50_000, 6.0, gamma=2.5, seed=9)
    rng = np.random.RandomState(int(alpha * 100) + L)
    starts = rng.randint(-3, g.V + 3, 20_000).astype(np.int32)
    emit = rng.permutation(g.V).astype(np.int32)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.as_tensor(a, device=dev)  # noqa: E731
    for em in (None, emit):
        got = device_walks(t(g.rowptr), t(g.col), t(starts), L, alpha=alpha, seed=2 ** 40 + 77,
                           walk_offset=offset, emit=None if em is None else t(em)).cpu().numpy()
        ref = orc.philox_walks(g.rowptr, g.col, starts, L, alpha, seed=2 ** 40 + 77,
                               walk_offset=offset, emit=em)
        np.testing.assert_array_equal(got, ref)
    assert (ref == -1).any() and (g.degree == 0).any()


def test_chung_lu_on_the_device_equals_host_build():
    """bench.py builds C3's graph with chung_lu(device=cuda) (torch 1-D sort / unique / gathers on
    the GPU): it must be the host numpy construction exactly, at the bench's 1M nodes / ~10M
    edges (C5's 10M-node graph: scripts/check_c5_inputs.py, profiles/r04k_*)."""
    import torch
    from come_amd.graph import chung_lu
    a = chung_lu(1_000_000, 20.0, gamma=2.5, seed=1)
    b = chung_lu(1_000_000, 20.0, gamma=2.5, seed=1, device=torch.device("cuda", 0))
    for n in ("edges", "col", "rowptr", "degree"):
        np.testing.assert_array_equal(getattr(a, n), getattr(b, n), err_msg=n)
