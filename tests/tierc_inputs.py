"""Tier-C inputs and the held-out loss (TEST INFRASTRUCTURE; SURVEY.md §8c tier C).

Inputs that are built on the host only -- Chung-Lu graph, the reference's make_table, walks from the
exact CPython-stream host walker (graph_utils._corpus, utils/graph_utils.py:20-46 + 187-192),
numpy RandomState picks / initial tables / per-walk seeds -- so the sequential oracle can replay
them anywhere (in the container, for a committed fixture) and the GPU side rebuilds the same
arrays on the box; the two are matched by a digest of the inputs.

No torch here: the fixture scripts run on a CPU-only host.
"""
import hashlib
import random

import numpy as np


def log_sigmoid(x):
    return -np.logaddexp(0.0, -x)


def sgns_loss(inp, out, rows_in, rows_pos, rows_neg, chunk=20000):
    """Mean held-out SGNS loss (float64, exact sigmoid): -log s(u.c+) - sum_k log s(-u.c_k),
    over pairs (rows_in[p], rows_pos[p], rows_neg[p, :]), evaluated `chunk` pairs at a time."""
    total = 0.0
    m = len(rows_in)
    for s in range(0, m, chunk):
        ri, rp, rn = rows_in[s:s + chunk], rows_pos[s:s + chunk], rows_neg[s:s + chunk]
        u = inp[ri].astype(np.float64)
        lp = log_sigmoid(np.einsum("pd,pd->p", u, out[rp].astype(np.float64)))
        ln = log_sigmoid(-np.einsum("pd,pkd->pk", u, out[rn].astype(np.float64))).sum(1)
        total += float((lp + ln).sum())
    return -total / m


def heldout_o2_pairs(walks, w, n, table, count, seed):
    """`count` (input row, positive row) window pairs of held-out walks (pyx:494-506: input
    idx[j], positive idx[i]) with n negatives each drawn from the negative table."""
    rng = np.random.RandomState(seed)
    P, L = walks.shape
    p = rng.randint(0, P, 4 * count)
    i = rng.randint(0, L, 4 * count)
    off = rng.randint(1, w + 1, 4 * count) * rng.choice([-1, 1], 4 * count)
    j = i + off
    ok = (j >= 0) & (j < L)
    p, i, j = p[ok], i[ok], j[ok]
    ci, cj = walks[p, i], walks[p, np.clip(j, 0, L - 1)]
    ok = (ci >= 0) & (cj >= 0)
    ci, cj = ci[ok][:count], cj[ok][:count]
    neg = table[rng.randint(0, len(table), (len(ci), n))].astype(np.int64)
    return cj, ci, neg


class HostInputs(object):
    """One tier-C workload built on the host (see the module docstring)."""

    def __init__(self, V, graph_seed, d, train_walks, held_walks=20000, T=100_000_000,
                 walk_streams=(11, 12), pick_seed=7, L=80, mean_degree=20.0, walker="host",
                 walk_seed=0, device=None):
        """walker "host": full corpus passes of the exact CPython-stream host walker (one per
        entry of walk_streams), then a random pick of walks; walker "philox": the device walker's
        stream (come_random_walks, seed walk_seed) from train + held distinct random starts --
        on `device` when given (a GPU: the product's kernel), else its CPU restatement
        (oracle/come_oracle_walks.c), identical walks (tests/test_gpu_walks.py)."""
        from oracle import oracle as orc
        from come_amd import graph_utils as gu
        from come_amd.graph import chung_lu
        g = chung_lu(V, mean_degree, gamma=2.5, seed=graph_seed, device=device)
        self.g = g
        self.table = orc.make_table(g.degree.astype(np.float64), T)
        rng = np.random.RandomState(pick_seed)
        if walker == "philox":
            starts = rng.choice(V, train_walks + held_walks, replace=False).astype(np.int32)
            if device is not None:
                import torch
                walks = gu.device_walks(torch.as_tensor(g.rowptr, device=device),
                                        torch.as_tensor(g.col, device=device),
                                        torch.as_tensor(starts, device=device), L, alpha=0.0,
                                        seed=walk_seed).cpu().numpy()
            else:
                walks = orc.philox_walks(g.rowptr, g.col, starts, L, 0.0, seed=walk_seed)
        else:
            gh = gu.Graph(np.arange(1, g.V + 1), g.rowptr, g.col.astype(np.int32), g.degree,
                          np.zeros((0, 2), np.int32))
            walks = gu._corpus(gh, [1] * len(walk_streams), L, 0.0,
                               [random.Random(s) for s in walk_streams],
                               threads=len(walk_streams))
            walks = np.asarray(walks, np.int32)
            pick = rng.choice(walks.shape[0], train_walks + held_walks, replace=False)
            walks = walks[pick]
        self.train, self.held = walks[:train_walks], walks[train_walks:]
        wbytes = walks.tobytes()
        del walks
        # = rng.uniform(-1, 1, (V, d)).astype(np.float32), drawn in row blocks (same stream,
        # without a V x d float64 temporary: 20 GB at C5's 10M x 256)
        self.node0 = np.empty((g.V, d), np.float32)
        for r0 in range(0, g.V, 1 << 20):
            r1 = min(g.V, r0 + (1 << 20))
            self.node0[r0:r1] = rng.uniform(-1, 1, (r1 - r0, d))
        self.seeds = rng.randint(0, 2 ** 48, train_walks, dtype=np.int64).astype(np.uint64)
        self.digest = hashlib.sha256(wbytes + self.seeds.tobytes() +
                                     self.node0.tobytes()[:1 << 20] +
                                     self.table.tobytes()[:1 << 20]).hexdigest()

    def heldout(self, w, n, count=200_000, seed=24):
        return heldout_o2_pairs(self.held, w, n, self.table, count, seed)


def compact_loss(node, ctx, rows_in, rows_pos, rows_neg):
    """sgns_loss with node / ctx given as row-indexable tables (numpy arrays or CUDA tensors):
    only the rows the held-out pairs name are gathered (and brought to the host), so a 10 GB
    device table is never copied whole.  Same float64 arithmetic, same value."""
    ui, ri = np.unique(rows_in, return_inverse=True)
    uc, rc = np.unique(np.concatenate([rows_pos, rows_neg.ravel()]), return_inverse=True)

    def take(t, rows):
        if isinstance(t, np.ndarray):
            return t[rows]
        import torch
        return t[torch.from_numpy(rows).to(t.device)].cpu().numpy()
    inp, out = take(node, ui), take(ctx, uc)
    npos = len(rows_pos)
    return sgns_loss(inp, out, ri.reshape(rows_in.shape), rc[:npos],
                     rc[npos:].reshape(rows_neg.shape))


# configs[4]/C5: Chung-Lu 10M nodes / ~100M edges (seed 4), d = 256, n = 10,
# T = 1e8, lr 0.1, w 5, L 80, one launch of 131,072 walks (1.0e8 pair updates).  C5_1M: the same
# kernel on a 1M-node graph of the same generator (hubs hold 10x the table share they hold at 10M
# nodes: the more contended case).
C5 = dict(V=10_000_000, graph_seed=4, d=256, train_walks=131_072, walker="philox",
          walk_seed=41, pick_seed=43)
C5_1M = dict(V=1_000_000, graph_seed=4, d=256, train_walks=131_072, walk_streams=(41,),
             pick_seed=43)
C5_HYPER = dict(window=5, negative=10, lr=0.1)


def c5_inputs(device=None):
    return HostInputs(device=device, **C5)


def c5_1m_inputs():
    return HostInputs(**C5_1M)


# configs[2]/C3 at the bench's own launch: the 1M-node graph, one launch of 1,048,576 walks
# (8.07e8 pair updates); fixture tests/golden/tierc_c3_1m_seq.json (scripts/tierc_c3_1m.py).
C3_1M = dict(V=1_000_000, graph_seed=1, d=128, train_walks=1 << 20, walk_streams=(11, 12),
             pick_seed=7)
C3_HYPER = dict(window=5, negative=5, lr=0.1)


def c3_1m_inputs():
    return HostInputs(**C3_1M)


# configs[2]/C3 over 4 launches' worth of walks (4,194,304 walks, 3.2e9 pair updates): the
# multi-GPU path's tier C at sync periods of up to 524,288 walks per rank with 8 ranks; fixture
# tests/golden/tierc_c3_4m_seq.json (scripts/make_tierc_fixture_host.py c3_4m, ~3 h of one core).
C3_4M = dict(V=1_000_000, graph_seed=1, d=128, train_walks=1 << 22,
             walk_streams=(11, 12, 13, 14, 15), pick_seed=7)


def c3_4m_inputs():
    return HostInputs(**C3_4M)
