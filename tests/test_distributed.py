"""Multi-process (world size 2, gloo, CPU) tests of the walk sharding and the delta all-reduce
that bench.py runs over RCCL on the GPU."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from come_amd.distributed import DeltaAllReduce, reference_delta_sum, shard_walks


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.RandomState(0)
    w_sync = [rng.randn(37, 8).astype(np.float32), rng.randn(37, 8).astype(np.float32)]
    tables = [torch.from_numpy(t.copy()) for t in w_sync]
    sync = DeltaAllReduce(tables, bucket_elems=50)  # several buckets per table
    # each rank makes its own local progress
    local = []
    for i, t in enumerate(tables):
        delta = np.random.RandomState(100 + 10 * rank + i).randn(*t.shape).astype(np.float32)
        t.add_(torch.from_numpy(delta))
        local.append(t.numpy().copy())
    sync.sync()
    np.save(os.path.join(out_dir, "r%d_t0.npy" % rank), tables[0].numpy())
    np.save(os.path.join(out_dir, "r%d_t1.npy" % rank), tables[1].numpy())
    np.save(os.path.join(out_dir, "r%d_local0.npy" % rank), local[0])
    np.save(os.path.join(out_dir, "r%d_local1.npy" % rank), local[1])
    # second sync with no progress is a no-op
    before = tables[0].clone()
    sync.sync()
    assert torch.equal(before, tables[0])
    # overlapped exchange: progress made between start() and finish() is kept, the other
    # rank's pre-start delta is added exactly once
    t = torch.from_numpy(np.full((5, 3), 1.0, np.float32))
    ov = DeltaAllReduce([t])
    t.add_(float(rank + 1))            # delta before start: rank 0 +1, rank 1 +2
    ov.start()
    t.add_(10.0 * (rank + 1))          # progress while the exchange is in flight
    ov.finish()
    expect = 1.0 + 1.0 + 2.0 + 10.0 * (rank + 1)
    assert torch.allclose(t, torch.full_like(t, expect)), (rank, t)
    ov.sync()                          # then a blocking sync reconciles the replicas
    assert torch.allclose(t, torch.full_like(t, 1.0 + 3.0 + 30.0)), (rank, t)
    # sharding: every walk exactly once across ranks
    walks = np.arange(101 * 3).reshape(101, 3)
    seeds = np.arange(101)
    ws, ss = shard_walks(walks, seeds, rank, world)
    got = [None] * world
    dist.all_gather_object(got, ss.tolist())
    if rank == 0:
        assert sorted(sum(got, [])) == list(range(101))
    dist.destroy_process_group()


def test_delta_allreduce_world2(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    rng = np.random.RandomState(0)
    w_sync = [rng.randn(37, 8).astype(np.float32), rng.randn(37, 8).astype(np.float32)]
    for i in range(2):
        locals_ = [np.load(os.path.join(str(tmp_path), "r%d_local%d.npy" % (r, i)))
                   for r in range(world)]
        expect = reference_delta_sum(w_sync[i], locals_)
        r0 = np.load(os.path.join(str(tmp_path), "r0_t%d.npy" % i))
        r1 = np.load(os.path.join(str(tmp_path), "r1_t%d.npy" % i))
        np.testing.assert_array_equal(r0, r1)          # replicas agree after a sync
        np.testing.assert_allclose(r0, expect, rtol=0, atol=1e-5)


def test_single_rank_sync_is_noop():
    t = torch.randn(10, 4)
    before = t.clone()
    DeltaAllReduce([t]).sync()
    assert torch.equal(t, before)


def _sparse_worker(rank, world, port, out_dir):
    """The same training-like sequence through DeltaAllReduce and SparseDeltaAllReduce: each rank
    changes a sparse, partly overlapping set of rows (some to -0.0, some touched then restored),
    exchanges blocking and overlapped; both protocols must leave bit-identical tables."""
    from come_amd.distributed import SparseDeltaAllReduce
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.RandomState(7)
    base = [rng.randn(200, 8).astype(np.float32), rng.randn(150, 16).astype(np.float32)]
    base[0][3] = 0.0
    results = []
    for cls in (DeltaAllReduce, SparseDeltaAllReduce):
        tables = [torch.from_numpy(b.copy()) for b in base]
        sync = cls(tables, bucket_elems=64)
        r2 = np.random.RandomState(50 + rank)
        for step in range(4):
            for t in tables:
                rows = r2.choice(t.shape[0], 12, replace=False)
                t[rows] += torch.from_numpy(r2.randn(12, t.shape[1]).astype(np.float32))
            if step == 0:
                tables[0][3] = -0.0                       # sign-only change is a change
                tables[1][5] += 1.0
                tables[1][5] -= 1.0                       # touched, maybe not restored exactly
            if step % 2 == 0:
                sync.sync()
            else:
                sync.start()
                for t in tables:                          # progress during the exchange
                    t[rank * 3:rank * 3 + 2] *= 1.5
                sync.finish()
        sync.sync()
        if cls is SparseDeltaAllReduce:
            assert 0 < sum(sync.last_rows) <= sum(t.shape[0] for t in tables)
        results.append([t.numpy().copy() for t in tables])
    for a, b in zip(results[0], results[1]):
        assert np.array_equal(a.view(np.int32), b.view(np.int32)), rank
    np.save(os.path.join(out_dir, "sparse_r%d.npy" % rank), results[1][0])
    dist.destroy_process_group()


def test_sparse_delta_allreduce_bit_identical_to_dense_world2(tmp_path):
    world = 2
    mp.spawn(_sparse_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r0 = np.load(os.path.join(str(tmp_path), "sparse_r0.npy"))
    r1 = np.load(os.path.join(str(tmp_path), "sparse_r1.npy"))
    np.testing.assert_array_equal(r0, r1)


def _worker_touched(rank, world, port, out_dir, sparse):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from come_amd.distributed import SparseDeltaAllReduce
    rng = np.random.RandomState(0)
    w_sync = rng.randn(41, 8).astype(np.float32)
    t = torch.from_numpy(w_sync.copy())
    cls = SparseDeltaAllReduce if sparse else DeltaAllReduce
    sync = cls([t], combine="touched_mean", bucket_elems=64)
    # rank 0 changes rows 0..19, rank 1 rows 10..29: rows 10..19 by both, 30.. by none
    lo, hi = (0, 20) if rank == 0 else (10, 30)
    t[lo:hi] += torch.from_numpy(np.random.RandomState(7 + rank).randn(hi - lo, 8)
                                 .astype(np.float32))
    np.save(os.path.join(out_dir, "loc%d.npy" % rank), t.numpy().copy())
    sync.sync()
    np.save(os.path.join(out_dir, "res%d.npy" % rank), t.numpy())
    dist.destroy_process_group()


def test_touched_mean_world2_dense_and_sparse(tmp_path):
    """combine='touched_mean' (the SGNS trainers' exchange): a row changed by k ranks gets the
    mean of their k deltas, a row changed by one rank its full delta, an unchanged row stays;
    dense and row-sparse forms agree and leave both replicas identical."""
    from come_amd.distributed import reference_touched_mean
    res = []
    for sparse in (False, True):
        d = tmp_path / ("s%d" % sparse)
        d.mkdir()
        mp.spawn(_worker_touched, args=(2, _free_port(), str(d), sparse), nprocs=2, join=True)
        w_sync = np.random.RandomState(0).randn(41, 8).astype(np.float32)
        locs = [np.load(str(d / ("loc%d.npy" % r))) for r in range(2)]
        r0, r1 = (np.load(str(d / ("res%d.npy" % r))) for r in range(2))
        np.testing.assert_array_equal(r0, r1)
        ref = reference_touched_mean(w_sync, locs)
        np.testing.assert_allclose(r0, ref, rtol=0, atol=1e-5)
        np.testing.assert_array_equal(r0[30:], w_sync[30:])
        np.testing.assert_allclose(r0[:10], locs[0][:10], rtol=0, atol=1e-6)  # one rank: full
        res.append(r0)
    np.testing.assert_allclose(res[0], res[1], rtol=0, atol=1e-6)


def test_pick_three_local_replicas_rotates_the_winner():
    """combine='pick' (the SGNS trainers' exchange) on three ranks simulated in one
    process (distributed.LocalReplicas): a row changed by one rank takes its full delta, a row
    changed by several takes the delta of the first of them in the rotating order star, star + 1,
    ... (star = exchange index mod N), unchanged rows stay; every replica ends equal; the ranks
    start from rank 0's tables whatever they held (the exchange broadcasts them)."""
    from come_amd.distributed import LocalReplicas, reference_pick
    W, V, d = 3, 12, 4
    g = LocalReplicas(W)
    base = torch.randn(V, d)
    tabs = [base.clone() + (0 if r == 0 else 7.0 * r) for r in range(W)]  # seeded apart
    exs = [DeltaAllReduce([tabs[r]], comm=g.comm(r), combine="pick") for r in range(W)]
    for t in tabs:
        assert torch.equal(t, base)
    rng = np.random.RandomState(5)
    for ex_i in range(4):
        w_sync = tabs[0].numpy().copy()
        for r in range(W):  # rank r changes rows r .. r + 5 (overlaps) and one row alone
            tabs[r][r:r + 6] += torch.from_numpy(rng.randn(6, d).astype(np.float32))
            tabs[r][9 + r] -= 1.0
        locs = [t.numpy().copy() for t in tabs]
        for e in exs:
            e.prepare()
        for e in exs:
            e.start()
        for e in exs:
            e.finish()
            e.settle()
        for t in tabs[1:]:
            assert torch.equal(t, tabs[0])
        ref = reference_pick(w_sync, locs, ex_i % W)
        np.testing.assert_allclose(tabs[0].numpy(), ref, rtol=0, atol=1e-5)
        np.testing.assert_array_equal(tabs[0].numpy()[9 + 0], locs[0][9])  # one rank: its row
        star = ex_i % W
        np.testing.assert_allclose(tabs[0].numpy()[5], locs[star][5], rtol=0, atol=1e-6)


def _worker_pick(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.RandomState(10 + rank)   # every rank seeded differently
    t = torch.from_numpy(rng.randn(41, 8).astype(np.float32))
    sync = DeltaAllReduce([t], combine="pick", bucket_elems=64)
    np.save(os.path.join(out_dir, "start%d.npy" % rank), t.numpy().copy())
    for step in range(3):
        w_sync = t.numpy().copy()
        lo, hi = (0, 20) if rank == 0 else (10, 30)
        t[lo:hi] += torch.from_numpy(np.random.RandomState(7 + rank + 10 * step)
                                     .randn(hi - lo, 8).astype(np.float32))
        np.save(os.path.join(out_dir, "sync%d_%d.npy" % (step, rank)), w_sync)
        np.save(os.path.join(out_dir, "loc%d_%d.npy" % (step, rank)), t.numpy().copy())
        if step == 1:      # overlapped: progress during the exchange is kept
            sync.start()
            t[35] += 1.0 + rank
            sync.finish()
            sync.sync()
        else:
            sync.sync()
        np.save(os.path.join(out_dir, "res%d_%d.npy" % (step, rank)), t.numpy().copy())
    dist.destroy_process_group()


def test_pick_world2_from_differently_seeded_ranks(tmp_path):
    """combine='pick' over a real process group (gloo, world 2): the replicas start from rank 0's
    table although the ranks were seeded differently, rows changed by both ranks take
    the rotating winner's delta (rank 0 at exchange 0, rank 1 at exchange 1, ...), rows changed by
    one rank its full delta, and the replicas agree after every exchange; progress made during an
    overlapped exchange lands on top."""
    from come_amd.distributed import reference_pick
    mp.spawn(_worker_pick, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    ld = lambda n: np.load(str(tmp_path / n))  # noqa: E731
    np.testing.assert_array_equal(ld("start0.npy"), ld("start1.npy"))
    np.testing.assert_array_equal(ld("start0.npy"), np.random.RandomState(10).randn(41, 8)
                                  .astype(np.float32))
    ex = 0
    for step in range(3):
        r0, r1 = ld("res%d_0.npy" % step), ld("res%d_1.npy" % step)
        np.testing.assert_array_equal(r0, r1)
        locs = [ld("loc%d_%d.npy" % (step, r)) for r in range(2)]
        ref = reference_pick(ld("sync%d_0.npy" % step), locs, ex % 2)
        np.testing.assert_allclose(r0[:30], ref[:30], rtol=0, atol=1e-5)
        if step >= 1:   # row 35, changed by both ranks during exchange 1, synced by exchange 2
            np.testing.assert_allclose(r0[35], ld("start0.npy")[35] + 1.0, rtol=0, atol=1e-6)
        if step == 1:   # (star 0 wins exchange 2: rank 0's +1)
            ex += 1
        np.testing.assert_array_equal(r0[30:35], ld("sync%d_0.npy" % step)[30:35])
        ex += 1


def test_pick_real_change_beats_rounding_level_change():
    """An overlapped exchange can leave W_sync + D_own one rounding away from W on a row nobody
    changed since; such a row must not win over a rank that trained it, whatever the rotation:
    keys of rounding-level deltas rank below every real change."""
    from come_amd.distributed import LocalReplicas
    W, V, d = 3, 6, 8
    g = LocalReplicas(W)
    base = torch.randn(V, d) + 3.0
    tabs = [base.clone() for _ in range(W)]
    exs = [DeltaAllReduce([tabs[r]], comm=g.comm(r), combine="pick") for r in range(W)]
    # exchange 0: star = rank 0.  Rank 0 nudges row 2 by one ulp (rounding-level), rank 2 trains it
    tabs[0][2] = torch.nextafter(tabs[0][2], tabs[0][2] + 1.0)
    tabs[2][2] += 0.5
    tabs[1][4] = torch.nextafter(tabs[1][4], tabs[1][4] + 1.0)  # rounding-level, nobody else
    for e in exs:
        e.prepare()
    for e in exs:
        e.start()
    for e in exs:
        e.finish()
        e.settle()
    np.testing.assert_allclose(tabs[0][2].numpy(), base[2].numpy() + 0.5, rtol=1e-6)
    assert torch.equal(tabs[0][4], torch.nextafter(base[4], base[4] + 1.0))  # still taken
    for t in tabs[1:]:
        assert torch.equal(t, tabs[0])


def test_pick_real_change_on_a_large_norm_row():
    """the rounding-level rule is per element.  A real late-training update that moves
    only the row's small elements (here by 1e-4 on elements of magnitude 1e-3) while its largest
    element is 1e3 -- below 2^-20 of the row's largest |W_sync|, the round-4 row-max rule -- is a
    real change and wins the row against a rank whose change is one ulp; reference_pick agrees."""
    from come_amd.distributed import LocalReplicas, reference_pick, _real_change
    W, V, d = 2, 3, 8
    g = LocalReplicas(W)
    base = torch.full((V, d), 1e-3)
    base[:, 0] = 1e3
    tabs = [base.clone() for _ in range(W)]
    exs = [DeltaAllReduce([tabs[r]], comm=g.comm(r), combine="pick") for r in range(W)]
    w_sync = base.numpy().copy()
    tabs[0][1] = torch.nextafter(tabs[0][1], tabs[0][1] + 1.0)  # rank 0 (the star): one ulp
    tabs[1][1, 1:] += 1e-4                                      # rank 1: a real, small update
    assert (tabs[1][1] - base[1]).abs().max() < base[1].abs().max() * 2.0 ** -20
    assert _real_change((tabs[1] - base).numpy(), w_sync)[1]
    assert not _real_change((tabs[0] - base).numpy(), w_sync)[1]
    locs = [t.numpy().copy() for t in tabs]
    for e in exs:
        e.prepare()
    for e in exs:
        e.start()
    for e in exs:
        e.finish()
        e.settle()
    np.testing.assert_array_equal(tabs[0][1].numpy(), locs[1][1])   # rank 1's delta won
    np.testing.assert_allclose(tabs[0].numpy(), reference_pick(w_sync, locs, 0), rtol=0, atol=0)
    assert torch.equal(tabs[1], tabs[0])


def _worker_reset(rank, world, port, out_dir):
    """reset(broadcast=None) after a blocking sync() compares table checksums across
    ranks and broadcasts rank 0's tables only if they differ."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from come_amd.distributed import SparseDeltaAllReduce
    for cls in (DeltaAllReduce, SparseDeltaAllReduce):
        rng = np.random.RandomState(0)
        tables = [torch.from_numpy(rng.randn(37, 8).astype(np.float32)) for _ in range(2)]
        ex = cls(tables)
        calls = [0]
        orig = ex._broadcast

        def counted():
            calls[0] += 1
            orig()
        ex._broadcast = counted
        tables[0][rank] += 1.0       # each rank trains a little, then a blocking sync
        ex.sync()
        ex.reset()                   # replicas identical: checksums agree, no broadcast
        assert calls[0] == 0
        if rank == 1:                # an in-place edit on one rank between two train() calls
            tables[1][5] *= 3.0
        ex.reset()
        assert calls[0] == 1, calls  # every rank saw the mismatch and took rank 0's tables
        got = [None] * world
        dist.all_gather_object(got, [t.numpy().tobytes() for t in tables])
        assert got[0] == got[1]
    dist.destroy_process_group()


def test_reset_repairs_replicas_that_drifted_after_a_sync(tmp_path):
    mp.spawn(_worker_reset, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)


def test_real_change_ignores_a_zero_crossing_rounding_residue():
    """an element that crossed zero in an exchange is tiny in W_sync while the residue
    the exchange left on it is an ulp of its old, large operands -- many ulps of the element
    itself.  A row whose only change is such a residue is not a real change (it must not win the
    row in pick over a rank that trained it); a dense small update still is."""
    from come_amd.distributed import LocalReplicas, reference_pick, _real_change
    W, V, d = 2, 3, 64
    rng = np.random.RandomState(4)
    base = torch.from_numpy(rng.uniform(0.5, 1.5, (V, d)).astype(np.float32))
    base[1, 3] = 3e-8                          # crossed zero: tiny now
    tabs = [base.clone() for _ in range(W)]
    g = LocalReplicas(W)
    exs = [DeltaAllReduce([tabs[r]], comm=g.comm(r), combine="pick") for r in range(W)]
    tabs[0][1, 3] += 6e-8                      # rank 0 (the star): an ulp of 1.0 left on it
    tabs[1][1] += torch.from_numpy(rng.uniform(-1e-4, 1e-4, d).astype(np.float32))  # trained
    w_sync = base.numpy().copy()
    d0 = (tabs[0] - base).numpy()
    assert (np.abs(d0) > np.abs(w_sync) * 2.0 ** -20).any(axis=1)[1]  # the old rule: "real"
    assert not _real_change(d0, w_sync)[1]
    assert not bool(_real_change(tabs[0] - base, base)[1])             # torch path agrees
    assert _real_change((tabs[1] - base).numpy(), w_sync)[1]
    locs = [t.numpy().copy() for t in tabs]
    assert not np.array_equal(locs[0][1], locs[1][1])
    for e in exs:
        e.prepare()
    for e in exs:
        e.start()
    for e in exs:
        e.finish()
        e.settle()
    np.testing.assert_array_equal(tabs[0][1].numpy(), locs[1][1])      # rank 1's update won
    np.testing.assert_allclose(tabs[0].numpy(), reference_pick(w_sync, locs, 0), rtol=0, atol=0)
    assert torch.equal(tabs[1], tabs[0])
