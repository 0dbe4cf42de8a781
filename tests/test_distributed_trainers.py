"""World-size-2 gloo tests (CPU) of the trainers' multi-GPU path (Context2Vec / Node2Vec with
distributed=True): corpus sharding, per-walk seeds identical to a one-process run, the global
numpy RNG advanced identically on every rank, the number and arithmetic of the exchanges, and
replicas identical at the end.

The kernels need a GPU, so the launches are replaced by an ADDITIVE stand-in (each walk / edge adds
a fixed function of its rows and seed to the rows it names): with additive updates the delta-sum
exchange must reproduce the one-process result exactly up to fp32 summation order, which pins the
orchestration independently of Hogwild statistics (those are tier C, tests/test_gpu_tierc.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_o2(node, ctx, walks, seeds, window, negative, table, lr, alpha, mode, hot=None,
             update_count=None, opts=None):
    w = walks.long()
    s = (seeds.long() % 7 + 1).to(torch.float32)
    for p in range(w.shape[0]):
        r = w[p][w[p] >= 0]
        node.index_add_(0, r, torch.full((len(r), node.shape[1]), 1e-3, dtype=torch.float32)
                        * s[p])
        ctx.index_add_(0, r, torch.full((len(r), ctx.shape[1]), 2e-3, dtype=torch.float32))


def _fake_o1(node, edges, seeds, negative, table, lr, mode, hot=None, opts=None):
    e = edges.long()
    s = (seeds.long() % 5 + 1).to(torch.float32)
    for p in range(e.shape[0]):
        node.index_add_(0, e[p], torch.full((2, node.shape[1]), 1e-3, dtype=torch.float32) * s[p])


def _setup(V=40, d=8, seed=11):
    import come_amd.training_sdg_inner as tsi
    from come_amd.model import Model
    tsi.sgns_o2 = _fake_o2
    tsi.sgns_o1 = _fake_o1
    np.random.seed(seed)
    model = Model((np.arange(1, V + 1), np.arange(1, V + 1) % 5 + 1), size=d, table_size=1000,
                  k=1, device="cpu")
    rng = np.random.RandomState(3)
    walks = rng.randint(1, V + 1, (53, 9))
    walks[5, 4:] = -1  # a short walk
    edges = rng.randint(1, V + 1, (31, 2))
    return model, walks, edges


def _run(model, walks, edges, distributed, sync_walks, combine="sum"):
    from come_amd.context_embeddings import Context2Vec
    from come_amd.node_embeddings import Node2Vec
    cl = Context2Vec(lr=0.1, window_size=2, negative=3, distributed=distributed,
                     sync_walks=sync_walks, combine=combine)
    p1 = cl.train(model, paths=walks, total_nodes=walks.size, alpha=1.0)
    if combine != "sum":
        return p1, None
    nl = Node2Vec(lr=0.1, negative=3, distributed=distributed, sync_edges=7, combine=combine)
    p2 = nl.train(model, edges=edges, iter=2)
    p3 = cl.train(model, paths=walks, total_nodes=walks.size, alpha=1.0)  # reuses the exchange
    return p1 + p3, p2


def _worker(rank, world, port, out_dir, sync_walks, overlap, combine="sum"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from come_amd import context_embeddings as ce
    model, walks, edges = _setup()
    orig = ce.Context2Vec.__init__

    def init(self, *a, **k):
        orig(self, *a, **k)
        self.overlap = overlap
    ce.Context2Vec.__init__ = init
    if combine != "sum":
        before = model.node_embedding.clone(), model.context_embedding.clone()
    p_o2, p_o1 = _run(model, walks, edges, True, sync_walks, combine)
    if combine != "sum":  # this rank's own progress (the stand-in on its shard, from the base)
        from come_amd.distributed import shard_walks
        import come_amd.training_sdg_inner as tsi
        own = _setup()[0]  # reseeds and builds the model: the RNG state train() drew from
        seeds = tsi.draw_seeds(len(walks))
        ws, _ = shard_walks(walks, np.zeros(len(walks)), rank, world)
        _, ss = shard_walks(walks, seeds, rank, world)
        rows = own.rows_of(ws.reshape(-1)).reshape(ws.shape).astype(np.int32)
        _fake_o2(own.node_embedding, own.context_embedding, torch.from_numpy(rows),
                 torch.from_numpy(ss.view(np.int64)), 2, 3, None, 0.1, 1.0, 0)
        np.save(os.path.join(out_dir, "own_node%d.npy" % rank), own.node_embedding.numpy())
        np.save(os.path.join(out_dir, "own_ctx%d.npy" % rank), own.context_embedding.numpy())
        np.save(os.path.join(out_dir, "base_node.npy"), before[0].numpy())
        np.save(os.path.join(out_dir, "base_ctx.npy"), before[1].numpy())
    np.save(os.path.join(out_dir, "node%d.npy" % rank), model.node_embedding.numpy())
    np.save(os.path.join(out_dir, "ctx%d.npy" % rank), model.context_embedding.numpy())
    np.save(os.path.join(out_dir, "rng%d.npy" % rank), np.random.random_sample(4))
    np.save(os.path.join(out_dir, "pairs%d.npy" % rank), np.array([p_o2, p_o1]))
    dist.destroy_process_group()


def _check(tmp_path, sync_walks, overlap):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), sync_walks, overlap),
             nprocs=world, join=True)
    model, walks, edges = _setup()
    p_o2, p_o1 = _run(model, walks, edges, False, sync_walks)
    rng = np.random.random_sample(4)
    ld = lambda n, r: np.load(os.path.join(str(tmp_path), "%s%d.npy" % (n, r)))  # noqa: E731
    for r in range(world):
        # replicas identical, equal to the one-process run (additive stand-in), RNG in step
        np.testing.assert_array_equal(ld("node", r), ld("node", 0))
        np.testing.assert_array_equal(ld("ctx", r), ld("ctx", 0))
        np.testing.assert_allclose(ld("node", r), model.node_embedding.numpy(), rtol=0,
                                   atol=2e-5)
        np.testing.assert_allclose(ld("ctx", r), model.context_embedding.numpy(), rtol=0,
                                   atol=2e-5)
        np.testing.assert_array_equal(ld("rng", r), rng)
    tot = ld("pairs", 0) + ld("pairs", 1)
    assert tot[0] == p_o2 and tot[1] == p_o1, (tot, p_o2, p_o1)


def test_trainers_distributed_world2_overlapped(tmp_path):
    _check(tmp_path, sync_walks=5, overlap=True)    # 6 exchanges per train(), overlapped


def test_trainers_distributed_world2_blocking_one_sync(tmp_path):
    _check(tmp_path, sync_walks=1 << 17, overlap=False)  # one exchange per train()


def test_trainers_distributed_world2_touched_mean(tmp_path):
    """The trainers' default combine rule, one exchange: every row gets the mean of the deltas
    of the ranks that changed it (distributed.reference_touched_mean), replicas identical."""
    from come_amd.distributed import reference_touched_mean
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), 1 << 17, False, "touched_mean"),
             nprocs=world, join=True)
    ld = lambda n: np.load(os.path.join(str(tmp_path), n + ".npy"))  # noqa: E731
    for tab in ("node", "ctx"):
        ref = reference_touched_mean(ld("base_" + tab), [ld("own_%s%d" % (tab, r))
                                                         for r in range(world)])
        for r in range(world):
            np.testing.assert_allclose(ld("%s%d" % (tab, r)), ref, rtol=0, atol=2e-6)
        np.testing.assert_array_equal(ld(tab + "0"), ld(tab + "1"))


def _worker_seeded(rank, world, port, out_dir, combine, sparse=False):
    """Every rank seeds numpy differently (so Model.reset_weights draws different tables)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from come_amd.context_embeddings import Context2Vec
    from come_amd.node_embeddings import Node2Vec
    model, walks, edges = _setup(seed=100 + rank)
    np.save(os.path.join(out_dir, "init%d.npy" % rank), model.node_embedding.numpy().copy())
    Context2Vec(lr=0.1, window_size=2, negative=3, distributed=True, sync_walks=5,
                combine=combine, sparse_sync=sparse).train(model, paths=walks,
                                                           total_nodes=walks.size, alpha=1.0)
    Node2Vec(lr=0.1, negative=3, distributed=True, combine=combine).train(model, edges=edges,
                                                                        iter=2)
    np.save(os.path.join(out_dir, "node%d.npy" % rank), model.node_embedding.numpy())
    np.save(os.path.join(out_dir, "ctx%d.npy" % rank), model.context_embedding.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("sparse", [False, True])
def test_trainers_distributed_ranks_seeded_differently(tmp_path, sparse):
    """the exchange adds deltas to each rank's own W_sync, so replicas that start
    apart would never meet.  The exchange -- dense, or row-sparse (Context2Vec(sparse_sync=True))
    -- takes rank 0's tables when it is built (a broadcast), so ranks seeded differently still
    leave train() with identical replicas."""
    world = 2
    mp.spawn(_worker_seeded, args=(world, _free_port(), str(tmp_path), "touched_mean", sparse),
             nprocs=world, join=True)
    ld = lambda n: np.load(os.path.join(str(tmp_path), n + ".npy"))  # noqa: E731
    assert not np.array_equal(ld("init0"), ld("init1"))   # the ranks did start apart
    np.testing.assert_array_equal(ld("node0"), ld("node1"))
    np.testing.assert_array_equal(ld("ctx0"), ld("ctx1"))


def test_trainers_distributed_world2_pick(tmp_path):
    """combine='pick', one exchange: a row changed by both ranks takes rank 0's delta (the star
    of exchange 0), a row changed by one rank its delta (distributed.reference_pick); replicas
    identical.  pick never overlaps its exchange (DeltaAllReduce.OVERLAP_SAFE)."""
    from come_amd.distributed import DeltaAllReduce, reference_pick
    assert "pick" not in DeltaAllReduce.OVERLAP_SAFE
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), 1 << 17, True, "pick"),
             nprocs=world, join=True)
    ld = lambda n: np.load(os.path.join(str(tmp_path), n + ".npy"))  # noqa: E731
    for tab in ("node", "ctx"):
        ref = reference_pick(ld("base_" + tab), [ld("own_%s%d" % (tab, r)) for r in range(world)],
                             0)
        for r in range(world):
            np.testing.assert_allclose(ld("%s%d" % (tab, r)), ref, rtol=0, atol=2e-6)
        np.testing.assert_array_equal(ld(tab + "0"), ld(tab + "1"))


def _worker_broadcasts(rank, world, port, out_dir, sparse):
    """Count the exchange's whole-table broadcasts over three train() calls of one trainer."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from come_amd import distributed as dd
    from come_amd.context_embeddings import Context2Vec
    calls = []
    orig = dd.TorchComm.broadcast

    def counted(self, t, src=0):
        calls.append(t.numel())
        return orig(self, t, src)
    dd.TorchComm.broadcast = counted
    model, walks, _ = _setup(seed=100 + rank)
    cl = Context2Vec(lr=0.1, window_size=2, negative=3, distributed=True, sync_walks=5,
                     sparse_sync=sparse)
    n = []
    for _ in range(3):
        cl.train(model, paths=walks, total_nodes=walks.size, alpha=1.0)
        n.append(len(calls))
    ex = cl.exchange(model)          # after a blocking sync: no broadcast
    n.append(len(calls))
    ex.start()                       # an exchange in flight: the replicas may differ ...
    ex.finish()
    ex.reset()                       # ... so reset() takes rank 0's tables again
    n.append(len(calls))
    ex.reset(broadcast=True)
    n.append(len(calls))
    np.save(os.path.join(out_dir, "bc%d.npy" % rank), np.array(n))
    dist.destroy_process_group()


@pytest.mark.parametrize("sparse", [False, True])
def test_exchange_broadcasts_only_when_replicas_may_differ(tmp_path, sparse):
    """train() ends with a blocking exchange, which leaves the replicas bit-identical,
    so the next train()'s reset() must not broadcast the whole tables again (41 GB per call at
    C5's shard).  Broadcasts: 2 tables when the exchange is built, none on later train() calls or
    a reset() after a blocking sync, 2 after an overlapped exchange or when forced."""
    world = 2
    mp.spawn(_worker_broadcasts, args=(world, _free_port(), str(tmp_path), sparse),
             nprocs=world, join=True)
    for r in range(world):
        n = np.load(os.path.join(str(tmp_path), "bc%d.npy" % r)).tolist()
        assert n == [2, 2, 2, 2, 4, 6], n
