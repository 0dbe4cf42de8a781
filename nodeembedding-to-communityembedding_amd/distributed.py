"""Multi-GPU data parallelism: walk sharding + periodic delta all-reduce for the SGNS path, row
sharding + all-gather / sufficient-statistics all-reduce for the community step and GMM EM.

The reference is one process with Hogwild threads over shared numpy tables; it has
no communication backend.  Across the GPUs of a node the same idea becomes: every rank (one
process per GPU) holds a full replica of node_embedding and context_embedding in HBM, trains its
own contiguous shard of the walks (each walk keeps its own seed, so a walk's negative stream is
identical to the single-GPU run), and every ``sync_every`` batches the ranks exchange what they
changed:

    delta_r = W_r - W_sync          (local progress since the last sync)
    W       = W_sync + combine_r delta_r  (all-reduce SUM over RCCL / xGMI, then the combine)
    W_sync  = W

Combine rules (``combine=``): "sum" (SURVEY.md §8e's first-order merge: every rank's progress
kept), "mean" (model averaging), "touched_mean" (a row moves by the mean delta of the ranks that
changed it -- one extra uint8 all-reduce of the per-row change flags) and "hot_mean" (given rows
averaged, the rest summed).  The SGNS trainers default to "touched_mean": at lr 0.1 the sum
diverges once N replicas saturate the same hub rows within a period (multi-rank tier C,
DESIGN.md §6).  With N = 1 sync is a no-op.  The all-reduce runs on torch.distributed with the
"nccl" backend (= RCCL on ROCm); tests run the same code on "gloo" with CPU tensors.

Overlap (``start`` / ``finish``): the exchange of batch s runs on RCCL's stream while batch s+1
trains.  ``start`` snapshots the local delta D_r = W_r - W_sync and launches the asynchronous
all-reduce of D; ``finish`` waits for it and applies the other ranks' deltas on top of whatever the
rank trained meanwhile:

    W      += sum_r D_r - D_own      (others' progress; own progress is already in W)
    W_sync += sum_r D_r

after which W - W_sync is exactly the rank's progress since ``start`` -- no update is lost or
counted twice, and the replicas differ only by what each trained after ``start`` (Hogwild-style
staleness of one batch).  ``sync`` = ``start`` + ``finish`` (no overlap).

``SparseDeltaAllReduce`` is the same protocol over the rows some rank changed only: each rank
flags the rows where W differs bitwise from W_sync, the flags are OR-ed across ranks (one uint8
all-reduce MAX of V bytes), and only the union's rows are gathered, all-reduced and scattered
back.  Unchanged rows have a delta of exactly +0 on every rank, so the tables end bit-identical
to the dense exchange.  It keeps one full replica per table (W_sync) instead of three; the
exchange buffers are [rows changed x d].
"""
import numpy as np


def shard_range(n, rank, world):
    """Contiguous block [lo, hi) of n units for `rank` (sizes differ by at most one)."""
    base, rem = divmod(int(n), int(world))
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard_walks(walks, seeds, rank, world):
    """This rank's contiguous shard of (walks, seeds)."""
    lo, hi = shard_range(len(seeds), rank, world)
    return walks[lo:hi], seeds[lo:hi]


def world_of(group=None):
    """(rank, world) of this process in `group`; (0, 1) without torch.distributed."""
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def all_gather_rows(x, group=None):
    """Row-sharded exchange for the community step: rank r owns rows
    shard_range(V, r, N) of the replicated [V, ...] tensor x and has updated only those; afterwards
    every replica holds every rank's rows.  One all_gather_into_tensor over shards padded to
    ceil(V / N) rows (RCCL on the GPU, gloo in the CPU tests)."""
    import torch.distributed as dist
    rank, world = world_of(group)
    if world == 1:
        return x
    V = x.shape[0]
    chunk = -(-V // world)
    lo, hi = shard_range(V, rank, world)
    send = x.new_empty((chunk,) + tuple(x.shape[1:]))
    send[:hi - lo].copy_(x[lo:hi])
    recv = x.new_empty((world * chunk,) + tuple(x.shape[1:]))
    dist.all_gather_into_tensor(recv, send, group=group)
    for r in range(world):
        if r != rank:
            l, h = shard_range(V, r, world)
            x[l:h].copy_(recv[r * chunk:r * chunk + (h - l)])
    return x


def all_reduce_sum(tensors, group=None):
    """In-place SUM all-reduce of a list of same-dtype tensors as ONE flat collective (the GMM
    sufficient statistics: K + K d floats, then K d^2; few large calls suit xGMI rings)."""
    import torch
    import torch.distributed as dist
    rank, world = world_of(group)
    if world == 1:
        return tensors
    flat = torch.cat([t.reshape(-1) for t in tensors])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    o = 0
    for t in tensors:
        t.copy_(flat[o:o + t.numel()].view_as(t))
        o += t.numel()
    return tensors


class TorchComm(object):
    """The collective the exchanges run on: torch.distributed over `group` ("nccl" = RCCL over
    xGMI on the GPUs, gloo in the CPU tests)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.group = group
        up = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if up else 1
        self.rank = dist.get_rank(group) if up else 0

    def all_reduce(self, t, op="sum", async_op=False):
        import torch.distributed as dist
        return dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX,
                               group=self.group, async_op=async_op)

    def broadcast(self, t, src=0):
        """Blocking broadcast of `t` from group rank `src`."""
        import torch.distributed as dist
        gsrc = src if self.group is None else dist.get_global_rank(self.group, src)
        dist.broadcast(t, gsrc, group=self.group)


class LocalReplicas(object):
    """`world` replicas in ONE process standing in for `world` ranks -- the multi-replica tier-C
    runs on one GPU (tests/test_gpu_tierc.py, scripts/tierc_replicas.py) drive N exchange objects
    through it with exactly the product's arithmetic.  ``comm(r)`` is rank r's collective; the
    k-th all-reduce of every rank forms one collective, which completes (SUM in rank order) when
    a handle of it is waited on -- after every rank has contributed.  Only asynchronous
    all-reduces are supported (a blocking one could not complete in a sequential simulation)."""

    def __init__(self, world):
        self.world = int(world)
        self.calls = [[] for _ in range(self.world)]
        self.done = 0
        self.bcast = []
        self.bcount = [0] * self.world

    def comm(self, rank):
        return _LocalComm(self, rank)

    def _complete(self, k):
        while self.done <= k:
            i = self.done
            ops = [self.calls[r][i] for r in range(self.world)]
            if len(set(op for op, _ in ops)) != 1:
                raise RuntimeError("LocalReplicas: ranks disagree on collective %d" % i)
            ts = [t for _, t in ops]
            acc = ts[0].clone()
            for t in ts[1:]:
                if ops[0][0] == "sum":
                    acc.add_(t)
                else:
                    torch_max(acc, t)
            for t in ts:
                t.copy_(acc)
            self.done += 1


def torch_max(acc, t):
    import torch
    torch.maximum(acc, t, out=acc)


class _LocalComm(object):
    def __init__(self, group, rank):
        self.g, self.rank, self.world = group, rank, group.world

    def all_reduce(self, t, op="sum", async_op=False):
        if not async_op or op not in ("sum", "max"):
            raise NotImplementedError("LocalReplicas: asynchronous SUM / MAX all-reduces only")
        k = len(self.g.calls[self.rank])
        self.g.calls[self.rank].append((op, t))
        return _LocalWork(self.g, k)

    def broadcast(self, t, src=0):
        """The k-th broadcast of every rank forms one collective.  Ranks run in rank order, so
        `src` = 0 has posted its tensor before the others copy it (a sequential simulation cannot
        block)."""
        if src != 0:
            raise NotImplementedError("LocalReplicas: broadcasts from rank 0 only")
        k = self.g.bcount[self.rank]
        self.g.bcount[self.rank] += 1
        if self.rank == 0:
            self.g.bcast.append(t.clone())
        else:
            t.copy_(self.g.bcast[k])


class _LocalWork(object):
    def __init__(self, group, k):
        self.g, self.k = group, k

    def wait(self):
        self.g._complete(self.k)


REAL_CHANGE_REL = 2.0 ** -20  # 8 ulps of fp32: above any rounding an exchange leaves behind
REAL_CHANGE_FRAC = 8          # a real change moves at least 1/8 of the row's elements that far


def _real_change(delta, base):
    """Per row: do at least max(1, d / REAL_CHANGE_FRAC) elements of ``delta`` exceed 8 ulps of
    the same element of ``base``?  A real SGD update of a row is a dense vector (g times another
    row, pyx:146-147): even with a decayed learning rate on a large-norm row it moves nearly every
    element by many of its own ulps.  The residue an overlapped exchange leaves on a row nobody
    changed is a few ulps of the exchange's operands -- above 8 ulps of the element itself only
    where the element lost most of its magnitude in that exchange (it crossed zero), which a few
    elements of a row do, not an eighth of them (a per-element "any" let such a
    crossing mark a rounding-only row as real)."""
    import torch
    if isinstance(delta, np.ndarray):
        v = np.abs(delta.reshape(delta.shape[0], -1).astype(np.float32))
        b = np.abs(base.reshape(base.shape[0], -1).astype(np.float32))
        need = max(1, v.shape[1] // REAL_CHANGE_FRAC)
        return (v > b * np.float32(REAL_CHANGE_REL)).sum(axis=1) >= need
    v = delta.reshape(delta.shape[0], -1)
    b = base.reshape(base.shape[0], -1)
    need = max(1, v.shape[1] // REAL_CHANGE_FRAC)
    out = torch.zeros(v.shape[0], dtype=torch.bool, device=v.device)
    step = max(1, (1 << 24) // max(1, v.shape[1]))  # row blocks: temporaries of <= 64 MB
    for lo in range(0, v.shape[0], step):
        hi = min(lo + step, v.shape[0])
        out[lo:hi] = (v[lo:hi].abs() > b[lo:hi].abs() * REAL_CHANGE_REL).sum(dim=1) >= need
    return out


def _checksums(tables):
    """Per table: the int64 sum of its 32-bit words, in blocks of 16M elements (no table-sized
    temporary).  Two replicas with equal sums are taken to be equal."""
    import torch
    out = []
    for t in tables:
        w = t.reshape(-1).view(torch.int32)
        acc = torch.zeros((), dtype=torch.int64, device=t.device)
        for lo in range(0, w.numel(), 1 << 24):
            acc += w[lo:lo + (1 << 24)].sum(dtype=torch.int64)
        out.append(acc)
    return torch.stack(out) if out else torch.zeros(0, dtype=torch.int64)


def _replicas_agree(comm, tables):
    """True when every rank's tables have the same checksums (_checksums): one all-reduce of 2 x
    len(tables) int64 (MAX of s and of -s, i.e. max and min), instead of broadcasting the tables.
    A one-process simulation (LocalReplicas) cannot run a blocking collective: it reports False,
    so its callers broadcast as before."""
    if isinstance(comm, _LocalComm):
        return False
    import torch
    c = _checksums(tables)
    both = torch.cat([c, -c])
    comm.all_reduce(both, op="max")
    n = c.numel()
    return bool(torch.equal(both[:n], -both[n:]))


def _fused(t):
    """CUDA fp32 tables with n % 4 == 0 use the fused HIP passes (come_delta_begin/end); CPU
    tensors (gloo tests) use the same arithmetic in torch ops."""
    import torch
    return t.is_cuda and t.dtype == torch.float32 and t.numel() % 4 == 0


def _native(name, a, b, c, d):
    from . import _lib
    from ._lib import check, ptr, stream_handle
    check(getattr(_lib.lib(), name)(ptr(a), ptr(b), ptr(c), ptr(d), a.numel(),
                                    stream_handle(a.device)), name)


class DeltaAllReduce(object):
    """Delta-sum synchronisation of a list of replicated tables (torch tensors, same shape on
    every rank).  ``bucket_elems`` bounds the size of each all-reduce call (large fp32 buckets:
    xGMI collectives are bandwidth-bound per link, so few big calls beat many small ones)."""

    COMBINES = ("sum", "mean", "touched_mean", "hot_mean", "pick", "hot_pick")
    # combines whose exchange may overlap the next batch (start() now, finish() after it).  pick
    # may not: a rank that lost a row keeps training its own copy meanwhile, and finish() then
    # adds that progress to the winner's copy -- on a 100k-node Chung-Lu graph at lr 0.1 the
    # held-out loss diverges (+45..+130%, scripts/replicas_cpu.py) where the blocking exchange
    # stays within a few percent
    OVERLAP_SAFE = ("sum", "mean", "touched_mean", "hot_mean")

    def __init__(self, tables, group=None, bucket_elems=1 << 26, comm=None, combine="sum",
                 mean_rows=None, pick_rows=None, same_start=True, force_exchange=False):
        import torch
        if combine not in self.COMBINES:
            raise ValueError("combine must be one of %s" % (self.COMBINES,))
        if combine == "hot_mean" and (mean_rows is None or len(mean_rows) != len(tables)):
            raise ValueError("combine='hot_mean' needs one boolean row mask per table")
        if combine == "hot_pick" and (pick_rows is None or len(pick_rows) != len(tables)):
            raise ValueError("combine='hot_pick' needs one boolean row mask per table")
        self.mean_rows = mean_rows
        self.pick_rows = pick_rows
        self.tables = list(tables)
        self.group = group
        self.comm = comm if comm is not None else TorchComm(group)
        self.world = self.comm.world
        self.rank = getattr(self.comm, "rank", 0)
        # one rank exchanges nothing; force_exchange (tests) runs the whole protocol anyway, so
        # a one-GPU box drives RCCL's collectives and the stream waits (tests/test_gpu_rccl.py)
        self.active = self.world > 1 or bool(force_exchange)
        self.bucket = int(bucket_elems)
        self.combine = combine
        self.exchanges = 0
        if self.active and same_start:
            self._broadcast()
        self.snap = [t.clone() for t in self.tables] if self.active else None
        self.dsum = [torch.empty_like(t) for t in self.tables] if self.active else None
        self.down = [torch.empty_like(t) for t in self.tables] if self.active else None
        self.cnt = None
        self.prio = None
        self.prepared = False
        self.pending = []
        self.synced = self.active and same_start  # replicas identical right now

    def _broadcast(self):
        """Every replica starts from rank 0's tables: the exchange adds deltas to each rank's own
        W_sync, so replicas that started apart (ranks seeded differently) would never meet."""
        for t in self.tables:
            self.comm.broadcast(t, 0)

    def reset(self, broadcast=None):
        """Make the current tables the sync base (W_sync = W), after taking rank 0's tables (the
        replicas must agree).  Call when the tables changed outside the exchange (e.g. another
        trainer's distributed step), so that change is not counted once per rank as a delta.
        ``broadcast=None``: broadcast when the replicas may differ.  After a blocking sync() (which
        leaves them bit-identical; a trainer's train() ends with one) the ranks first compare
        table checksums (_replicas_agree: one all-reduce of a few int64) and broadcast only if
        they differ -- a non-distributed step that ran differently per rank, or an in-place edit
        on one rank, is repaired as before, while the common case skips a whole-table
        broadcast per train() call (2 GB of xGMI traffic per call at C3, 41 GB at C5's shard).
        True / False force it."""
        self.finish()
        if self.active:
            if broadcast or (broadcast is None and not (self.synced and
                                                        _replicas_agree(self.comm, self.tables))):
                self._broadcast()
            for t, s in zip(self.tables, self.snap):
                s.copy_(t)
            self.synced = True

    def prepare(self):
        """First half of start(): finish any pending exchange, snapshot this rank's delta
        D = W - W_sync and post the per-row flag all-reduces the combine needs (touched_mean: the
        number of ranks that changed each row; pick: the priority of the rank whose delta a row
        takes).  start() calls it when it has not run; a one-process simulation of N ranks
        (LocalReplicas) calls it on every rank before any rank's start()."""
        if not self.active or self.prepared:
            return
        import torch
        self.finish()
        count = self.combine in ("touched_mean", "hot_pick")
        pick = self.combine in ("pick", "hot_pick")
        self.cnt = [] if count else None
        self.prio = [] if pick else None
        # pick: rank (star + j) % N has priority N - j; the star rotates with every exchange
        if pick and self.world > 127:
            raise ValueError("combine='pick' supports at most 127 ranks (uint8 priorities)")
        star = self.exchanges % self.world
        mine = self.world - (self.rank - star) % self.world
        for t, s, ds, do in zip(self.tables, self.snap, self.dsum, self.down):
            if _fused(t):
                _native("come_delta_begin", t, s, ds, do)  # D = Down = W - W_sync
            else:
                ds.copy_(t)
                ds.sub_(s)                                 # D_own = W - W_sync
                do.copy_(ds)
            if count or pick:  # the rows this rank changed (bitwise W != W_sync)
                f = SparseDeltaAllReduce._flags(t, s)
            if count:
                c = f.clone()
                self.cnt.append(c)
                self.pending.append(self.comm.all_reduce(c, async_op=True))
            if pick:
                # A rank whose change of a row is rounding-level only (an overlapped exchange
                # leaves W_sync + D_own a few roundings away from W on rows nobody else changed)
                # must not win the row over a rank that trained it: such keys carry bit 7 clear.
                # Per element, against that element's own magnitude (reference_pick restates it)
                p = f * (mine + 128 * _real_change(ds, s).to(torch.uint8))
                self.prio.append((p, p.clone()))
                self.pending.append(self.comm.all_reduce(self.prio[-1][1], op="max",
                                                         async_op=True))
        self.prepared = True

    def start(self):
        """Snapshot this rank's delta and launch its asynchronous all-reduce (finishes any
        exchange still pending first).  pick / hot_pick wait for the priority all-reduce first
        (on the device: RCCL's stream, no host block) and zero the rows another rank wins."""
        if not self.active:
            return
        self.prepare()
        self.prepared = False
        self.exchanges += 1
        self.synced = False
        if self.prio is not None:
            for w in self.pending:
                w.wait()
            self.pending = []
        for i, (t, ds) in enumerate(zip(self.tables, self.dsum)):
            if self.prio is not None:
                p, pmax = self.prio[i]
                lose = (p != pmax) | (p == 0)        # another rank's delta wins this row
                if self.combine == "hot_pick":
                    lose &= self.pick_rows[i]
                ds.masked_fill_(lose.view((-1,) + (1,) * (ds.dim() - 1)), 0.0)
            flat = ds.view(-1)
            for lo in range(0, flat.numel(), self.bucket):
                hi = min(lo + self.bucket, flat.numel())
                self.pending.append(self.comm.all_reduce(flat[lo:hi], async_op=True))
        self.prio = None

    def finish(self):
        """Wait for the pending all-reduce (device-side wait on the current stream) and apply
        the other ranks' deltas."""
        if not self.active or not self.pending:
            return
        if self.prepared:
            raise RuntimeError("DeltaAllReduce: prepare() without start()")
        for w in self.pending:
            w.wait()
        self.pending = []
        for i, (t, s, ds, do) in enumerate(zip(self.tables, self.snap, self.dsum, self.down)):
            if self.combine == "mean":
                ds.mul_(1.0 / self.world)
            elif self.combine in ("touched_mean", "hot_pick"):
                c = self.cnt[i].clamp_min(1)
                if self.combine == "hot_pick":      # picked rows hold one rank's delta
                    c = c.masked_fill(self.pick_rows[i], 1)
                ds.div_(c.to(ds.dtype).view((-1,) + (1,) * (ds.dim() - 1)))
            elif self.combine == "hot_mean":  # contended rows averaged, the others summed
                ds[self.mean_rows[i]] *= 1.0 / self.world
            if _fused(t):
                _native("come_delta_end", t, s, ds, do)    # S += Dsum; W += Dsum - Down
            else:
                s.add_(ds)                                 # W_sync += sum_r D_r
                ds.sub_(do)                                # others' deltas
                t.add_(ds)                                 # W += sum_r D_r - D_own

    def sync(self):
        """Blocking exchange: afterwards every replica equals W_sync + sum_r D_r, bit for bit
        (nothing trained in between, so W is set to the new W_sync itself rather than to
        W + others' deltas, which differs from it by rounding)."""
        if not self.active:
            return
        self.start()
        self.finish()
        self.settle()

    def settle(self):
        """After a finish() with nothing trained since its start(): W = W_sync exactly."""
        if self.active:
            for t, s in zip(self.tables, self.snap):
                t.copy_(s)
            self.synced = True

    @property
    def busy(self):
        return bool(self.pending)

    @property
    def overlap_safe(self):
        return self.combine in self.OVERLAP_SAFE

    def bytes_per_sync(self):
        return sum(t.numel() * t.element_size() for t in self.tables)


class SparseDeltaAllReduce(object):
    """DeltaAllReduce restricted to the rows that changed on some rank (see the module docstring).
    Same start / finish / sync protocol; ``last_rows`` / ``last_bytes`` report the previous
    exchange (rows in the union, bytes all-reduced per rank)."""

    def __init__(self, tables, group=None, bucket_elems=1 << 26, comm=None, combine="sum",
                 same_start=True, force_exchange=False):
        if combine not in ("sum", "touched_mean"):
            raise ValueError("SparseDeltaAllReduce: combine must be 'sum' or 'touched_mean'")
        self.combine = combine
        self.tables = list(tables)
        self.group = group
        self.comm = comm if comm is not None else TorchComm(group)
        self.world = self.comm.world
        self.active = self.world > 1 or bool(force_exchange)  # as DeltaAllReduce
        self.bucket = int(bucket_elems)
        if self.active and same_start:  # as DeltaAllReduce: replicas start from rank 0's
            self._broadcast()
        self.snap = [t.clone() for t in self.tables] if self.active else None
        self.pending = []
        self.state = []
        self.last_rows = [0] * len(self.tables)
        self.last_bytes = 0
        self.synced = self.active and same_start

    def _broadcast(self):
        for t in self.tables:
            self.comm.broadcast(t, 0)

    def reset(self, broadcast=None):
        """As DeltaAllReduce.reset (rank 0's tables taken unless a blocking sync() left the
        replicas identical)."""
        self.finish()
        if self.active:
            if broadcast or (broadcast is None and not (self.synced and
                                                        _replicas_agree(self.comm, self.tables))):
                self._broadcast()
            for t, s in zip(self.tables, self.snap):
                s.copy_(t)
            self.synced = True

    @staticmethod
    def _flags(t, s):
        import torch
        if _fused(t) and t.shape[1] % 4 == 0:
            from . import _lib
            from ._lib import check, ptr, stream_handle
            f = torch.empty(t.shape[0], dtype=torch.uint8, device=t.device)
            check(_lib.lib().come_delta_flags(ptr(t), ptr(s), t.shape[0], t.shape[1], ptr(f),
                                              stream_handle(t.device)), "come_delta_flags")
            return f
        return (t.view(torch.int32) != s.view(torch.int32)).any(dim=1).to(torch.uint8)

    def start(self):
        if not self.active:
            return
        import torch
        self.finish()
        self.synced = False
        flags = [self._flags(t, s) for t, s in zip(self.tables, self.snap)]
        flat = torch.cat(flags)
        # union over ranks (touched_mean: the number of ranks that changed each row).
        # Blocking, and torch.nonzero below waits for the device: start() returns only after the
        # batch in flight and this flag exchange have finished, so the row-sparse form does not
        # overlap its exchange with the next batch
        self.comm.all_reduce(flat, op="sum" if self.combine == "touched_mean" else "max")
        self.state = []
        self.last_bytes = 0
        o = 0
        for i, (t, s) in enumerate(zip(self.tables, self.snap)):
            idx = torch.nonzero(flat[o:o + t.shape[0]]).view(-1)
            o += t.shape[0]
            n, d = idx.numel(), t.shape[1]
            ds = t.new_empty((n, d))
            do = t.new_empty((n, d))
            if n and _fused(t) and d % 4 == 0:
                from . import _lib
                from ._lib import check, ptr, stream_handle
                check(_lib.lib().come_delta_gather(ptr(t), ptr(s), ptr(idx), n, d, ptr(ds),
                                                   ptr(do), stream_handle(t.device)),
                      "come_delta_gather")
            elif n:
                torch.sub(t.index_select(0, idx), s.index_select(0, idx), out=ds)
                do.copy_(ds)
            fl = ds.view(-1)
            for lo in range(0, fl.numel(), self.bucket):
                hi = min(lo + self.bucket, fl.numel())
                self.pending.append(self.comm.all_reduce(fl[lo:hi], async_op=True))
            cnt = flat[o - t.shape[0]:o].index_select(0, idx) if self.combine == "touched_mean" \
                else None
            self.state.append((idx, ds, do, cnt))
            self.last_rows[i] = n
            self.last_bytes += n * d * t.element_size()

    def finish(self):
        if not self.active or not self.state:
            return
        for w in self.pending:
            w.wait()
        self.pending = []
        for t, s, (idx, ds, do, cnt) in zip(self.tables, self.snap, self.state):
            n, d = idx.numel(), t.shape[1]
            if not n:
                continue
            if cnt is not None:  # mean over the ranks that changed the row
                ds.div_(cnt.to(ds.dtype).view(-1, 1))
            if _fused(t) and d % 4 == 0:
                from . import _lib
                from ._lib import check, ptr, stream_handle
                check(_lib.lib().come_delta_scatter(ptr(t), ptr(s), ptr(idx), n, d, ptr(ds),
                                                    ptr(do), stream_handle(t.device)),
                      "come_delta_scatter")
            else:
                s.index_add_(0, idx, ds)          # W_sync += sum_r D_r
                t.index_add_(0, idx, ds - do)     # W += sum_r D_r - D_own
        self.state = []

    def sync(self):
        """Blocking exchange; every replica then equals W_sync bit for bit (as DeltaAllReduce)."""
        if not self.active:
            return
        self.start()
        touched = [st[0] for st in self.state]
        self.finish()
        for t, s, idx in zip(self.tables, self.snap, touched):
            if idx.numel():
                t.index_copy_(0, idx, s.index_select(0, idx))
        self.synced = True

    @property
    def busy(self):
        return bool(self.pending)


def reference_delta_sum(w_sync, locals_):
    """Host restatement of one sync for tests: w_sync + sum_r (w_r - w_sync)."""
    out = np.array(w_sync, np.float64, copy=True)
    for w in locals_:
        out += np.asarray(w, np.float64) - np.asarray(w_sync, np.float64)
    return out


def reference_touched_mean(w_sync, locals_):
    """Host restatement of one touched_mean sync for tests: every row gets the mean of the deltas
    of the ranks that changed it (bitwise), rows nobody changed stay."""
    s = np.asarray(w_sync, np.float32)
    out = np.array(s, np.float64, copy=True)
    tot = np.zeros(s.shape, np.float64)
    cnt = np.zeros(s.shape[0], np.int64)
    for w in locals_:
        w = np.asarray(w, np.float32)
        tot += w.astype(np.float64) - s.astype(np.float64)
        cnt += (w.view(np.int32) != s.view(np.int32)).any(axis=1)
    return out + tot / np.maximum(cnt, 1)[:, None]


def reference_pick(w_sync, locals_, star):
    """Host restatement of one pick sync for tests: a row changed (bitwise) by some rank takes
    the delta of the first rank in the order star, star + 1, ... (mod N) that changed it by more
    than rounding (_real_change), else of the first that changed it at all; rows nobody changed
    stay."""
    s = np.asarray(w_sync, np.float32)
    out = np.array(s, np.float64, copy=True)
    n = len(locals_)
    done = np.zeros(s.shape[0], bool)
    for real_only in (True, False):
        for j in range(n):
            w = np.asarray(locals_[(star + j) % n], np.float32)
            ch = (w.view(np.int32) != s.view(np.int32)).any(axis=1) & ~done
            if real_only:
                ch &= _real_change(w - s, s)
            out[ch] += w[ch].astype(np.float64) - s[ch].astype(np.float64)
            done |= ch
    return out

