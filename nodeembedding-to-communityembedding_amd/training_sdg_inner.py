"""Drop-in for the reference's Cython module ``utils/training_sdg_inner.pyx``.

Same names and argument meaning as the reference:

    train_o1(py_node_embedding, py_edge, py_lr, py_negative, py_table, py_size=None, py_work=None)
        -> int                                                          (pyx:407-450)
    train_o2(py_node_embedding, py_context_embedding, py_path, py_lr, py_negative, py_window,
             py_table, py_alpha=1.0, py_size=None, py_work=None) -> int (pyx:454-509)
    init() -> int, FAST_VERSION                                         (pyx:512-549)

Like the reference they mutate the embedding tables IN PLACE and draw each call's initial
``next_random`` from the global numpy RNG (2 draws, pyx:427,477), and they are re-entrant: the
reference's worker threads may call them concurrently.  The tables may be CUDA tensors (the
kernels, on the current stream, no copies) or numpy arrays (libcome's host twin, in place, the GIL
released as the reference's ``nogil`` block releases it); see "per-call drop-ins" below.
``py_size`` and ``py_work`` are accepted and ignored (the work vector lives in registers).

The batched entry points ``sgns_o2`` / ``sgns_o1`` take whole batches of walks / edges already on
the device and are what the trainers (Context2Vec / Node2Vec) call: one launch per batch instead
of one Python call per walk.
"""
import ctypes
import threading

import numpy as np

from . import _lib
from ._lib import (HOT_NONE, MODE_HOGWILD, MODE_SEQUENTIAL, TABLE_PACKED, check, ptr,
                   stream_handle)

FAST_VERSION = 0
MAX_SENTENCE_LEN = 10000
_SEED_LOCK = threading.Lock()


def init():
    """Returns FAST_VERSION (pyx:512-549).  The sigmoid table is uploaded per device by the
    library on first use (come_init)."""
    return _lib.lib().come_fast_version()


def exp_table():
    """The reference's EXP_TABLE (pyx:531-533) as a float32 numpy array of 1000 entries."""
    out = np.zeros(1000, np.float32)
    _lib.lib().come_exp_table(ptr(out))
    return out


def draw_seeds(n, out=None):
    """Initial next_random of n consecutive train_o1/train_o2 calls, drawn from the global numpy
    RNG exactly as pyx:427/477 does per call: 2^24 * randint(0, 2^24) + randint(0, 2^24).
    The stream is generated natively (come_np_draw_seeds: numpy's legacy MT19937, ~10 ms per 1M
    calls instead of numpy's 56 ms -- the host cost of every O1 pass and O2 batch) from
    np.random.get_state(), and the global state is advanced with set_state() exactly as numpy's
    own 2n randint draws would leave it (tests/test_host.py)."""
    n = int(n)
    if n == 0:
        return np.zeros(0, np.uint64)
    if out is not None and (out.dtype != np.uint64 or out.shape != (n,) or
                            not out.flags["C_CONTIGUOUS"]):
        raise ValueError("out must be a contiguous uint64 array of %d seeds" % n)
    with _SEED_LOCK:  # get_state -> native draws (GIL released) -> set_state is one step
        st = np.random.get_state()
        if st[0] != "MT19937":  # pragma: no cover (the legacy global RNG is always MT19937)
            ab = np.random.randint(0, 2 ** 24, size=2 * n).astype(np.uint64)
            return (ab[0::2] << np.uint64(24)) + ab[1::2]
        state = np.empty(625, np.uint32)
        state[:624] = st[1]
        state[624] = st[2]
        out = np.empty(n, np.uint64) if out is None else out
        check(_lib.lib().come_np_draw_seeds(ptr(state), n, ptr(out)), "come_np_draw_seeds")
        np.random.set_state((st[0], state[:624].copy(), int(state[624]), st[3], st[4]))
    return out


def _require_cuda(t, name, dtype):
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError("%s must be a CUDA tensor" % name)
    if t.dtype != dtype:
        raise TypeError("%s must be %s (got %s)" % (name, dtype, t.dtype))
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % name)


class PackedTable(object):
    """Exact 16x smaller device form of a negative table (come_pack_table): ``words`` is a CUDA
    int32 tensor [ceil(T/64), 4], ``T`` the number of slots.  Accepted wherever a table is."""

    def __init__(self, words, T):
        self.words, self.T = words, int(T)


def pack_table(table):
    """Pack a CUDA uint32-as-int32 table [T]; returns a PackedTable, or None if some step inside
    a 64-slot word is not 0 or 1 (then keep using the plain table)."""
    import torch
    _require_cuda(table, "table", torch.int32)
    T = table.numel()
    words = torch.empty(((T + 63) // 64, 4), dtype=torch.int32, device=table.device)
    status = torch.empty(1, dtype=torch.int32, device=table.device)
    check(_lib.lib().come_pack_table(ptr(table), T, ptr(words), ptr(status),
                                     stream_handle(table.device)), "come_pack_table")
    return PackedTable(words, T) if int(status.item()) == 0 else None


def _table_args(table):
    """(pointer, T, mode flag) for a plain CUDA table tensor or a PackedTable."""
    import torch
    if isinstance(table, PackedTable):
        return ptr(table.words), table.T, TABLE_PACKED
    _require_cuda(table, "table", torch.int32)
    return ptr(table), table.numel(), 0


def _opts_arg(opts, update_count=None):
    """ctypes argument for the *_ex entry points: None (process-wide options) or a LaunchOpts."""
    import ctypes
    if opts is None and update_count is None:
        return None
    if update_count is not None:
        import torch
        _require_cuda(update_count, "update_count", torch.int64)
    o = _lib.launch_opts(update_count, **(opts or {}))
    return ctypes.byref(o)


# Rows holding at least this share of the negative table are "hot" (contended in Hogwild mode,
# see come_hot.hip): updated by float-atomic deltas, so no concurrent update of theirs is lost.
# d <= 128 (C2, C3): measured (scripts/diag_tierc.py, profiles/r02_ab_hot_threshold.txt) on C3's
# shape at 100k nodes the held-out loss is 0.81% / 0.11% above the sequential oracle's at shares
# 1e-5 / 5e-6; at C3 (1M nodes) 5e-6 marks 10k rows and costs no time vs 1e-5; lower shares cost
# time there without bringing the bench launch closer to the oracle (1e-6: -0.68% vs -0.80%,
# +19% time; profiles/r06_hot_share.txt).
# d > 128 (C5's kernel, d = 256, n = 10): on a 1M-node graph of C5's generator the plain stores of
# rows between 8e-7 and 5e-6 of the table lose enough concurrent updates (every update of such a
# row races ~0.1-0.2 others in flight) to train 1.8% BELOW the sequential oracle, outside tier C;
# 8e-7 lands at -0.40% (+15% launch time on that graph) and leaves C5 itself unchanged (+0.47%
# -> +0.50%, launch time within 1%); making every row atomic overshoots (+1.5%: stale deltas of
# thousands of wavefronts summed).  profiles/r06_hot_share.txt.
DEFAULT_HOT_P = 5e-6
DEFAULT_HOT_P_WIDE = 8e-7


def default_hot_share(d):
    """The contended-row share the product uses for rows of width d (COME_DEFAULT_HOT_SHARE /
    _WIDE in come.h)."""
    return DEFAULT_HOT_P if int(d) <= 128 else DEFAULT_HOT_P_WIDE


def hot_rows(table, V, min_count):
    """Bitmap (CUDA int32 tensor [ceil(V/32)]) of the rows holding >= min_count slots of the
    negative table `table` (CUDA uint32-as-int32 [T]): come_hot_rows."""
    import torch
    _require_cuda(table, "table", torch.int32)
    counts = torch.empty(int(V), dtype=torch.int32, device=table.device)
    bits = torch.empty((int(V) + 31) // 32, dtype=torch.int32, device=table.device)
    check(_lib.lib().come_hot_rows(ptr(table), table.numel(), int(V), int(min_count), ptr(counts),
                                   ptr(bits), stream_handle(table.device)), "come_hot_rows")
    return bits


def _hot_arg(hot, node, V):
    """(pointer, mode flag) for the contended-row argument: "auto" -> NULL (libcome derives the
    bitmap from the table at default_hot_share(d)), None -> COME_HOT_NONE (every row cold), else a CUDA
    int32 bitmap of at least ceil(V / 32) words on the tables' device."""
    import torch
    if isinstance(hot, str):
        if hot != "auto":
            raise ValueError("hot must be a bitmap tensor, None or 'auto'")
        return None, 0
    if hot is None:
        return None, HOT_NONE
    _require_cuda(hot, "hot", torch.int32)
    if hot.device != node.device:
        raise ValueError("hot must be on the tables' device (%s, got %s)" % (node.device,
                                                                            hot.device))
    if hot.numel() < (int(V) + 31) // 32:
        raise ValueError("hot bitmap has %d words, needs ceil(V/32) = %d" % (
            hot.numel(), (int(V) + 31) // 32))
    return ptr(hot), 0


def sgns_o2(node, ctx, walks, seeds, window, negative, table, lr, alpha=1.0, mode=MODE_HOGWILD,
            opts=None, update_count=None, hot="auto"):
    """Batched train_o2: every walk of ``walks`` [P, L] (int32 rows, -1 = None) in one launch.

    node, ctx: float32 CUDA tensors [V, d], updated in place.  seeds: uint64 (stored as int64)
    CUDA tensor [P].  table: uint32 (stored as int32) CUDA tensor [T].  mode: MODE_HOGWILD (all
    walks in flight, one wavefront each) or MODE_SEQUENTIAL (walks in order: workers=1).  table
    may also be a PackedTable (same draws, 16x less table traffic).  opts: per-call launch
    options (dict of come_launch_opts fields, see include/come.h); update_count: CUDA int64
    tensor [1] that the launch adds its number of applied target-row updates to; hot: the
    contended-row bitmap of hot_rows() (Hogwild mode: those rows are read per pair and updated
    with float atomics), "auto" (default: derived from `table` by the library at default_hot_share(d)
    before EVERY launch, ~0.1 ms at T = 1e8 -- callers launching many small batches pass
    Model.hot_rows() instead, as the trainers do) or None (no contended rows: every row updated
    with plain stores)."""
    import torch
    _require_cuda(node, "node", torch.float32)
    _require_cuda(ctx, "ctx", torch.float32)
    _require_cuda(walks, "walks", torch.int32)
    _require_cuda(seeds, "seeds", torch.int64)
    tp, T, flag = _table_args(table)
    if node.shape != ctx.shape or node.dim() != 2:
        raise ValueError("node and ctx must both be [V, d]")
    if walks.dim() != 2 or seeds.shape != (walks.shape[0],):
        raise ValueError("walks must be [P, L] and seeds [P]")
    if walks.shape[1] > MAX_SENTENCE_LEN:  # pyx:480 truncates silently; so do we
        walks = walks[:, :MAX_SENTENCE_LEN].contiguous()
    V, d = node.shape
    hp, hflag = _hot_arg(hot, node, V)
    rc = _lib.lib().come_sgns_o2_ex(ptr(node), ptr(ctx), V, d, ptr(walks), walks.shape[0],
                                    walks.shape[1], ptr(seeds), int(window), int(negative),
                                    tp, T, float(lr), float(alpha), int(mode) | flag | hflag,
                                    hp, _opts_arg(opts, update_count),
                                    stream_handle(node.device))
    check(rc, "come_sgns_o2")


def sgns_o1(node, edges, seeds, negative, table, lr, mode=MODE_HOGWILD, opts=None, hot="auto"):
    """Batched train_o1 over ``edges`` [E, 2] (int32 rows) in one launch; node updated in place.
    opts: per-call launch options (dict of come_launch_opts fields); hot: contended-row bitmap
    (hot_rows(); Hogwild: updates of those rows are float-atomic deltas), "auto" or None as for
    sgns_o2."""
    import torch
    _require_cuda(node, "node", torch.float32)
    _require_cuda(edges, "edges", torch.int32)
    _require_cuda(seeds, "seeds", torch.int64)
    tp, T, flag = _table_args(table)
    if edges.dim() != 2 or edges.shape[1] != 2 or seeds.shape != (edges.shape[0],):
        raise ValueError("edges must be [E, 2] and seeds [E]")
    V, d = node.shape
    hp, hflag = _hot_arg(hot, node, V)
    rc = _lib.lib().come_sgns_o1_ex(ptr(node), V, d, ptr(edges), edges.shape[0], ptr(seeds),
                                    int(negative), tp, T, float(lr), int(mode) | flag | hflag,
                                    hp, _opts_arg(opts), stream_handle(node.device))
    check(rc, "come_sgns_o1")


def count_o2_pairs(walks_np, window):
    """Number of pair updates (fast_o2 calls) train_o2 makes over host walks [P, L]."""
    w = np.ascontiguousarray(walks_np, np.int32)
    if w.ndim != 2 or w.size == 0:
        return 0
    return int(_lib.lib().come_count_o2_pairs(ptr(w), w.shape[0], w.shape[1], int(window)))


# ---- per-call drop-ins (reference signatures) -------------------------------------------------
#
# The reference's callers run train_o2 / train_o1 from `workers` Python threads at once, each call
# releasing the GIL around its update loop (pyx:443,493; context_embeddings.py:72-98,
# node_embeddings.py:58-83): calls must be re-entrant, and updates of one call must not undo
# another's.  Where the tables live decides the route:
#   * host route (every table a numpy array, the reference's own case): the call runs libcome's
#     host twin come_cpu_sgns_o2 / _o1 in sequential mode on the caller's arrays, in place, through
#     ctypes (which drops the GIL, as the reference's `nogil` block does).  Concurrent calls race
#     per element exactly like the reference's threads; nothing is copied.
#   * device route (any table a CUDA tensor): the kernels, on the caller's current stream.  numpy
#     tables among the arguments go through cached device mirrors, and the whole
#     upload -> launch -> writeback sequence of such a call holds _DEVICE_LOCK, so no other call's
#     upload or writeback lands in between (a call that only has CUDA tensors takes no lock).
# set_numpy_route("device") sends all-numpy calls down the device route as well (serialised by
# the lock; see INTEGRATION.md for what each route costs).

_DEVICE_LOCK = threading.Lock()
_NUMPY_ROUTE = ["host"]


def set_numpy_route(route):
    """Where calls whose tables are all numpy arrays run: "host" (default: libcome's host twin on
    the arrays in place) or "device" (the kernels through device mirrors, serialised)."""
    if route not in ("host", "device"):
        raise ValueError("route must be 'host' or 'device'")
    prev, _NUMPY_ROUTE[0] = _NUMPY_ROUTE[0], route
    return prev


_PYEXT = []


def _pyext():
    """The host route's CPython extension (_come_pyext, csrc/come_pyext.c), bound on first use to
    libcome's host twins; raises if it is not built (no slower Python stand-in)."""
    if _PYEXT:
        return _PYEXT[0]
    with _SEED_LOCK:
        if not _PYEXT:
            try:
                from . import _come_pyext as ext
            except ImportError as e:
                raise _lib.ComeError("_come_pyext is not built (%s): run `make -C "
                                     "nodeembedding-to-communityembedding_amd/csrc`" % e)
            L = _lib.lib()
            addr = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
            ext.init(addr(L.come_cpu_sgns_o2), addr(L.come_cpu_sgns_o1), addr(L.come_last_error),
                     np.random.randint)
            _PYEXT.append(ext)
    return _PYEXT[0]


def _call_seed():
    """One call's initial next_random, drawn as pyx:427/477 draws it (two global-RNG draws)."""
    return (1 << 24) * int(np.random.randint(0, 1 << 24)) + int(np.random.randint(0, 1 << 24))


def _rows_of(items):
    """Vocab objects (or None) -> int32 rows, -1 for None (codelens 0, pyx:483-490)."""
    return np.array([-1 if it is None else int(it.index) for it in items], np.int32)


def _host_table_arg(arr, name):
    """A float32 [V, d] numpy embedding table for the host route, used in place."""
    if not (isinstance(arr, np.ndarray) and arr.dtype == np.float32 and arr.ndim == 2 and
            arr.flags.c_contiguous and arr.flags.writeable):
        raise TypeError("%s must be a writable C-contiguous float32 [V, d] numpy array or a CUDA "
                        "tensor" % name)
    return arr


def _host_neg_table(table):
    """The negative table as contiguous uint32 (the reference reads it as np.uint32_t *,
    pyx:421,472); an int32 array is viewed, other integer arrays are converted (a copy)."""
    t = np.asarray(table)
    if t.dtype == np.int32:
        t = t.view(np.uint32)
    if t.dtype != np.uint32 or not t.flags.c_contiguous:
        t = np.ascontiguousarray(t, np.uint32)
    return t


class _Mirrors(object):
    """Device mirrors of the numpy arrays handed to device-route calls (used under _DEVICE_LOCK).

    Copying whole tables per call (400 MB for a 1e8-slot negative table, V x d per embedding
    table) would make every call O(V + T), so:
      * a numpy embedding table gets ONE device buffer of its shape, kept across calls (keyed by
        the array's buffer address, shape and dtype) and never uploaded whole: each call uploads
        exactly the rows it can touch and downloads the same rows afterwards (rows outside the
        call are not read by the kernel, so their device contents do not matter);
      * a numpy negative table is uploaded once and kept, keyed by buffer address and size and
        re-checked per call against a fingerprint of 64 strided entries plus both ends (the
        reference never mutates it after make_table, model.py:97-122; a table rewritten in place
        with the same fingerprint is not detected -- pass a new array instead).
    Per-call cost is O(rows a walk / edge can touch), independent of V and T."""

    def __init__(self):
        self.tables = {}
        self.neg = {}

    def table(self, arr, device):
        import torch
        key = (arr.__array_interface__["data"][0], arr.shape, arr.dtype.str, str(device))
        t = self.tables.get(key)
        if t is None:
            if len(self.tables) >= 16:  # bounded: a long-running caller cycling arrays
                self.tables.clear()
            t = self.tables[key] = torch.empty(arr.shape, dtype=torch.float32, device=device)
        return t

    @staticmethod
    def _fingerprint(arr):
        idx = np.linspace(0, len(arr) - 1, 64).astype(np.int64)
        return arr[idx].tobytes()

    def negative_table(self, arr, device):
        import torch
        key = (arr.__array_interface__["data"][0], arr.shape[0], str(device))
        fp = self._fingerprint(arr)
        hit = self.neg.get(key)
        if hit is None or hit[0] != fp:
            if len(self.neg) >= 4:
                self.neg.clear()
            hit = self.neg[key] = (fp, torch.from_numpy(arr.view(np.int32)).to(device))
        return hit[1]


_MIRRORS = _Mirrors()


def _device_of(*arrays):
    import torch
    for a in arrays:
        if isinstance(a, torch.Tensor):
            if not a.is_cuda:
                raise TypeError("tables must be CUDA tensors or numpy arrays")
            return a.device
    return torch.device("cuda", torch.cuda.current_device())


def _is_tensor(a):
    import torch
    return isinstance(a, torch.Tensor)


def _resolve_table(py_table, device):
    """The negative table as a CUDA int32 tensor and as host uint32 numpy (None when it is a
    tensor: then the touched rows are not computed on the host)."""
    import torch
    if isinstance(py_table, torch.Tensor):
        t = py_table if py_table.dtype == torch.int32 else py_table.view(torch.int32)
        return t.to(device), None
    host = _host_neg_table(py_table)
    return _MIRRORS.negative_table(host, device), host


def _draw_rows(seed, count, host_table):
    """Rows of `count` consecutive negative draws from `seed` (come_lcg_table_draws)."""
    out = np.empty(int(count), np.uint32)
    if count:
        check(_lib.lib().come_lcg_table_draws(int(seed), int(count), ptr(host_table),
                                              host_table.shape[0], ptr(out)),
              "come_lcg_table_draws")
    return out.astype(np.int64)


class _Borrowed(object):
    """One reference-style table argument for one device-route call: a CUDA tensor is used as
    is; a numpy array goes through its device mirror, `rows` up before the launch and down after
    it (the caller holds _DEVICE_LOCK)."""

    def __init__(self, arr, device, rows):
        import torch
        self.arr = arr
        if isinstance(arr, torch.Tensor):
            self.dev, self.rows = arr, None
            return
        _host_table_arg(arr, "embedding table")
        self.dev = _MIRRORS.table(arr, device)
        r = np.unique(rows)
        self.rows = r[(r >= 0) & (r < arr.shape[0])]
        if len(self.rows):
            ri = torch.from_numpy(self.rows).to(device)
            self.ridx = ri
            self.dev.index_copy_(0, ri, torch.from_numpy(arr[self.rows]).to(device))

    def writeback(self):
        if self.rows is not None and len(self.rows):
            self.arr[self.rows] = self.dev.index_select(0, self.ridx).cpu().numpy()


def _host_o2(node, ctx, rows, nr, lr, negative, window, table, alpha):
    _host_table_arg(node, "py_node_embedding")
    _host_table_arg(ctx, "py_context_embedding")
    if node.shape != ctx.shape:
        raise ValueError("node and context embeddings must have the same shape")
    tab = _host_neg_table(table)
    seed = ctypes.c_uint64(nr)
    check(_lib.lib().come_cpu_sgns_o2(node.ctypes.data, ctx.ctypes.data, node.shape[0],
                                      node.shape[1], rows.ctypes.data, 1, rows.shape[0],
                                      ctypes.byref(seed), int(window), int(negative),
                                      tab.ctypes.data, tab.shape[0], float(lr), float(alpha),
                                      MODE_SEQUENTIAL, 1, None), "come_cpu_sgns_o2")


def _device_o2(node_in, ctx_in, rows, nr, lr, negative, window, table_in, alpha):
    import torch
    device = _device_of(node_in, ctx_in, table_in)
    table, host_table = _resolve_table(table_in, device)
    walk_rows = rows[rows >= 0].astype(np.int64)
    ctx_rows = walk_rows
    if not _is_tensor(ctx_in):  # positives are walk rows; negatives come from this call's draws
        if host_table is None:
            host_table = table.cpu().numpy().view(np.uint32)
        pairs = count_o2_pairs(rows.reshape(1, -1), window)
        ctx_rows = np.concatenate([walk_rows, _draw_rows(nr, pairs * int(negative),
                                                         host_table)])
    node = _Borrowed(node_in, device, walk_rows)
    ctx = _Borrowed(ctx_in, device, ctx_rows)
    walks = torch.from_numpy(rows.reshape(1, -1)).to(device)
    seeds = torch.from_numpy(np.array([nr], np.uint64).view(np.int64)).to(device)
    sgns_o2(node.dev, ctx.dev, walks, seeds, window, negative, table, lr, alpha, MODE_SEQUENTIAL)
    node.writeback()
    ctx.writeback()


def _route(*args):
    """"host", "device" (CUDA tensors only: no lock needed) or "locked" (device route with numpy
    arguments mirrored: under _DEVICE_LOCK)."""
    tensors = [_is_tensor(a) for a in args]
    if all(tensors):
        return "device"
    if any(tensors) or _NUMPY_ROUTE[0] == "device":
        return "locked"
    return "host"


def train_o2(py_node_embedding, py_context_embedding, py_path, py_lr, py_negative, py_window,
             py_table, py_alpha=1.0, py_size=None, py_work=None):
    """One walk (pyx:454-509).  Returns the number of non-None entries.  numpy tables are updated
    in place by libcome's host twin (re-entrant: the reference's worker threads may call it
    concurrently); CUDA tensors by the kernel on the current stream (see the routes above)."""
    if (type(py_node_embedding) is np.ndarray and type(py_context_embedding) is np.ndarray and
            type(py_table) is np.ndarray and _NUMPY_ROUTE[0] == "host"):
        try:  # the reference's own case, in C: seeds, path rows, the twin with the GIL released
            return _pyext().train_o2(py_node_embedding, py_context_embedding, py_path, py_lr,
                                     py_negative, py_window, py_table, py_alpha)
        except TypeError:  # raised before the RNG draw: e.g. a non-uint32 table, converted below
            pass
    nr = _call_seed()  # pyx:477: two draws from the global numpy RNG, per call
    rows = _rows_of(py_path[:MAX_SENTENCE_LEN] if isinstance(py_path, (list, tuple))
                    else list(py_path)[:MAX_SENTENCE_LEN])
    result = int((rows >= 0).sum())
    if not rows.size:
        return result
    args = (py_node_embedding, py_context_embedding, rows, nr, py_lr, py_negative, py_window,
            py_table, py_alpha)
    route = _route(py_node_embedding, py_context_embedding, py_table)
    if route == "host":
        _host_o2(*args)
    elif route == "device":
        _device_o2(*args)
    else:
        with _DEVICE_LOCK:
            _device_o2(*args)
    return result


def _host_o1(node, rows, nr, lr, negative, table):
    _host_table_arg(node, "py_node_embedding")
    tab = _host_neg_table(table)
    seed = ctypes.c_uint64(nr)
    check(_lib.lib().come_cpu_sgns_o1(node.ctypes.data, node.shape[0], node.shape[1],
                                      rows.ctypes.data, 1, ctypes.byref(seed), int(negative),
                                      tab.ctypes.data, tab.shape[0], float(lr), MODE_SEQUENTIAL,
                                      1, None), "come_cpu_sgns_o1")


def _device_o1(node_in, rows, nr, lr, negative, table_in):
    import torch
    device = _device_of(node_in, table_in)
    table, host_table = _resolve_table(table_in, device)
    touched = rows[rows >= 0].astype(np.int64)
    if not _is_tensor(node_in):
        if host_table is None:
            host_table = table.cpu().numpy().view(np.uint32)
        touched = np.concatenate([touched, _draw_rows(nr, 2 * int(negative), host_table)])
    node = _Borrowed(node_in, device, touched)
    edges = torch.from_numpy(rows.reshape(1, 2)).to(device)
    seeds = torch.from_numpy(np.array([nr], np.uint64).view(np.int64)).to(device)
    sgns_o1(node.dev, edges, seeds, negative, table, lr, MODE_SEQUENTIAL)
    node.writeback()


def train_o1(py_node_embedding, py_edge, py_lr, py_negative, py_table, py_size=None, py_work=None):
    """One edge (pyx:407-450): pairs (edge[0] -> edge[1]) then (edge[1] -> edge[0]).  Returns the
    number of non-None endpoints.  Routes as train_o2 (numpy: the host twin in place; CUDA
    tensors: the kernel)."""
    if (type(py_node_embedding) is np.ndarray and type(py_table) is np.ndarray and
            _NUMPY_ROUTE[0] == "host"):
        try:
            return _pyext().train_o1(py_node_embedding, py_edge, py_lr, py_negative, py_table)
        except TypeError:
            pass
    nr = _call_seed()  # pyx:427
    rows = _rows_of(list(py_edge)[:2])
    result = int((rows >= 0).sum())
    if rows.size != 2:
        return result
    args = (py_node_embedding, rows, nr, py_lr, py_negative, py_table)
    route = _route(py_node_embedding, py_table)
    if route == "host":
        _host_o1(*args)
    elif route == "device":
        _device_o1(*args)
    else:
        with _DEVICE_LOCK:
            _device_o1(*args)
    return result
