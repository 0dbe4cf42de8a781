"""ctypes binding of libcome.so (the C-ABI in include/come.h).

The HIP library is the only compute path: if it is missing or fails to load, every entry point
raises -- there is no CPU fallback on the product path.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# COME_LIB_PATH: an alternative in-tree build of the same library (A/B experiments only)
DEFAULT_LIB_PATH = os.path.join(HERE, "libcome.so")
LIB_PATH = os.environ.get("COME_LIB_PATH") or DEFAULT_LIB_PATH

MODE_HOGWILD = 0
MODE_SEQUENTIAL = 1
TABLE_PACKED = 0x100  # COME_TABLE_PACKED mode flag
HOT_NONE = 0x200      # COME_HOT_NONE mode flag
ABI_VERSION = 5       # COME_ABI_VERSION this binding is written for

# Every symbol include/come.h declares (checked by tests/test_capi.py).
SYMBOLS = ("come_abi_version", "come_last_error", "come_init", "come_exp_table",
           "come_fast_version", "come_sgns_o2", "come_sgns_o1", "come_community_grad",
           "come_gmm_resp", "come_make_table", "come_count_o2_pairs", "come_set_option",
           "come_random_walks", "come_walks_reference", "come_pyrandom_seed",
           "come_pyrandom_draw", "come_np_draw_seeds", "come_graph_from_edges",
           "come_read_int_rows",
           "come_write_int_rows", "come_save_embedding", "come_format_f32",
           "come_gmm_estep", "come_gmm_scatter", "come_gmm_params", "come_pack_table",
           "come_delta_begin", "come_delta_end", "come_get_options", "come_sgns_o2_ex",
           "come_sgns_o1_ex", "come_hot_rows", "come_lcg_table_draws", "come_delta_flags",
           "come_delta_gather", "come_delta_scatter", "come_cpu_sgns_o2", "come_cpu_sgns_o1",
           "come_cpu_community_grad", "come_cpu_gmm_resp", "come_cpu_gmm_estep",
           "come_source_sha256")

OPTION_FIELDS = ("o2_kernel", "o2_blocks_per_cu", "o2_waves_per_block",
                 "o2_static", "rows_per_wave", "o1_rows_per_wave",
                 "max_waves", "o1_blocks_per_cu", "resident_cap", "community_async",
                 "gmm_cov_async", "walk_staged", "o2_fresh_loads", "o2_atomic_writeback",
                 "gmm_resp16", "o1_chunk")


class LaunchOpts(ctypes.Structure):
    """come_launch_opts (include/come.h): per-call launch options of the *_ex entry points."""
    _fields_ = [(f, ctypes.c_int) for f in OPTION_FIELDS] + [("o2_update_count",
                                                             ctypes.c_void_p)]

_lib = None


def source_sha256():
    """SHA-256 of the sources libcome.so is built from, as the Makefile stamps it (csrc/*.hip,
    *.cpp, *.h in name order, then the Makefile and include/come.h); None without the sources."""
    import hashlib
    csrc = os.path.join(HERE, "csrc")
    header = os.path.join(os.path.dirname(HERE), "include", "come.h")
    if not os.path.isdir(csrc) or not os.path.exists(header):
        return None
    names = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".cpp", ".h")))
    h = hashlib.sha256()
    for f in [os.path.join(csrc, n) for n in names] + [os.path.join(csrc, "Makefile"), header]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


class ComeError(RuntimeError):
    pass


def build():
    """Compile libcome.so in-tree with hipcc (gfx950)."""
    import subprocess
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "csrc"), "-j4"])


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ComeError("libcome.so not found at %s -- build it with "
                        "`make -C nodeembedding-to-communityembedding_amd/csrc` or "
                        "`python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)
    # torch first: it ships its own HIP runtime, and libcome.so must bind to that same instance
    # (loaded first, libcome would pull /opt/rocm's copy and torch would then see no device)
    import torch  # noqa: F401
    L = ctypes.CDLL(LIB_PATH)
    P, i32, i64, u64, f32, f64 = (ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64,
                                  ctypes.c_float, ctypes.c_double)
    L.come_abi_version.restype = i32
    L.come_source_sha256.restype = ctypes.c_char_p
    L.come_last_error.restype = ctypes.c_char_p
    L.come_init.argtypes = [i32]
    L.come_exp_table.argtypes = [P]
    L.come_exp_table.restype = None
    L.come_sgns_o2.argtypes = [P, P, i64, i32, P, i64, i32, P, i32, i32, P, u64, f32, f32, i32, P]
    L.come_sgns_o1.argtypes = [P, i64, i32, P, i64, P, i32, P, u64, f32, i32, P]
    L.come_community_grad.argtypes = [P, i64, i32, P, P, P, i32, f32, f32, i32, P]
    L.come_gmm_resp.argtypes = [P, i64, i32, P, P, P, i32, P, P]
    L.come_pack_table.argtypes = [P, u64, P, P, P]
    L.come_delta_begin.argtypes = [P, P, P, P, i64, P]
    L.come_delta_end.argtypes = [P, P, P, P, i64, P]
    L.come_gmm_estep.argtypes = [P, i64, i32, P, P, P, i32, P, P, P]
    L.come_gmm_scatter.argtypes = [P, i64, i32, P, P, i32, i32, P, P, P]
    L.come_gmm_params.argtypes = [P, P, P, P, i32, i32, f64, P, P, P, P, P, P, P]
    L.come_make_table.argtypes = [P, i64, P, u64, f64]
    L.come_count_o2_pairs.argtypes = [P, i64, i32, i32]
    L.come_count_o2_pairs.restype = i64
    L.come_set_option.argtypes = [ctypes.c_char_p, i32]
    L.come_get_options.argtypes = [P]
    L.come_sgns_o2_ex.argtypes = [P, P, i64, i32, P, i64, i32, P, i32, i32, P, u64, f32, f32, i32,
                                  P, P, P]
    L.come_hot_rows.argtypes = [P, u64, i64, u64, P, P, P]
    L.come_lcg_table_draws.argtypes = [u64, i64, P, u64, P]
    L.come_delta_flags.argtypes = [P, P, i64, i32, P, P]
    L.come_delta_gather.argtypes = [P, P, P, i64, i32, P, P, P]
    L.come_delta_scatter.argtypes = [P, P, P, i64, i32, P, P, P]
    L.come_sgns_o1_ex.argtypes = [P, i64, i32, P, i64, P, i32, P, u64, f32, i32, P, P, P]
    L.come_cpu_sgns_o2.argtypes = [P, P, i64, i32, P, i64, i32, P, i32, i32, P, u64, f32, f32,
                                   i32, i32, P]
    L.come_cpu_sgns_o1.argtypes = [P, i64, i32, P, i64, P, i32, P, u64, f32, i32, i32, P]
    L.come_cpu_community_grad.argtypes = [P, i64, i32, P, P, P, i32, f32, f32, i32, i32]
    L.come_cpu_gmm_resp.argtypes = [P, i64, i32, P, P, P, i32, P, i32]
    L.come_cpu_gmm_estep.argtypes = [P, i64, i32, P, P, P, i32, P, P, i32]
    cp = ctypes.c_char_p
    L.come_random_walks.argtypes = [P, P, i64, P, i64, i32, f32, u64, i64, P, P, P]
    L.come_walks_reference.argtypes = [P, P, i64, i32, P, P, i32, f64, P, i32, P]
    L.come_pyrandom_seed.argtypes = [u64, P]
    L.come_pyrandom_draw.argtypes = [P, i32, u64, i64, P]
    L.come_np_draw_seeds.argtypes = [P, i64, P]
    L.come_graph_from_edges.argtypes = [P, i64, P, P, P, P, P, P, P]
    L.come_read_int_rows.argtypes = [cp, P, i64, i32, P, P]
    L.come_write_int_rows.argtypes = [cp, P, i64, i32, i32]
    L.come_save_embedding.argtypes = [cp, P, i64, i32, i64]
    L.come_format_f32.argtypes = [f32, cp]
    if L.come_abi_version() != ABI_VERSION:
        raise ComeError("libcome.so ABI version %d, this binding needs %d (rebuild the library)"
                        % (L.come_abi_version(), ABI_VERSION))
    want = source_sha256()
    if want is not None and LIB_PATH == DEFAULT_LIB_PATH:
        got = L.come_source_sha256().decode()
        if got != want:
            raise ComeError("%s was built from other sources (stamp %s, the sources beside it "
                            "hash to %s): rebuild it with `make -C %s`" % (
                                LIB_PATH, got[:12], want[:12], os.path.join(HERE, "csrc")))
    _lib = L
    return L


def check(rc, what):
    if rc != 0:
        msg = lib().come_last_error().decode(errors="replace")
        raise ComeError("%s failed (rc=%d): %s" % (what, rc, msg))


def ptr(t):
    """Raw address of a torch tensor or numpy array (no torch types cross the C-ABI)."""
    if hasattr(t, "data_ptr"):
        return ctypes.c_void_p(t.data_ptr())
    return t.ctypes.data_as(ctypes.c_void_p)


def stream_handle(device=None):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def set_option(name, value):
    """Process-wide launch option (see include/come.h come_set_option)."""
    check(lib().come_set_option(name.encode(), int(value)), "come_set_option(%s)" % name)


def launch_opts(update_count=None, **overrides):
    """A LaunchOpts holding the current process-wide options with `overrides` applied, and
    o2_update_count = the address of `update_count` (a CUDA int64 tensor of one element)."""
    o = LaunchOpts()
    check(lib().come_get_options(ctypes.byref(o)), "come_get_options")
    for k, v in overrides.items():
        if k not in OPTION_FIELDS:
            raise ValueError("unknown launch option %r" % k)
        setattr(o, k, int(v))
    if update_count is not None:
        o.o2_update_count = update_count.data_ptr()
    return o
