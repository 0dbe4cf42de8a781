// come_host.cpp -- host side of libcome.so: error reporting, per-device init, the reference's
// EXP_TABLE, the exact make_table, pair counting.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stddef.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <algorithm>
#include <mutex>
#include <unordered_map>

#include "come_internal.h"

extern "C" int come_upload_exp_table(const float *host1000);  // come_sgns.hip

namespace come {

static thread_local char g_err[512] = "";

int set_error(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int hip_error(hipError_t e, const char *what) {
    if (e == hipSuccess) return COME_OK;
    return set_error(COME_E_HIP, "%s: %s", what, hipGetErrorString(e));
}

static constexpr int kMaxDevices = 64;
static std::once_flag g_once[kMaxDevices];
static int g_init_rc[kMaxDevices];
static int g_cus[kMaxDevices];

// Work-queue counters for dynamically scheduled launches: a ring of kCounterSlots int64 per
// device, allocated once at init; each launch takes the next slot (a launch only touches its own
// slot, so up to kCounterSlots launches may be in flight on different streams at once).
static constexpr int kCounterSlots = 256;
static int64_t *g_counters[kMaxDevices];
static std::atomic<unsigned> g_counter_next[kMaxDevices];

static void init_device(int dev) {
    if (hipMalloc((void **)&g_counters[dev], sizeof(int64_t) * kCounterSlots) != hipSuccess)
        g_counters[dev] = nullptr;
    float tab[kExpTableSize];
    come_exp_table(tab);
    g_init_rc[dev] = come_upload_exp_table(tab);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) g_cus[dev] = prop.multiProcessorCount;
    if (g_cus[dev] <= 0) g_cus[dev] = 256;
}

int ensure_init(int *device_out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_error(e, "hipGetDevice");
    if (dev < 0 || dev >= kMaxDevices) return set_error(COME_E_UNSUPPORTED, "device %d", dev);
    std::call_once(g_once[dev], init_device, dev);
    if (device_out) *device_out = dev;
    if (g_init_rc[dev]) return set_error(g_init_rc[dev], "come_init failed on device %d", dev);
    return COME_OK;
}

int num_cus(int device) { return g_cus[device] > 0 ? g_cus[device] : 256; }

// Growable scratch, one buffer per (device, slot, stream) so launches on different streams never
// share a region (never shrinks; growing frees the old buffer, which waits for the device).
// Slots: the O2 ring kernel's entry snapshots; the GMM E-step's per-component flags.
struct Scratch {
    float *ptr = nullptr;
    size_t bytes = 0;
};
static std::unordered_map<void *, Scratch> g_scratch[kMaxDevices][kScratchSlots];
static std::mutex g_scratch_mu;


// Per-(device, slot, stream) scratch that only grows.  A growth is stream-ordered (hipFreeAsync /
// hipMallocAsync on the stream the scratch serves): the kernels still reading the old buffer on
// that stream finish first, and no device-wide synchronisation happens in the middle of a stream
// (a plain hipFree here stalled the device).  Grown by at least 1.5x so a slowly
// growing caller reallocates O(log) times.
// A growth inside a stream capture is refused: hipFreeAsync / hipMallocAsync would
// become graph nodes, and the cache would keep a graph-owned pointer that later eager launches on
// the stream reuse.  Failures set the error message; callers return scratch_failed().
static thread_local int g_scratch_rc = COME_OK;

int scratch_failed() { return g_scratch_rc; }

float *stream_scratch(int device, void *stream, int slot, size_t bytes) {
    if (slot < 0 || slot >= kScratchSlots) {
        g_scratch_rc = set_error(COME_E_INVALID, "scratch slot %d", slot);
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    Scratch &s = g_scratch[device][slot][stream];
    if (s.bytes >= bytes) return s.ptr;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing((hipStream_t)stream, &cap) != hipSuccess ||
        cap != hipStreamCaptureStatusNone) {
        g_scratch_rc = set_error(COME_E_INVALID,
                                 "library scratch must grow to %zu bytes while the stream is being "
                                 "captured: run the same call once before capturing it", bytes);
        return nullptr;
    }
    if (s.bytes) bytes = std::max(bytes, s.bytes + s.bytes / 2);
    if (s.ptr) (void)hipFreeAsync(s.ptr, (hipStream_t)stream);
    s = Scratch{};
    const hipError_t e = hipMallocAsync((void **)&s.ptr, bytes, (hipStream_t)stream);
    if (e != hipSuccess) {
        s.ptr = nullptr;
        g_scratch_rc = hip_error(e, "library scratch allocation");
        return nullptr;
    }
    s.bytes = bytes;
    return s.ptr;
}

int64_t *launch_counter(int device, void *stream) {
    if (!g_counters[device]) return nullptr;
    int64_t *c = g_counters[device] + (g_counter_next[device]++ % kCounterSlots);
    if (hipMemsetAsync(c, 0, sizeof(int64_t), (hipStream_t)stream) != hipSuccess) return nullptr;
    return c;
}

// ---- process-wide launch options (come_set_option / come_get_options) ----
static std::mutex g_opts_mu;
static come_launch_opts g_opts = [] {
    come_launch_opts o;
    memset(&o, 0, sizeof(o));
    // Hogwild concurrency: at most max(1, V / rows_per_wave) wavefronts in flight.  Hogwild
    // needs sparse updates: with every wavefront holding ~17 rows (O2: the 2w+1 window, the
    // positive, the pair's negatives; O1 12), a vocabulary smaller than ~16 rows per wavefront
    // in flight has most rows held by several wavefronts at once and the embeddings stop
    // converging -- measured on a 2,000-node planted partition (round 1; the numbers are in
    // profiles/r01_hogwild_concurrency_nmi.txt, the one-off script is gone):
    // community NMI 0.75 with 6,000 waves in flight, 0.97-0.98 with <= V/16 (= the sequential
    // run's 0.97); at 100,000 nodes the cap is inactive (V/16 > occupancy) and NMI 0.99 either way.
    o.rows_per_wave = 16;
    o.o1_rows_per_wave = 12;
    o.community_async = 3;
    o.gmm_cov_async = 4;
    o.gmm_resp16 = 3;
    o.o1_chunk = -1;
    o.walk_staged = 1;
    return o;
}();

come_launch_opts current_opts() {
    std::lock_guard<std::mutex> lock(g_opts_mu);
    come_launch_opts o = g_opts;
    o.o2_update_count = nullptr;
    return o;
}

}  // namespace come

using namespace come;

extern "C" int come_get_options(come_launch_opts *out) {
    if (!out) return set_error(COME_E_INVALID, "null options pointer");
    *out = current_opts();
    return COME_OK;
}

extern "C" int come_set_option(const char *name, int value) {
    if (!name) return set_error(COME_E_INVALID, "null option name");
#define COME_OPT(f) {#f, offsetof(come_launch_opts, f)}
    static const struct {
        const char *k;
        size_t off;
    } fields[] = {COME_OPT(o2_kernel),        COME_OPT(o2_blocks_per_cu),
                  COME_OPT(o2_waves_per_block), COME_OPT(o2_static),
                  COME_OPT(rows_per_wave),    COME_OPT(o1_rows_per_wave),
                  COME_OPT(max_waves),        COME_OPT(o1_blocks_per_cu),
                  COME_OPT(resident_cap),     COME_OPT(community_async),
                  COME_OPT(gmm_cov_async),    COME_OPT(walk_staged),
                  COME_OPT(o2_fresh_loads),   COME_OPT(o2_atomic_writeback),
                  COME_OPT(gmm_resp16),
                  COME_OPT(o1_chunk)};
#undef COME_OPT
    for (const auto &f : fields)
        if (!strcmp(f.k, name)) {
            std::lock_guard<std::mutex> lock(g_opts_mu);
            *reinterpret_cast<int *>(reinterpret_cast<char *>(&g_opts) + f.off) = value;
            return COME_OK;
        }
    return set_error(COME_E_INVALID, "unknown option '%s'", name);
}

extern "C" int come_abi_version(void) { return COME_ABI_VERSION; }

extern "C" const char *come_last_error(void) { return g_err; }

extern "C" int come_fast_version(void) { return 0; }

extern "C" int come_init(int device) {
    int cur = 0;
    hipError_t e = hipGetDevice(&cur);
    if (e != hipSuccess) return hip_error(e, "hipGetDevice");
    if (device != cur) {
        e = hipSetDevice(device);
        if (e != hipSuccess) return hip_error(e, "hipSetDevice");
    }
    int rc = ensure_init(nullptr);
    if (device != cur) (void)hipSetDevice(cur);
    return rc;
}

// pyx:531-533, with the promotions of the generated C: i/(float)1000 in float, the rest in double,
// stored as float twice.
extern "C" void come_exp_table(float *out) {
    for (int i = 0; i < kExpTableSize; ++i) {
        const float q = (float)i / (float)kExpTableSize;
        const float e = (float)exp(((double)q * 2.0 - 1.0) * 6.0);
        out[i] = (float)((double)e / ((double)e + 1.0));
    }
}

// model.py:97-122.  The literal loop is O(T) with one double division per slot; here each run of
// equal values is located directly: the slot where `widx` advances is the first t >= pos with
// (double)t / T > d1 (the predicate is monotone in t), found from floor(d1 * T) and corrected by
// exact re-evaluation of the reference's own predicate, so the output is identical slot for slot.
extern "C" int come_make_table(const double *counts_by_id, int64_t V, uint32_t *table, uint64_t T,
                               double power) {
    if (!counts_by_id || !table) return set_error(COME_E_INVALID, "null pointer");
    if (V < 2) return set_error(COME_E_INVALID, "make_table needs V >= 2 (got %lld)", (long long)V);
    if (T == 0) return COME_OK;
    double z = 0.0;
    for (int64_t id = 1; id <= V; ++id) z += pow(counts_by_id[id], power);
    const double Td = (double)T;
    auto pred = [&](uint64_t t, double d1) { return 1.0 * (double)t / Td > d1; };
    int64_t widx = 1;
    double d1 = pow(counts_by_id[1], power) / z;
    uint64_t pos = 0;
    while (pos < T) {
        // first t >= pos at which the reference advances widx (stores widx at t, then advances)
        uint64_t t;
        if (pred(pos, d1)) {
            t = pos;
        } else {
            double guess = floor(d1 * Td);
            uint64_t c = guess < (double)pos ? pos : (guess >= Td ? T : (uint64_t)guess);
            while (c > pos && pred(c - 1, d1)) --c;
            while (c < T && !pred(c, d1)) ++c;
            t = c;  // may be T: no further advance
        }
        const uint64_t end = t < T ? t + 1 : T;  // slots [pos, end) hold widx
        for (uint64_t s = pos; s < end; ++s) table[s] = (uint32_t)widx;
        pos = end;
        if (t >= T) break;
        widx += 1;
        d1 += pow(counts_by_id[widx], power) / z;
        if (widx >= V) {  // clamp (model.py:120-121): every later slot holds V-1
            for (uint64_t s = pos; s < T; ++s) table[s] = (uint32_t)(V - 1);
            break;
        }
    }
    return COME_OK;
}

// train_o2's loop nest (pyx:494-506) without the work: one count per fast_o2 call.
extern "C" int64_t come_count_o2_pairs(const int32_t *walks, int64_t P, int L, int window) {
    if (!walks || P <= 0 || L <= 0 || window < 0) return 0;
    const int path_len = L < kMaxSentenceLen ? L : kMaxSentenceLen;
    int64_t total = 0;
    for (int64_t p = 0; p < P; ++p) {
        const int32_t *idx = walks + p * (int64_t)L;
        for (int i = 0; i < path_len; ++i) {
            if (idx[i] < 0) continue;
            const int j0 = i - window < 0 ? 0 : i - window;
            const int j1 = i + window + 1 > path_len ? path_len : i + window + 1;
            for (int j = j0; j < j1; ++j)
                if (j != i && idx[j] >= 0) ++total;
        }
    }
    return total;
}

extern "C" int come_lcg_table_draws(uint64_t seed, int64_t count, const uint32_t *table,
                                    uint64_t T, uint32_t *out) {
    if (count < 0 || (count > 0 && (!table || !out || T == 0)))
        return set_error(COME_E_INVALID, "lcg_table_draws: bad arguments");
    uint64_t nr = seed & kLcgMask;
    for (int64_t i = 0; i < count; ++i) {  // pyx:133-134: draw, then advance
        out[i] = table[(nr >> 16) % T];
        nr = (nr * kLcgMul + kLcgAdd) & kLcgMask;
    }
    return COME_OK;
}
