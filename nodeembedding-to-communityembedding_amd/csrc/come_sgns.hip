// come_sgns.hip -- launchers and C-ABI entry points of the SGNS kernels (come_sgns_impl.h).
#include <string.h>

#include <map>
#include <mutex>
#include <tuple>

#include "come_sgns_impl.h"

namespace come {

constexpr size_t kLdsPerCu = 160 * 1024;
constexpr size_t kRingMaxWaveBytes = 40 * 1024;

// Tuning / experiment knobs (come_set_option); 0 = automatic.
static int g_opt_o2_kernel = 0;         // 1 = direct kernel, 2 = ring kernel
static int g_opt_o2_blocks_per_cu = 0;  // grid cap override
static int g_opt_o2_plain_writeback = 0;  // 1 = Hogwild with plain-store write-back (lossy)
static int g_opt_o2_waves_per_block = 0;
static int g_opt_o2_static = 0;  // 1 = grid-stride walk assignment instead of the work queue
static int g_opt_o2_pair_atomics = 0;  // 1 = HOG node rows: one atomic per pair (no snapshots)
// Hogwild concurrency: at most max(1, V / rows_per_wave) wavefronts in flight (0 = no V-based
// cap) and at most max_waves (0 = the hardware's occupancy).  Hogwild needs sparse updates: with
// every wavefront holding ~17 rows (O2: the 2w+1 window, the positive, the pair's negatives; O1
// 12), a vocabulary smaller than ~16 rows per wavefront in flight has most rows held by several
// wavefronts at once and the embeddings stop converging -- measured on a 2,000-node planted
// partition (scripts/diag_hogwild.py): community NMI 0.75 with 6,000 waves in flight, 0.97-0.98
// with <= V/16 (= the sequential run's 0.97); at 100,000 nodes the cap is inactive (V/16 >
// occupancy) and NMI 0.99 either way.
static int g_opt_rows_per_wave = 16;     // O2
static int g_opt_o1_rows_per_wave = 12;  // O1
static int g_opt_max_waves = 0;
static int g_opt_o1_blocks_per_cu = 0;    // O1 grid cap (0 = 6 four-wave workgroups per CU)
static int g_opt_resident_cap = 0;        // 1 = clamp grids to resident workgroups (A/B)

// Cap on the number of workgroups of a Hogwild launch (0 = none).
static int64_t hog_max_blocks(int64_t V, int wpb, int rows_per_wave) {
    int64_t waves = 0;
    if (rows_per_wave > 0) waves = V / rows_per_wave > 1 ? V / rows_per_wave : 1;
    if (g_opt_max_waves > 0 && (waves == 0 || g_opt_max_waves < waves)) waves = g_opt_max_waves;
    return waves > 0 ? (waves + wpb - 1) / wpb : 0;
}

// ---- launchers -----------------------------------------------------------------------------
static const KernelSet &kernel_set(int d, int *full) {
    const int vec = d <= 64 ? 1 : d <= 128 ? 2 : d <= 256 ? 4 : 8;
    *full = (vec > 1 && d == 64 * vec) ? 1 : 0;
    switch (vec) {
        case 1: return kernels_vec1();
        case 2: return kernels_vec2();
        case 4: return kernels_vec4();
        default: return kernels_vec8();
    }
}
static int maxn_index(int n) { return n <= 5 ? 0 : (n <= 10 ? 1 : 2); }

// Workgroups of `fn` resident per CU at this block size and LDS (cached; 0 = unknown).  Clamping a
// grid-stride launch to it is an A/B knob only (resident_cap=1): measured on O1 at C2 (d = 128,
// 7 waves/SIMD resident), 4-wave workgroups per CU 8 (over-subscribed) / 7 (clamped) / 6 / 5 / 4
// -> 1.28 / 1.42 / 1.08 / 1.12 / 1.27 ms per pass (profiles/r01h_ab_o1_grid.txt): what matters
// is the number of wavefronts contending for the memory system, 24 per CU as for O2.
static int resident_blocks(void *fn, int threads, size_t lds) {
    static std::mutex mu;
    static std::map<std::tuple<void *, int, size_t>, int> cache;
    std::lock_guard<std::mutex> lock(mu);
    const auto key = std::make_tuple(fn, threads, lds);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void *)fn, threads, lds) !=
            hipSuccess || n < 0) {
        (void)hipGetLastError();
        n = 0;
    }
    cache[key] = n;
    return n;
}

// Launch `fn` with one wavefront per unit (walk / edge), `wpb` wavefronts per workgroup, grid
// capped at `blocks_per_cu` workgroups per CU and at what is resident (grid-stride beyond);
// SEQUENTIAL = one wavefront.
static int launch(void *fn, void *args, int64_t units, int mode, int wpb, int blocks_per_cu,
                  size_t lds_bytes, void *stream, int64_t max_blocks = 0) {
    int dev = 0;
    int rc = ensure_init(&dev);
    if (rc) return rc;
    dim3 grid, block;
    if (mode == COME_MODE_SEQUENTIAL) {
        grid = dim3(1);
        block = dim3(64);
    } else {
        int64_t blocks = (units + wpb - 1) / wpb;
        const int res = resident_blocks(fn, 64 * wpb, lds_bytes);
        if (res > 0 && blocks_per_cu > res && g_opt_resident_cap) blocks_per_cu = res;
        int64_t cap = (int64_t)num_cus(dev) * blocks_per_cu;
        if (max_blocks > 0 && max_blocks < cap) cap = max_blocks;
        if (blocks > cap) blocks = cap;
        grid = dim3((unsigned)(blocks > 0 ? blocks : 1));
        block = dim3(64 * wpb);
    }
    void *kargs[] = {args};  // each kernel takes its argument struct by value
    hipError_t e = hipLaunchKernel(fn, grid, block, kargs, lds_bytes, (hipStream_t)stream);
    return hip_error(e, "kernel launch");
}

}  // namespace come

using namespace come;

static int check_common(int64_t V, int d, int negative, const uint32_t *table, uint64_t T,
                        int &mode, int &packed) {
    packed = (mode & COME_TABLE_PACKED) ? 1 : 0;
    mode &= ~COME_TABLE_PACKED;
    if (packed && ((uintptr_t)table % 16) != 0)
        return set_error(COME_E_INVALID, "packed table must be 16-byte aligned");
    if (V <= 0) return set_error(COME_E_INVALID, "V must be > 0 (got %lld)", (long long)V);
    if (V > INT32_MAX)
        return set_error(COME_E_INVALID, "V must fit int32 row indices (got %lld)", (long long)V);
    if (d < 1 || d > kMaxDim)
        return set_error(COME_E_INVALID, "d must be in [1, %d] (got %d)", kMaxDim, d);
    if (negative < 0 || negative > kMaxNegative)
        return set_error(COME_E_INVALID, "negative must be in [0, %d] (got %d)", kMaxNegative,
                         negative);
    if (negative > 0 && (table == nullptr || T == 0))
        return set_error(COME_E_INVALID, "negative sampling needs a non-empty table");
    if (mode != COME_MODE_HOGWILD && mode != COME_MODE_SEQUENTIAL)
        return set_error(COME_E_INVALID, "mode must be COME_MODE_HOGWILD or COME_MODE_SEQUENTIAL");
    return COME_OK;
}

static bool aligned_for(const void *p, int d) {
    const int vec = (d + 63) / 64;
    if (d != 64 * vec || vec < 2) return true;
    const int bytes = (vec >= 4 ? 16 : 8);
    return ((uintptr_t)p % bytes) == 0;
}

extern "C" int come_sgns_o2(float *node, float *ctx, int64_t V, int d, const int32_t *walks,
                            int64_t P, int L, const uint64_t *seeds, int window, int negative,
                            const uint32_t *table, uint64_t T, float lr, float alpha, int mode,
                            void *stream) {
    int packed = 0;
    int rc = check_common(V, d, negative, table, T, mode, packed);
    if (rc) return rc;
    if (P < 0 || L < 0 || window < 0)
        return set_error(COME_E_INVALID, "P, L and window must be >= 0");
    if (P == 0 || L == 0) return COME_OK;
    if (!node || !ctx || !walks || !seeds)
        return set_error(COME_E_INVALID, "null node/ctx/walks/seeds pointer");
    if (!aligned_for(node, d) || !aligned_for(ctx, d))
        return set_error(COME_E_INVALID, "node/ctx must be 16-byte aligned for d=%d", d);
    O2Args a{node, ctx, walks, seeds, table, V, P, L, d, window, negative, lr, alpha,
             make_fastmod(T), packed, nullptr, nullptr};
    int full = 0;
    const KernelSet &ks = kernel_set(d, &full);
    const int mi = maxn_index(negative);
    const bool hog = mode == COME_MODE_HOGWILD;
    // LDS ring of the cached kernel: (2w+1) rows + their ids, per wave
    const int rs = 2 * window + 1;
    const size_t wave_bytes = 4 * (size_t)((rs * d + 3) & ~3);
    const bool ring_ok = rs <= 64 && wave_bytes <= kRingMaxWaveBytes;
    if (g_opt_o2_kernel != 1 && ring_ok) {
        // __launch_bounds__(128): at most 2 wavefronts per workgroup
        const int wpb = g_opt_o2_waves_per_block == 1 ? 1 : 2;
        const size_t lds = wave_bytes * (hog ? wpb : 1);
        // 24 wavefronts per CU measured best on MI355X (d=128, n=5: 16/20/24/28 waves ->
        // 141/123/110/132 ms per 1e8-pair launch with the first write-back; with the work queue
        // and delta write-back 20/22/24/26 -> 111.0/104.6/100.3/100.3 ms, scripts/ab_o2.py).
        int per_cu = (int)(kLdsPerCu / (wave_bytes * wpb));
        per_cu = per_cu < 1 ? 1 : (per_cu > 24 / wpb ? 24 / wpb : per_cu);
        if (g_opt_o2_blocks_per_cu > 0) per_cu = g_opt_o2_blocks_per_cu;
        const int variant = (hog && !g_opt_o2_plain_writeback) ? 1 : 0;
        if (hog) {
            int dev = 0;
            rc = ensure_init(&dev);
            if (rc) return rc;
            if (!g_opt_o2_static) a.counter = launch_counter(dev, stream);  // else grid-stride
            if (variant == 1 && !g_opt_o2_pair_atomics) {
                // entry snapshots, one [2w+1][d] region per wavefront of the (capped) grid
                int64_t blocks = (P + wpb - 1) / wpb;
                int64_t cap = (int64_t)num_cus(dev) * per_cu;
                const int64_t hcap = hog_max_blocks(V, wpb, g_opt_rows_per_wave);
                if (hcap > 0 && hcap < cap) cap = hcap;
                if (blocks > cap) blocks = cap;
                a.orig = o2_scratch(dev, stream, (size_t)blocks * wpb * rs * d * sizeof(float));
            }
        }
        return launch(ks.o2_ring[full][mi][variant], &a, P, mode, wpb, per_cu, lds, stream,
                      hog ? hog_max_blocks(V, wpb, g_opt_rows_per_wave) : 0);
    }
    return launch(ks.o2_direct[full][mi], &a, P, mode, 4,
                  g_opt_o2_blocks_per_cu > 0 ? g_opt_o2_blocks_per_cu : 6, 0, stream,
                  hog ? hog_max_blocks(V, 4, g_opt_rows_per_wave) : 0);
}

extern "C" int come_sgns_o1(float *node, int64_t V, int d, const int32_t *edges, int64_t E,
                            const uint64_t *seeds, int negative, const uint32_t *table, uint64_t T,
                            float lr, int mode, void *stream) {
    int packed = 0;
    int rc = check_common(V, d, negative, table, T, mode, packed);
    if (rc) return rc;
    if (E < 0) return set_error(COME_E_INVALID, "E must be >= 0");
    if (E == 0) return COME_OK;
    if (!node || !edges || !seeds) return set_error(COME_E_INVALID, "null node/edges/seeds");
    if (2 * negative > 64)
        return set_error(COME_E_INVALID, "O1 supports negative <= 32 (got %d)", negative);
    if (!aligned_for(node, d))
        return set_error(COME_E_INVALID, "node must be 16-byte aligned for d=%d", d);
    O1Args a{node, edges, seeds, table, V, E, d, negative, lr, make_fastmod(T), packed};
    int full = 0;
    const KernelSet &ks = kernel_set(d, &full);
    return launch(ks.o1[full][maxn_index(negative)], &a, E, mode, 4,
                  g_opt_o1_blocks_per_cu > 0 ? g_opt_o1_blocks_per_cu : 6, 0, stream,
                  mode == COME_MODE_HOGWILD ? hog_max_blocks(V, 4, g_opt_o1_rows_per_wave) : 0);
}

// One wavefront per 64-slot word: lane i loads slot 64w + i (one coalesced 256-B read), the
// steps to the previous lane are balloted into the word's bit mask; a step other than 0 or 1
// marks the table unpackable (status = 1).
__global__ void __launch_bounds__(256) k_pack_table(const uint32_t *__restrict__ table, uint64_t T,
                                                    uint4 *__restrict__ packed,
                                                    int32_t *__restrict__ status) {
    const int lane = threadIdx.x & 63;
    const uint64_t words = (T + 63) / 64;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    bool bad = false;
    for (uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); w < words;
         w += nwaves) {
        const uint64_t s = w * 64 + lane;
        const uint32_t v = s < T ? table[s] : 0u;
        const uint32_t prev = (uint32_t)__shfl_up((int)v, 1);
        const uint32_t step = v - prev;
        const bool inc = lane > 0 && s < T && step == 1u;
        bad |= lane > 0 && s < T && step > 1u;
        const uint64_t bits = __ballot(inc);
        if (lane == 0) packed[w] = make_uint4(v, 0u, (uint32_t)bits, (uint32_t)(bits >> 32));
    }
    if (__any(bad) && lane == 0) atomicOr(status, 1);
}

extern "C" int come_pack_table(const uint32_t *table, uint64_t T, void *packed, int32_t *status,
                               void *stream) {
    if (!table || !packed || !status || T == 0)
        return set_error(COME_E_INVALID, "pack_table: null pointer or empty table");
    if (((uintptr_t)packed % 16) != 0)
        return set_error(COME_E_INVALID, "packed table must be 16-byte aligned");
    int dev = 0;
    int rc = ensure_init(&dev);
    if (rc) return rc;
    hipError_t e = hipMemsetAsync(status, 0, sizeof(int32_t), (hipStream_t)stream);
    if (e != hipSuccess) return hip_error(e, "hipMemsetAsync(status)");
    const uint64_t words = (T + 63) / 64;
    uint64_t blocks = (words + 3) / 4;
    const uint64_t cap = (uint64_t)num_cus(dev) * 8;
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL(k_pack_table, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       table, T, (uint4 *)packed, status);
    return hip_error(hipGetLastError(), "k_pack_table launch");
}

extern "C" int come_upload_exp_table(const float *host1000) {
    hipError_t (*const up[])(const float *) = {upload_exp_table_vec1, upload_exp_table_vec2,
                                                upload_exp_table_vec4, upload_exp_table_vec8};
    for (auto f : up) {
        const int rc = hip_error(f(host1000), "hipMemcpyToSymbol(exp table)");
        if (rc) return rc;
    }
    return COME_OK;
}

extern "C" int come_set_option(const char *name, int value) {
    if (!name) return set_error(COME_E_INVALID, "null option name");
    struct {
        const char *k;
        int *v;
    } opts[] = {{"o2_kernel", &g_opt_o2_kernel},
                {"o2_blocks_per_cu", &g_opt_o2_blocks_per_cu},
                {"o2_plain_writeback", &g_opt_o2_plain_writeback},
                {"o2_waves_per_block", &g_opt_o2_waves_per_block},
                {"o2_static", &g_opt_o2_static},
                {"o2_pair_atomics", &g_opt_o2_pair_atomics},
                {"rows_per_wave", &g_opt_rows_per_wave},
                {"o1_rows_per_wave", &g_opt_o1_rows_per_wave},
                {"max_waves", &g_opt_max_waves},
                {"o1_blocks_per_cu", &g_opt_o1_blocks_per_cu},
                {"resident_cap", &g_opt_resident_cap},
                {"community_async", &g_comm_async},
                {"gmm_cov_async", &g_cov_async},
                {"walk_staged", &g_walk_staged}};
    for (auto &o : opts)
        if (!strcmp(o.k, name)) {
            *o.v = value;
            return COME_OK;
        }
    return set_error(COME_E_INVALID, "unknown option '%s'", name);
}
