// come_sgns.hip -- launchers and C-ABI entry points of the SGNS kernels (come_sgns_impl.h).
#include <string.h>

#include <map>
#include <mutex>
#include <tuple>

#include "come_sgns_impl.h"

namespace come {

constexpr size_t kRingMaxWaveBytes = 40 * 1024;
constexpr int64_t kStreamRowsPerWave = 32;  // automatic Hogwild O2 kernel choice (come_sgns_o2_ex)

// Cap on the number of workgroups of a Hogwild launch (0 = none).
// Launch knobs come from the caller's come_launch_opts or one snapshot of the process-wide ones
// (come_set_option); see include/come.h for their meaning.
static int64_t hog_max_blocks(const come_launch_opts &o, int64_t V, int wpb, int rows_per_wave) {
    int64_t waves = 0;
    if (rows_per_wave > 0) waves = V / rows_per_wave > 1 ? V / rows_per_wave : 1;
    if (o.max_waves > 0 && (waves == 0 || o.max_waves < waves)) waves = o.max_waves;
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
static int launch(const come_launch_opts &o, void *fn, void *args, int64_t units, int mode,
                  int wpb, int blocks_per_cu, size_t lds_bytes, void *stream,
                  int64_t max_blocks = 0) {
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
        if (res > 0 && blocks_per_cu > res && o.resident_cap) blocks_per_cu = res;
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
                        int &mode, int &packed, int &hot_none) {
    packed = (mode & COME_TABLE_PACKED) ? 1 : 0;
    hot_none = (mode & COME_HOT_NONE) ? 1 : 0;
    mode &= ~(COME_TABLE_PACKED | COME_HOT_NONE);
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

extern "C" int come_sgns_o2_ex(float *node, float *ctx, int64_t V, int d, const int32_t *walks,
                               int64_t P, int L, const uint64_t *seeds, int window, int negative,
                               const uint32_t *table, uint64_t T, float lr, float alpha, int mode,
                               const uint32_t *hot_rows, const come_launch_opts *opts,
                               void *stream) {
    const come_launch_opts o = opts ? *opts : current_opts();
    int packed = 0, hot_none = 0;
    int rc = check_common(V, d, negative, table, T, mode, packed, hot_none);
    if (rc) return rc;
    if (P < 0 || L < 0 || window < 0)
        return set_error(COME_E_INVALID, "P, L and window must be >= 0");
    if (mode == COME_MODE_HOGWILD && o.o2_kernel == 2)
        return set_error(COME_E_INVALID, "o2_kernel=2 (LDS ring) is the sequential kernel only");
    if (P == 0 || L == 0) return COME_OK;
    if (!node || !ctx || !walks || !seeds)
        return set_error(COME_E_INVALID, "null node/ctx/walks/seeds pointer");
    if (!aligned_for(node, d) || !aligned_for(ctx, d))
        return set_error(COME_E_INVALID, "node/ctx must be 16-byte aligned for d=%d", d);
    if (hot_none) {
        hot_rows = nullptr;
    } else if (mode == COME_MODE_HOGWILD && hot_rows == nullptr && table != nullptr && T > 0) {
        int dev = 0;
        rc = ensure_init(&dev);
        if (rc) return rc;
        rc = derive_hot_rows(dev, table, T, packed, V, d, stream, &hot_rows);
        if (rc) return rc;
    }
    O2Args a{node, ctx, walks, seeds, table, V, P, L, d, window, negative, lr, alpha,
             make_fastmod(T), packed, nullptr,
             reinterpret_cast<unsigned long long *>(o.o2_update_count), o.o2_fresh_loads,
             o.o2_atomic_writeback, mode == COME_MODE_HOGWILD ? hot_rows : nullptr};
    int full = 0;
    const KernelSet &ks = kernel_set(d, &full);
    const int mi = maxn_index(negative);
    const bool hog = mode == COME_MODE_HOGWILD;
    // 4-wave workgroups; max_waves 1..3 shrinks them, so max_waves=1 is exactly one wavefront
    const int wpb = (o.max_waves > 0 && o.max_waves < 4) ? o.max_waves : 4;
    if (hog && (o.o2_kernel == 0 || o.o2_kernel == 3) && window <= 31) {
        // streaming Hogwild kernel: 4-wave workgroups, 8 per CU (= its 8 waves per SIMD at
        // d <= 128, n <= 5; measured 6 / 7 / 8 -> 122 / 115 / 108 ms per C3 launch), device work
        // queue
        int dev = 0;
        rc = ensure_init(&dev);
        if (rc) return rc;
        const int bpc = o.o2_blocks_per_cu > 0 ? o.o2_blocks_per_cu : 8;
        const int64_t hcap = hog_max_blocks(o, V, wpb, o.rows_per_wave);
        int64_t blocks = (P + wpb - 1) / wpb;
        if (blocks > (int64_t)num_cus(dev) * bpc) blocks = (int64_t)num_cus(dev) * bpc;
        if (hcap > 0 && blocks > hcap) blocks = hcap;
        // Automatic choice: the streaming kernel reads each pair's rows one pair ahead and runs
        // 1.4x the direct kernel's pair rate, so a hub row collects that many more concurrent
        // updates computed from a stale copy.  With fewer than kStreamRowsPerWave rows per
        // wavefront in flight that occasionally throws a hub's node row into the +-6 skip region
        // for good (100k-node Chung-Lu, 10k walks: held-out loss +3..7% in 2-4 of 10 launches;
        // none at 200k-1M nodes; profiles/r02_ab_hogwild_contention.txt), so small vocabularies
        // run the direct kernel, which reads every row when its pair starts (stable in every
        // run, the same speed there: nearly every row is hot and atomic-bound).
        if (o.o2_kernel == 3 || V >= kStreamRowsPerWave * wpb * blocks) {
            if (!o.o2_static) a.counter = launch_counter(dev, stream);  // else grid-stride
            return launch(o, ks.o2_stream[full][mi], &a, P, mode, wpb, bpc, 0, stream, hcap);
        }
    }
    // LDS ring of the sequential kernel: (2w+1) rows + their ids
    const int rs = 2 * window + 1;
    const size_t wave_bytes = 4 * (size_t)((rs * d + 3) & ~3);
    const bool ring_ok = rs <= 64 && wave_bytes <= kRingMaxWaveBytes;
    if (!hog && o.o2_kernel != 1 && ring_ok)
        return launch(o, ks.o2_ring[full][mi], &a, P, mode, 1, 1, wave_bytes, stream);
    return launch(o, ks.o2_direct[full][mi], &a, P, mode, wpb,
                  o.o2_blocks_per_cu > 0 ? o.o2_blocks_per_cu : 6, 0, stream,
                  hog ? hog_max_blocks(o, V, wpb, o.rows_per_wave) : 0);
}

extern "C" int come_sgns_o2(float *node, float *ctx, int64_t V, int d, const int32_t *walks,
                            int64_t P, int L, const uint64_t *seeds, int window, int negative,
                            const uint32_t *table, uint64_t T, float lr, float alpha, int mode,
                            void *stream) {
    return come_sgns_o2_ex(node, ctx, V, d, walks, P, L, seeds, window, negative, table, T, lr,
                           alpha, mode, nullptr, nullptr, stream);
}

extern "C" int come_sgns_o1_ex(float *node, int64_t V, int d, const int32_t *edges, int64_t E,
                               const uint64_t *seeds, int negative, const uint32_t *table,
                               uint64_t T, float lr, int mode, const uint32_t *hot_rows,
                               const come_launch_opts *opts, void *stream) {
    const come_launch_opts o = opts ? *opts : current_opts();
    int packed = 0, hot_none = 0;
    int rc = check_common(V, d, negative, table, T, mode, packed, hot_none);
    if (rc) return rc;
    if (E < 0) return set_error(COME_E_INVALID, "E must be >= 0");
    if (E == 0) return COME_OK;
    if (!node || !edges || !seeds) return set_error(COME_E_INVALID, "null node/edges/seeds");
    if (2 * negative > 64)
        return set_error(COME_E_INVALID, "O1 supports negative <= 32 (got %d)", negative);
    if (!aligned_for(node, d))
        return set_error(COME_E_INVALID, "node must be 16-byte aligned for d=%d", d);
    if (hot_none) {
        hot_rows = nullptr;
    } else if (mode == COME_MODE_HOGWILD && hot_rows == nullptr && table != nullptr && T > 0) {
        int dev = 0;
        rc = ensure_init(&dev);
        if (rc) return rc;
        rc = derive_hot_rows(dev, table, T, packed, V, d, stream, &hot_rows);
        if (rc) return rc;
    }
    // default grid: 8 four-wave workgroups per CU where the run kernel is compiled for 8 waves per
    // SIMD (d <= 128, n <= 5: o1_runs_waves_per_eu), else 6
    const int bpc = o.o1_blocks_per_cu > 0 ? o.o1_blocks_per_cu
                    : (o.o1_chunk != 0 && d <= 128 && negative <= 5) ? 8 : 6;
    const int64_t hcap = mode == COME_MODE_HOGWILD ? hog_max_blocks(o, V, 4, o.o1_rows_per_wave) : 0;
    int64_t chunk = o.o1_chunk;
    if (chunk < 0) {  // auto: one contiguous chunk per wavefront of the grid
        int dev = 0;
        rc = ensure_init(&dev);
        if (rc) return rc;
        int64_t blocks = (int64_t)num_cus(dev) * bpc;
        if (hcap > 0 && hcap < blocks) blocks = hcap;
        const int64_t waves = mode == COME_MODE_HOGWILD ? 4 * blocks : 1;
        chunk = (E + waves - 1) / waves;
    }
    O1Args a{node,           edges, seeds, table, V, E, d, negative, lr, make_fastmod(T), packed,
             mode == COME_MODE_HOGWILD ? hot_rows : nullptr, chunk > 0 ? chunk : 1};
    int full = 0;
    const KernelSet &ks = kernel_set(d, &full);
    if (chunk > 0)  // one wavefront per chunk of consecutive edges, the input row held
        return launch(o, ks.o1_runs[full][maxn_index(negative)], &a, (E + chunk - 1) / chunk, mode,
                      4, bpc, 0, stream, hcap);
    return launch(o, ks.o1[full][maxn_index(negative)], &a, E, mode, 4,
                  o.o1_blocks_per_cu > 0 ? o.o1_blocks_per_cu : 6, 0, stream,
                  mode == COME_MODE_HOGWILD ? hog_max_blocks(o, V, 4, o.o1_rows_per_wave) : 0);
}

extern "C" int come_sgns_o1(float *node, int64_t V, int d, const int32_t *edges, int64_t E,
                            const uint64_t *seeds, int negative, const uint32_t *table, uint64_t T,
                            float lr, int mode, void *stream) {
    return come_sgns_o1_ex(node, V, d, edges, E, seeds, negative, table, T, lr, mode, nullptr,
                           nullptr, stream);
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
