// come_hot.hip -- "hot" rows of a negative-sampling table: the rows so frequent that several
// Hogwild wavefronts update them at the same time.
//
// Why: the reference's Hogwild has `workers` CPU threads, each reading a row fresh from coherent
// memory right before its saxpy (pyx:140-149), so a hub row is seldom updated by two threads at
// once.  On MI355X thousands of wavefronts are in flight and the per-XCD L2s are not coherent, so
// a plain read-modify-write of a hub row (drawn as a negative every few hundred draws, visited by
// a large share of walks) loses most concurrent updates, and a row cached in a wavefront for a
// whole window collects updates computed from a stale copy.  The O2 kernel therefore treats hot
// rows differently from the rest: read right before each pair and updated with float atomics at
// the memory side (no update lost, no stale cache); cold rows keep the cached / plain form.
//
// Hotness is measured on the table itself: a row's draw probability is its number of slots / T
// (model.py:97-122 gives each row count^0.75 / Z of the slots), and the walk-visit frequency of a
// node grows with the same count (its degree), so the rows with the most slots are the contended
// ones in both roles.  come_hot_rows counts each row's slots and marks rows with >= min_count.
#include "come_internal.h"

namespace come {

// counts[v] += occurrences of v in table[0, T); a wavefront whose 64 slots hold one value (the
// common case: make_table's runs are ~T/V slots long) adds once.
__global__ void __launch_bounds__(256) k_table_counts(const uint32_t *__restrict__ table,
                                                      uint64_t T, int64_t V,
                                                      uint32_t *__restrict__ counts) {
    const uint64_t n = (uint64_t)gridDim.x * blockDim.x;
    const int lane = threadIdx.x & 63;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < T;
         base += n) {
        const uint64_t s = base + lane;
        const bool in = s < T;
        const uint32_t v = in ? table[s] : 0xFFFFFFFFu;
        const uint32_t first = (uint32_t)__shfl((int)v, 0);
        const bool uniform_wave = __all(!in || v == first) && first < (uint64_t)V;
        if (uniform_wave) {
            const int cnt = __popcll(__ballot(in));
            if (lane == 0) atomicAdd(counts + first, (uint32_t)cnt);
        } else if (in && (int64_t)v < V) {
            atomicAdd(counts + v, 1u);
        }
    }
}

// The same over come_pack_table's words: slot s = 64 w + i holds base_w + popcount(bits_w & (2^(i+1)
// - 1)) (one 16-B word per 64 slots, read by every lane of the wavefront: one line).
__global__ void __launch_bounds__(256) k_table_counts_packed(const uint4 *__restrict__ words,
                                                             uint64_t T, int64_t V,
                                                             uint32_t *__restrict__ counts) {
    const uint64_t n = (uint64_t)gridDim.x * blockDim.x;
    const int lane = threadIdx.x & 63;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < T;
         base += n) {
        const uint64_t s = base + lane;
        const bool in = s < T;
        const uint4 wd = words[base >> 6];
        const uint64_t bits = ((uint64_t)wd.w << 32) | wd.z;
        const uint64_t mask = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
        const uint32_t v = in ? wd.x + (uint32_t)__popcll(bits & mask) : 0xFFFFFFFFu;
        const uint32_t first = (uint32_t)__shfl((int)v, 0);
        const bool uniform_wave = __all(!in || v == first) && first < (uint64_t)V;
        if (uniform_wave) {
            const int cnt = __popcll(__ballot(in));
            if (lane == 0) atomicAdd(counts + first, (uint32_t)cnt);
        } else if (in && (int64_t)v < V) {
            atomicAdd(counts + v, 1u);
        }
    }
}

// hot_bits[w] bit b = counts[32 w + b] >= min_count
__global__ void __launch_bounds__(256) k_hot_bits(const uint32_t *__restrict__ counts, int64_t V,
                                                  uint64_t min_count,
                                                  uint32_t *__restrict__ hot_bits) {
    const int64_t words = (V + 31) / 32;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words;
         w += (int64_t)gridDim.x * blockDim.x) {
        uint32_t bits = 0;
        for (int b = 0; b < 32; ++b) {
            const int64_t r = 32 * w + b;
            if (r < V && counts[r] >= min_count) bits |= 1u << b;
        }
        hot_bits[w] = bits;
    }
}

static int hot_rows_impl(int dev, const uint32_t *table, uint64_t T, int packed, int64_t V,
                         uint64_t min_count, uint32_t *counts, uint32_t *hot_bits, void *stream) {
    hipError_t e = hipMemsetAsync(counts, 0, sizeof(uint32_t) * (size_t)V, (hipStream_t)stream);
    if (e != hipSuccess) return hip_error(e, "hipMemsetAsync(counts)");
    uint64_t blocks = (T + 255) / 256;
    const uint64_t cap = (uint64_t)num_cus(dev) * 16;
    if (blocks > cap) blocks = cap;
    if (packed)
        hipLaunchKernelGGL(k_table_counts_packed, dim3((unsigned)blocks), dim3(256), 0,
                           (hipStream_t)stream, (const uint4 *)table, T, V, counts);
    else
        hipLaunchKernelGGL(k_table_counts, dim3((unsigned)blocks), dim3(256), 0,
                           (hipStream_t)stream, table, T, V, counts);
    int rc = hip_error(hipGetLastError(), "k_table_counts launch");
    if (rc) return rc;
    const int64_t words = (V + 31) / 32;
    int64_t wb = (words + 255) / 256;
    if (wb > 4096) wb = 4096;
    hipLaunchKernelGGL(k_hot_bits, dim3((unsigned)wb), dim3(256), 0, (hipStream_t)stream,
                       (const uint32_t *)counts, V, min_count, hot_bits);
    return hip_error(hipGetLastError(), "k_hot_bits launch");
}

int derive_hot_rows(int dev, const uint32_t *table, uint64_t T, int packed, int64_t V, int d,
                    void *stream, const uint32_t **bits_out) {
    uint32_t *counts = (uint32_t *)stream_scratch(dev, stream, kScratchHotCounts,
                                                  sizeof(uint32_t) * (size_t)V);
    uint32_t *bits = (uint32_t *)stream_scratch(dev, stream, kScratchHotBits,
                                                sizeof(uint32_t) * (size_t)((V + 31) / 32));
    if (!counts || !bits) return scratch_failed();
    const double share = d <= 128 ? COME_DEFAULT_HOT_SHARE : COME_DEFAULT_HOT_SHARE_WIDE;
    uint64_t min_count = (uint64_t)(share * (double)T);
    if (min_count < 1) min_count = 1;
    *bits_out = bits;
    return hot_rows_impl(dev, table, T, packed, V, min_count, counts, bits, stream);
}

}  // namespace come

using namespace come;

extern "C" int come_hot_rows(const uint32_t *table, uint64_t T, int64_t V, uint64_t min_count,
                             uint32_t *counts, uint32_t *hot_bits, void *stream) {
    if (V <= 0 || V > INT32_MAX) return set_error(COME_E_INVALID, "hot_rows: V out of range");
    if (!table || !counts || !hot_bits || T == 0)
        return set_error(COME_E_INVALID, "hot_rows: null pointer or empty table");
    int dev = 0;
    int rc = ensure_init(&dev);
    if (rc) return rc;
    return hot_rows_impl(dev, table, T, 0, V, min_count, counts, hot_bits, stream);
}
