// come_walk.hip -- device random-walk generator (gfx950): the producer of train_o2's input.
//
// Reference: utils/graph_utils.py __random_walk__ (:20-46) driven by build_deepwalk_corpus_iter
// (:187-192).  Same distribution as the reference walker -- from the current node, with
// probability alpha jump back to the walk's first node, otherwise move to a uniformly chosen
// neighbour; a node without neighbours ends the walk -- but not the same random stream: the
// reference's CPython MT19937 stream is restated exactly on the host (come_walks_reference).
//
// One lane per walk.  The random numbers come from Philox-4x32-10 keyed by the seed and counted
// by (walk, step), so a walk's path does not depend on the launch shape, the batch it is in or
// the device.  Per step a lane reads rowptr[cur], rowptr[cur + 1] (one 16-B pair) and one col
// entry: latency-bound gathers with thousands of walks in flight per CU.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "come_internal.h"

namespace come {

struct WalkArgs {
    const int64_t *rowptr;
    const int32_t *col;
    const int32_t *starts;
    const int32_t *emit;
    int32_t *out;
    int64_t V;
    int64_t P;
    int64_t walk_offset;  // global index of walk 0 of this launch (counter of the stream)
    uint64_t seed;
    int L;
    uint32_t restart_threshold;  // restart iff 24-bit uniform < threshold (alpha * 2^24)
};

struct Philox {
    uint32_t r[4];
};

__device__ inline Philox philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                       uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return {{c0, c1, c2, c3}};
}

__global__ void __launch_bounds__(256) k_random_walks(WalkArgs a) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= a.P) return;
    int32_t *row = a.out + w * (int64_t)a.L;
    const int32_t start = a.starts[w];
    const uint64_t gw = (uint64_t)(a.walk_offset + w);
    const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
    int t = 0;
    if (start < 0 || start >= a.V) {  // not a node: an empty walk
        for (; t < a.L; ++t) row[t] = -1;
        return;
    }
    int32_t cur = start;
    row[t++] = a.emit ? a.emit[cur] : cur;
    for (; t < a.L; ++t) {
        const int64_t b = a.rowptr[cur];
        const int64_t deg = a.rowptr[cur + 1] - b;
        if (deg <= 0) break;  // graph_utils.py:44-45
        const Philox x = philox4x32_10((uint32_t)t, (uint32_t)gw, (uint32_t)(gw >> 32), 0u, k0, k1);
        if ((x.r[1] >> 8) >= a.restart_threshold) {  // rand.random() >= alpha (:39)
            // uniform neighbour (:40): multiply-shift of a 32-bit uniform, bias <= deg / 2^32
            const uint32_t pick = (uint32_t)(((uint64_t)x.r[0] * (uint64_t)deg) >> 32);
            cur = a.col[b + pick];
        } else {
            cur = start;  // restart (:42)
        }
        row[t] = a.emit ? a.emit[cur] : cur;
    }
    for (; t < a.L; ++t) row[t] = -1;
}

// The same walks (same Philox counters, same steps), with the output staged through LDS: a lane's
// row is L ints at a 4L-byte stride, so the direct kernel's per-step store touches 64 cache lines
// per wavefront.  Here each lane fills a WALK_CHUNK-step slice of its row in LDS and the
// workgroup then writes the slice out as 64-B row segments, 16 lanes per segment.  Lanes past P
// or past a dead end keep going through the chunk loop (they emit -1) so every lane reaches the
// barriers.
constexpr int WALK_BLOCK = 256;

template <int WALK_CHUNK>
__global__ void __launch_bounds__(WALK_BLOCK) k_random_walks_staged(WalkArgs a) {
    __shared__ int32_t tile[WALK_BLOCK][WALK_CHUNK + 1];  // +1: column writes hit distinct banks
    const int tid = threadIdx.x;
    const int64_t w0 = (int64_t)blockIdx.x * WALK_BLOCK;
    const int64_t w = w0 + tid;
    const uint64_t gw = (uint64_t)(a.walk_offset + w);
    const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
    int32_t start = -1;
    if (w < a.P) start = a.starts[w];
    bool alive = start >= 0 && start < a.V;  // not a node: an empty walk
    int32_t cur = alive ? start : -1;
    const int64_t rows = a.P - w0 < WALK_BLOCK ? a.P - w0 : WALK_BLOCK;
    for (int c0 = 0; c0 < a.L; c0 += WALK_CHUNK) {
        const int cn = a.L - c0 < WALK_CHUNK ? a.L - c0 : WALK_CHUNK;
        for (int j = 0; j < cn; ++j) {
            const int t = c0 + j;
            if (alive && t > 0) {
                const int64_t b = a.rowptr[cur];
                const int64_t deg = a.rowptr[cur + 1] - b;
                if (deg <= 0) {  // graph_utils.py:44-45
                    alive = false;
                } else {
                    const Philox x = philox4x32_10((uint32_t)t, (uint32_t)gw, (uint32_t)(gw >> 32),
                                                   0u, k0, k1);
                    if ((x.r[1] >> 8) >= a.restart_threshold) {  // rand.random() >= alpha (:39)
                        const uint32_t pick = (uint32_t)(((uint64_t)x.r[0] * (uint64_t)deg) >> 32);
                        cur = a.col[b + pick];
                    } else {
                        cur = start;  // restart (:42)
                    }
                }
            }
            tile[tid][j] = alive ? (a.emit ? a.emit[cur] : cur) : -1;
        }
        __syncthreads();
        // rows x cn slice -> global, consecutive lanes on consecutive columns of one row
        for (int i = tid; i < (int)rows * cn; i += WALK_BLOCK) {
            const int r = i / cn, j = i - r * cn;
            a.out[(w0 + r) * (int64_t)a.L + c0 + j] = tile[r][j];
        }
        __syncthreads();
    }
}

}  // namespace come

using namespace come;

extern "C" int come_random_walks(const int64_t *rowptr, const int32_t *col, int64_t V,
                                 const int32_t *starts, int64_t P, int L, float alpha,
                                 uint64_t seed, int64_t walk_offset, const int32_t *emit,
                                 int32_t *out, void *stream) {
    if (V <= 0 || V > INT32_MAX) return set_error(COME_E_INVALID, "V must be in [1, 2^31)");
    if (P < 0 || L < 0 || walk_offset < 0)
        return set_error(COME_E_INVALID, "P, L and walk_offset must be >= 0");
    if (!(alpha >= 0.0f && alpha <= 1.0f)) return set_error(COME_E_INVALID, "alpha not in [0,1]");
    if (P == 0 || L == 0) return COME_OK;
    if (!rowptr || !col || !starts || !out) return set_error(COME_E_INVALID, "null pointer");
    int dev = 0;
    int rc = ensure_init(&dev);
    if (rc) return rc;
    WalkArgs a{rowptr, col, starts, emit, out, V, P, walk_offset, seed, L,
               (uint32_t)ceil((double)alpha * 16777216.0)};
    const int64_t blocks = (P + WALK_BLOCK - 1) / WALK_BLOCK;
    if (blocks > INT32_MAX) return set_error(COME_E_INVALID, "too many walks in one launch");
    void *kargs[] = {&a};
    // walk_staged: 1 = 16-step slices (default), 2 = 8, 3 = 32 (A/B), 0 = direct stores
    const int staged = current_opts().walk_staged;
    const void *k = staged == 0   ? (const void *)k_random_walks
                    : staged == 2 ? (const void *)k_random_walks_staged<8>
                    : staged == 3 ? (const void *)k_random_walks_staged<32>
                                         : (const void *)k_random_walks_staged<16>;
    hipError_t e = hipLaunchKernel(k, dim3((unsigned)blocks), dim3(WALK_BLOCK), kargs, 0,
                                   (hipStream_t)stream);
    return hip_error(e, "k_random_walks launch");
}
