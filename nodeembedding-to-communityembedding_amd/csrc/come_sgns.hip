// come_sgns.hip -- skip-gram negative-sampling updates for gfx950 (MI355X, CDNA4).
//
// Replaces the reference's Cython hot loop, /root/reference/utils/training_sdg_inner.pyx:
//   fast0_o2/fast1_o2 (pyx:105-201) + train_o2 (pyx:454-509)   -> k_sgns_o2
//   fast0_o1/fast1_o1 (pyx:205-296) + train_o1 (pyx:407-450)   -> k_sgns_o1
//
// Execution model:
//  * One 64-lane wavefront owns one walk (O2) or one edge (O1) and processes its positive pairs in
//    the reference's order, one pair at a time -- exactly the work one reference thread does per
//    nogil call (pyx:493).  All walks/edges of a batch are in flight at once (Hogwild across
//    wavefronts, as the reference's worker threads are Hogwild across walks).
//  * A d-dim fp32 row is spread over the wave: lane l holds elements l*VEC .. l*VEC+VEC-1
//    (VEC = ceil(d/64)); at d = 128 a row is one coalesced 512-B dwordx2 load per wave.
//  * The (1 + negative) target rows of a pair are gathered together, their dot products reduced
//    with interleaved xor butterflies, then resolved in reference order (a negative that repeats an
//    earlier target sees that target's updated row, pyx:147, via register forwarding).
//  * Negatives never touch the host: lane k of the wave computes LCG draw (base + k) by jump-ahead
//    (the LCG is affine mod 2^48, pyx:134) and gathers table[(s >> 16) % T] for 64 draws at once;
//    each pair then reads its n draws with v_readlane (wave-uniform, scalar registers).
//  * Dot product order is fixed: per-lane fmaf chain, then xor butterfly 32,16,8,4,2,1.  The CPU
//    oracle's WAVE64 mode restates this order, so COME_MODE_SEQUENTIAL is bit-exact with it.
//  * Compiled with -ffp-contract=off: every fused multiply-add is an explicit fmaf, matching the
//    reference's saxpy (pyx:146-149) element for element.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "come_internal.h"

namespace come {

__constant__ float c_exp_table[kExpTableSize];

struct LcgLane {  // this lane's jump-ahead (A^k, C_k): s_{b+k} = A^k s_b + C_k  (mod 2^48)
    uint64_t a, c;
};

__device__ inline LcgLane lcg_lane_constants(int k) {
    uint64_t a = 1, c = 0;
    for (int i = 0; i < k; ++i) {
        a = (a * kLcgMul) & kLcgMask;
        c = (c * kLcgMul + kLcgAdd) & kLcgMask;
    }
    return {a, c};
}

__device__ inline uint64_t lcg_next(uint64_t s) { return (s * kLcgMul + kLcgAdd) & kLcgMask; }

__device__ inline uint32_t table_slot(uint64_t s, uint64_t m, uint32_t d) {
    const uint32_t x = (uint32_t)(s >> 16);  // < 2^32 because s < 2^48 (pyx:133)
    if (d == 0) return x;                     // T >= 2^32: x % T == x
    return (uint32_t)__umul64hi(m * (uint64_t)x, (uint64_t)d);
}

__device__ inline int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ inline float uniformf(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ inline uint64_t uniform64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ inline uint32_t readlane_u32(uint32_t v, int lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ inline uint64_t readlane_u64(uint64_t v, int lane) {
    const uint32_t lo = readlane_u32((uint32_t)v, lane);
    const uint32_t hi = readlane_u32((uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

// ---- row <-> registers -------------------------------------------------------------------------
template <int VEC, bool FULL>
struct Row {
    float v[VEC];

    __device__ inline void load(const float *__restrict__ row, int lane, int d) {
        if constexpr (FULL && VEC == 2) {
            const float2 t = *reinterpret_cast<const float2 *>(row + lane * 2);
            v[0] = t.x;
            v[1] = t.y;
        } else if constexpr (FULL && VEC == 4) {
            const float4 t = *reinterpret_cast<const float4 *>(row + lane * 4);
            v[0] = t.x, v[1] = t.y, v[2] = t.z, v[3] = t.w;
        } else if constexpr (FULL && VEC == 8) {
            const float4 t0 = *reinterpret_cast<const float4 *>(row + lane * 8);
            const float4 t1 = *reinterpret_cast<const float4 *>(row + lane * 8 + 4);
            v[0] = t0.x, v[1] = t0.y, v[2] = t0.z, v[3] = t0.w;
            v[4] = t1.x, v[5] = t1.y, v[6] = t1.z, v[7] = t1.w;
        } else {
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                const int e = lane * VEC + i;
                v[i] = e < d ? row[e] : 0.0f;
            }
        }
    }

    __device__ inline void store(float *__restrict__ row, int lane, int d) const {
        if constexpr (FULL && VEC == 2) {
            *reinterpret_cast<float2 *>(row + lane * 2) = make_float2(v[0], v[1]);
        } else if constexpr (FULL && VEC == 4) {
            *reinterpret_cast<float4 *>(row + lane * 4) = make_float4(v[0], v[1], v[2], v[3]);
        } else if constexpr (FULL && VEC == 8) {
            *reinterpret_cast<float4 *>(row + lane * 8) = make_float4(v[0], v[1], v[2], v[3]);
            *reinterpret_cast<float4 *>(row + lane * 8 + 4) = make_float4(v[4], v[5], v[6], v[7]);
        } else {
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                const int e = lane * VEC + i;
                if (e < d) row[e] = v[i];
            }
        }
    }
};

template <int VEC, bool FULL>
__device__ inline float lane_partial(const Row<VEC, FULL> &a, const Row<VEC, FULL> &b) {
    float p = 0.0f;
#pragma unroll
    for (int i = 0; i < VEC; ++i) p = __builtin_fmaf(a.v[i], b.v[i], p);
    return p;
}

__device__ inline float wave_sum(float p) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) p += __shfl_xor(p, off, 64);
    return p;
}

// sigma lookup exactly as generated from pyx:141-143: skip if f <= -6 or f >= 6, else
// EXP_TABLE[(int)(((double)f + 6.0) * 83.0)].  Returns false for a skipped target.
__device__ inline bool sigmoid_ref(float f, float *sig) {
    if (f <= -(float)kMaxExp || f >= (float)kMaxExp) return false;
    const int b = (int)(((double)f + 6.0) * 83.0);
    *sig = c_exp_table[b];
    return true;
}

// ---- batch of 64 negative draws held one per lane ------------------------------------------
struct DrawBatch {
    uint32_t target;  // this lane's table value for draw (base + lane)
    uint64_t base;    // LCG state of draw `base`'s index 0 (wave-uniform)
    int used;         // draws of the batch already consumed (wave-uniform)
};

__device__ inline void draws_fill(DrawBatch &b, uint64_t state0, const LcgLane &lc,
                                  const uint32_t *__restrict__ table, FastMod fm, int64_t V) {
    b.base = state0;
    b.used = 0;
    const uint64_t s = (lc.a * state0 + lc.c) & kLcgMask;
    const uint32_t slot = table_slot(s, fm.m, fm.d);
    uint32_t t = table[slot];
    b.target = t;
}

// State of the draw `b.used` positions after the batch base (0 < used <= 64).
__device__ inline uint64_t draws_state_at_used(const DrawBatch &b, const LcgLane &lc) {
    const uint64_t s = (lc.a * b.base + lc.c) & kLcgMask;  // this lane's state
    if (b.used < 64) return uniform64(readlane_u64(s, b.used));
    return lcg_next(uniform64(readlane_u64(s, 63)));
}

// ---- O2: one wavefront per walk ------------------------------------------------------------
struct O2Args {
    float *node;
    float *ctx;
    const int32_t *walks;
    const uint64_t *seeds;
    const uint32_t *table;
    int64_t V;
    int64_t P;
    int L;
    int d;
    int window;
    int negative;
    float lr;
    float alpha;
    FastMod fm;
};

template <int VEC, bool FULL, int MAXN>
__global__ void __launch_bounds__(256) k_sgns_o2(O2Args a) {
    using R = Row<VEC, FULL>;
    const int lane = threadIdx.x & 63;
    const int64_t waves_per_block = blockDim.x >> 6;
    const int64_t gw = (int64_t)blockIdx.x * waves_per_block + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * waves_per_block;
    const LcgLane lc = lcg_lane_constants(lane);
    const int n = a.negative;
    const int d = a.d;
    const int path_len = a.L < kMaxSentenceLen ? a.L : kMaxSentenceLen;  // pyx:480

    for (int64_t p = gw; p < a.P; p += nwaves) {
        const int32_t *__restrict__ idx = a.walks + p * (int64_t)a.L;
        DrawBatch db;
        db.used = 0;
        db.base = uniform64(a.seeds[p]);
        db.target = 0;
        if (n > 0) draws_fill(db, db.base, lc, a.table, a.fm, a.V);

        for (int i = 0; i < path_len; ++i) {
            const int ci = uniform(idx[i]);
            if (ci < 0 || ci >= a.V) continue;  // codelens[i] == 0 (pyx:495)
            const int j0 = i - a.window < 0 ? 0 : i - a.window;
            const int j1 = i + a.window + 1 > path_len ? path_len : i + a.window + 1;
            for (int j = j0; j < j1; ++j) {
                if (j == i) continue;
                const int cj = uniform(idx[j]);
                if (cj < 0 || cj >= a.V) continue;  // pyx:504

                // ---- the pair's n draws (pyx:133-134), consumed whether used or not ----
                if (n > 0 && db.used + n > 64) draws_fill(db, draws_state_at_used(db, lc), lc, a.table, a.fm, a.V);
                int t[MAXN + 1];
                bool valid[MAXN + 1];
                t[0] = ci;
                valid[0] = true;
#pragma unroll
                for (int k = 1; k <= MAXN; ++k) {
                    if (k <= n) {
                        const int tk = (int)readlane_u32(db.target, db.used + k - 1);
                        t[k] = tk;
                        // pyx:135 skip == positive; out-of-range table values skipped (no OOB)
                        valid[k] = tk != ci && tk >= 0 && tk < a.V;
                    } else {
                        t[k] = -1;
                        valid[k] = false;
                    }
                }
                db.used += n;

                // ---- gather: input row (node[cj]) + every valid target row (ctx[t]) ----
                R in;
                in.load(a.node + (int64_t)cj * d, lane, d);
                R r[MAXN + 1];
#pragma unroll
                for (int k = 0; k <= MAXN; ++k)
                    if (valid[k]) r[k].load(a.ctx + (int64_t)t[k] * d, lane, d);

                // ---- dots of every target against the (fixed) input row, interleaved ----
                float part[MAXN + 1];
#pragma unroll
                for (int k = 0; k <= MAXN; ++k) part[k] = valid[k] ? lane_partial(in, r[k]) : 0.0f;
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
                    for (int k = 0; k <= MAXN; ++k)
                        if (k <= n) part[k] += __shfl_xor(part[k], off, 64);
                }

                // ---- resolve targets in reference order (pyx:128-147) ----
                R work;
#pragma unroll
                for (int e = 0; e < VEC; ++e) work.v[e] = 0.0f;
                bool upd[MAXN + 1];
#pragma unroll
                for (int k = 0; k <= MAXN; ++k) {
                    upd[k] = false;
                    if (!valid[k]) continue;
                    float f = part[k];
                    // A repeated negative sees the row as left by its latest earlier occurrence.
                    int prev = -1;
#pragma unroll
                    for (int q = 1; q < k; ++q)
                        if (valid[q] && t[q] == t[k]) prev = q;
                    if (prev >= 0) {
#pragma unroll
                        for (int q = 1; q < k; ++q) {
                            if (q == prev) {
                                r[k] = r[q];
                                f = upd[q] ? wave_sum(lane_partial(in, r[k])) : part[q];
                            }
                        }
                    }
                    f = uniformf(f);
                    part[k] = f;  // effective dot of this occurrence (a later repeat may reuse it)
                    float sig;
                    if (!sigmoid_ref(f, &sig)) continue;  // pyx:141-142
                    const float label = k == 0 ? 1.0f : 0.0f;
                    const float g = ((label - sig) * a.lr) * a.alpha;  // pyx:144
#pragma unroll
                    for (int e = 0; e < VEC; ++e) {
                        work.v[e] = __builtin_fmaf(g, r[k].v[e], work.v[e]);  // pyx:146
                        r[k].v[e] = __builtin_fmaf(g, in.v[e], r[k].v[e]);    // pyx:147
                    }
                    upd[k] = true;
                }
                // ---- write back (in order, so a repeated row ends with its last version) ----
#pragma unroll
                for (int k = 0; k <= MAXN; ++k)
                    if (upd[k]) r[k].store(a.ctx + (int64_t)t[k] * d, lane, d);
#pragma unroll
                for (int e = 0; e < VEC; ++e) in.v[e] = in.v[e] + work.v[e];  // pyx:149
                in.store(a.node + (int64_t)cj * d, lane, d);
            }
        }
    }
}

// ---- O1: one wavefront per edge ------------------------------------------------------------
struct O1Args {
    float *node;
    const int32_t *edges;
    const uint64_t *seeds;
    const uint32_t *table;
    int64_t V;
    int64_t E;
    int d;
    int negative;
    float lr;
    FastMod fm;
};

template <int VEC, bool FULL, int MAXN>
__global__ void __launch_bounds__(256) k_sgns_o1(O1Args a) {
    using R = Row<VEC, FULL>;
    const int lane = threadIdx.x & 63;
    const int64_t waves_per_block = blockDim.x >> 6;
    const int64_t gw = (int64_t)blockIdx.x * waves_per_block + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * waves_per_block;
    const LcgLane lc = lcg_lane_constants(lane);
    const int n = a.negative;
    const int d = a.d;

    for (int64_t e = gw; e < a.E; e += nwaves) {
        const int u = uniform(a.edges[2 * e]);
        const int v = uniform(a.edges[2 * e + 1]);
        if (u < 0 || u >= a.V || v < 0 || v >= a.V) continue;  // reference: undefined behaviour
        // 2n draws: pair 1 uses draws 0..n-1, pair 2 draws n..2n-1 (state carried, pyx:444-448)
        DrawBatch db;
        db.used = 0;
        db.base = uniform64(a.seeds[e]);
        db.target = 0;
        if (n > 0) draws_fill(db, db.base, lc, a.table, a.fm, a.V);

        int t1[MAXN + 1], t2[MAXN + 1];
        bool v1[MAXN + 1], v2[MAXN + 1];
        t1[0] = v;  // pair 1: input u, positive v (pyx:444)
        t2[0] = u;  // pair 2: input v, positive u (pyx:447)
        v1[0] = v2[0] = true;
#pragma unroll
        for (int k = 1; k <= MAXN; ++k) {
            if (k <= n) {
                t1[k] = (int)readlane_u32(db.target, k - 1);
                t2[k] = (int)readlane_u32(db.target, n + k - 1);
                v1[k] = t1[k] != v && t1[k] >= 0 && t1[k] < a.V;
                v2[k] = t2[k] != u && t2[k] >= 0 && t2[k] < a.V;
            } else {
                t1[k] = t2[k] = -1;
                v1[k] = v2[k] = false;
            }
        }
        // Every row both pairs read can be gathered up front: pair 1 writes only node[u]; pair 2
        // never reads node[u] through a negative (skipped, == its positive) and gets its positive
        // (and, for a self-loop, its input) forwarded from pair 1's registers.
        R in1, in2;
        in1.load(a.node + (int64_t)u * d, lane, d);
        if (v != u) in2.load(a.node + (int64_t)v * d, lane, d);
        R r1[MAXN + 1], r2[MAXN + 1];
#pragma unroll
        for (int k = 1; k <= MAXN; ++k) {
            if (v1[k]) r1[k].load(a.node + (int64_t)t1[k] * d, lane, d);
            if (v2[k]) r2[k].load(a.node + (int64_t)t2[k] * d, lane, d);
        }
        if (v != u) r1[0] = in2; else r1[0] = in1;  // positive of pair 1 = node[v] (pre-update)

        // pair 1
        {
            float part[MAXN + 1];
#pragma unroll
            for (int k = 0; k <= MAXN; ++k) part[k] = v1[k] ? lane_partial(in1, r1[k]) : 0.0f;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
                for (int k = 0; k <= MAXN; ++k)
                    if (k <= n) part[k] += __shfl_xor(part[k], off, 64);
            }
            R work;
#pragma unroll
            for (int q = 0; q < VEC; ++q) work.v[q] = 0.0f;
#pragma unroll
            for (int k = 0; k <= MAXN; ++k) {
                if (!v1[k]) continue;
                float sig;
                if (!sigmoid_ref(uniformf(part[k]), &sig)) continue;
                const float g = ((k == 0 ? 1.0f : 0.0f) - sig) * a.lr;  // pyx:243
#pragma unroll
                for (int q = 0; q < VEC; ++q) work.v[q] = __builtin_fmaf(g, r1[k].v[q], work.v[q]);
            }
#pragma unroll
            for (int q = 0; q < VEC; ++q) in1.v[q] = in1.v[q] + work.v[q];  // pyx:247
            in1.store(a.node + (int64_t)u * d, lane, d);
        }
        // pair 2: positive = node[u] as pair 1 left it; self-loop: the input is that row too.
        r2[0] = in1;
        if (v == u) in2 = in1;
        {
            float part[MAXN + 1];
#pragma unroll
            for (int k = 0; k <= MAXN; ++k) part[k] = v2[k] ? lane_partial(in2, r2[k]) : 0.0f;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
                for (int k = 0; k <= MAXN; ++k)
                    if (k <= n) part[k] += __shfl_xor(part[k], off, 64);
            }
            R work;
#pragma unroll
            for (int q = 0; q < VEC; ++q) work.v[q] = 0.0f;
#pragma unroll
            for (int k = 0; k <= MAXN; ++k) {
                if (!v2[k]) continue;
                float sig;
                if (!sigmoid_ref(uniformf(part[k]), &sig)) continue;
                const float g = ((k == 0 ? 1.0f : 0.0f) - sig) * a.lr;
#pragma unroll
                for (int q = 0; q < VEC; ++q) work.v[q] = __builtin_fmaf(g, r2[k].v[q], work.v[q]);
            }
#pragma unroll
            for (int q = 0; q < VEC; ++q) in2.v[q] = in2.v[q] + work.v[q];
            in2.store(a.node + (int64_t)v * d, lane, d);
        }
    }
}

// ---- launchers -----------------------------------------------------------------------------
template <int VEC, bool FULL, int MAXN>
struct O2K {
    static void *fn() { return reinterpret_cast<void *>(&k_sgns_o2<VEC, FULL, MAXN>); }
};
template <int VEC, bool FULL, int MAXN>
struct O1K {
    static void *fn() { return reinterpret_cast<void *>(&k_sgns_o1<VEC, FULL, MAXN>); }
};

template <template <int, bool, int> class K, int VEC, bool FULL>
static void *pick_maxn(int n) {
    if (n <= 5) return K<VEC, FULL, 5>::fn();
    if (n <= 10) return K<VEC, FULL, 10>::fn();
    return K<VEC, FULL, 20>::fn();
}

template <template <int, bool, int> class K>
static void *pick_kernel(int d, int n) {
    if (d <= 64) return pick_maxn<K, 1, false>(n);
    if (d <= 128) return d == 128 ? pick_maxn<K, 2, true>(n) : pick_maxn<K, 2, false>(n);
    if (d <= 256) return d == 256 ? pick_maxn<K, 4, true>(n) : pick_maxn<K, 4, false>(n);
    return d == 512 ? pick_maxn<K, 8, true>(n) : pick_maxn<K, 8, false>(n);
}

static int launch(void *fn, void *args, size_t args_size, int64_t units, int mode,
                  void *stream) {
    int dev = 0;
    int rc = ensure_init(&dev);
    if (rc) return rc;
    dim3 grid, block;
    if (mode == COME_MODE_SEQUENTIAL) {
        grid = dim3(1);
        block = dim3(64);
    } else {
        const int wpb = 4;  // 256-thread workgroups, one unit (walk / edge) per wavefront
        int64_t blocks = (units + wpb - 1) / wpb;
        const int64_t cap = (int64_t)num_cus(dev) * 8;  // grid-stride beyond 8 blocks per CU
        if (blocks > cap) blocks = cap;
        grid = dim3((unsigned)(blocks > 0 ? blocks : 1));
        block = dim3(64 * wpb);
    }
    (void)args_size;
    void *kargs[] = {args};  // each kernel takes its argument struct by value
    hipError_t e = hipLaunchKernel(fn, grid, block, kargs, 0, (hipStream_t)stream);
    return hip_error(e, "kernel launch");
}

}  // namespace come

using namespace come;

static int check_common(int64_t V, int d, int negative, const uint32_t *table, uint64_t T,
                        int mode) {
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
    int rc = check_common(V, d, negative, table, T, mode);
    if (rc) return rc;
    if (P < 0 || L < 0 || window < 0)
        return set_error(COME_E_INVALID, "P, L and window must be >= 0");
    if (P == 0 || L == 0) return COME_OK;
    if (!node || !ctx || !walks || !seeds)
        return set_error(COME_E_INVALID, "null node/ctx/walks/seeds pointer");
    if (!aligned_for(node, d) || !aligned_for(ctx, d))
        return set_error(COME_E_INVALID, "node/ctx must be 16-byte aligned for d=%d", d);
    O2Args a{node, ctx, walks, seeds, table, V, P, L, d, window, negative, lr, alpha,
             make_fastmod(T)};
    return launch(pick_kernel<O2K>(d, negative), &a, sizeof(a), P, mode, stream);
}

extern "C" int come_sgns_o1(float *node, int64_t V, int d, const int32_t *edges, int64_t E,
                            const uint64_t *seeds, int negative, const uint32_t *table, uint64_t T,
                            float lr, int mode, void *stream) {
    int rc = check_common(V, d, negative, table, T, mode);
    if (rc) return rc;
    if (E < 0) return set_error(COME_E_INVALID, "E must be >= 0");
    if (E == 0) return COME_OK;
    if (!node || !edges || !seeds) return set_error(COME_E_INVALID, "null node/edges/seeds");
    if (2 * negative > 64)
        return set_error(COME_E_INVALID, "O1 supports negative <= 32 (got %d)", negative);
    if (!aligned_for(node, d))
        return set_error(COME_E_INVALID, "node must be 16-byte aligned for d=%d", d);
    O1Args a{node, edges, seeds, table, V, E, d, negative, lr, make_fastmod(T)};
    return launch(pick_kernel<O1K>(d, negative), &a, sizeof(a), E, mode, stream);
}

extern "C" int come_upload_exp_table(const float *host1000) {
    return hip_error(hipMemcpyToSymbol(HIP_SYMBOL(c_exp_table), host1000,
                                       sizeof(float) * kExpTableSize),
                     "hipMemcpyToSymbol(exp table)");
}
