// come_community.hip -- community-embedding step and GMM responsibilities (gfx950).
//
// Replaces /root/reference/ADSCModel/community_embeddings.py:
//   Community2Vec.train (:61-78)  -> k_community_grad
//   GaussianMixture.predict_proba (:37, covariance_type='full') -> k_gmm_resp
//
// Both are dense contractions, 2*V*K*d^2 flops per pass: for a tile of TR rows held in LDS the
// kernel streams each component's d x d matrix through LDS and accumulates the per-component
// matrix-vector products in registers.  Rows are independent in both steps (community_embeddings
// .py:65 takes a snapshot per iteration and every row's gradient reads only its own row), so the
// `iters` loop runs inside the kernel on the LDS-resident tile and x is written back once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <math.h>
#include <stdint.h>

#include "come_internal.h"
#include "come_wave.h"

namespace come {

constexpr int kTR = 16;        // rows per workgroup tile

// A/B hook (scripts/build_ab.sh ... -DCOME_AB_PRIO): raise the wave priority over the MFMA
// clusters of the 16x16x4 kernels (MI355X guide T5); off in the product build.
#ifdef COME_AB_PRIO
#define COME_PRIO(x) __builtin_amdgcn_s_setprio(x)
#else
#define COME_PRIO(x) ((void)0)
#endif
// A/B hooks of k_gmm_cov16 (build_ab.sh only; results are garbage for DIAG != 0):
// COME_COV_DIAG 1 = staging re-stages the first 3 blocks' registers (no global loads after the
// prologue), 2 = MFMA wavefronts consume buffer 0 without barriers (the MFMA stream alone), 3 =
// every load reads the chunk's first block (the same instructions, cache-resident data).
// COME_RESP_DIAG (k_gmm_resp16t) 1 = no copies after component 0, 2 = and no barriers (both read
// the never-written second buffer for odd components: zero-like data, which clocks higher), 3 /
// 4 = as 1 / 2 with every component read from buffer 0 (real data: component 0 repeated).
#ifndef COME_COV_DIAG
#define COME_COV_DIAG 0
#endif
#ifndef COME_RESP_DIAG
#define COME_RESP_DIAG 0
#endif
// k_gmm_cov16 at d = 128: staging register sets (3 / 4 / 5+: 7.266 / 7.247 ms at C4 / spills)
#ifndef COME_COV_NS
#define COME_COV_NS 4
#endif
// k_gmm_cov_bf3 at d = 128: staging wavefronts per workgroup (8: 5.32-5.35 vs 5.49-5.50 ms with 4,
// profiles/r06_ab_scatter_bf3.txt) and staging register sets (A/B hooks)
#ifndef COME_COV3_SW
#define COME_COV3_SW 8
#endif
#ifndef COME_COV3_NS
#define COME_COV3_NS 3
#endif
// MFMA wavefronts per d = 128 component (4: 5.50 vs 5.42-5.44 ms with 2, r06zl)
#ifndef COME_COV3_WPC
#define COME_COV3_WPC 2
#endif
constexpr int kThreads = 256;

// out[r][c] = sum_j A[r][j] * B(c, j) for the tile, where B(c, j) = Bm[c*d + j] (TRANS=false,
// i.e. B used as M @ a) or Bm[j*d + c] (TRANS=true, i.e. a @ B).  A and Bm live in LDS.
template <bool TRANS>
__device__ inline float tile_dot(const float *A, const float *Bm, int r, int c, int d) {
    float acc = 0.0f;
    if (TRANS) {
        for (int j = 0; j < d; ++j) acc = __builtin_fmaf(A[r * d + j], Bm[j * d + c], acc);
    } else {
        for (int j = 0; j < d; ++j) acc = __builtin_fmaf(A[r * d + j], Bm[c * d + j], acc);
    }
    return acc;
}

struct CommArgs {
    float *x;
    const float *pi;
    const float *mu;
    const float *inv_cov;
    int64_t V;
    int d;
    int K;
    float coef;  // (float)(beta / K), community_embeddings.py:77 (numpy weak-scalar cast)
    float lr;
    int iters;
    const void *img;  // k_community_b16: inv_cov as k_comm_split16's bf16 part images
};

__global__ void __launch_bounds__(kThreads) k_community_grad(CommArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int d = a.d;
    float *X = smem;                  // [kTR][d]   current rows
    float *D = X + kTR * d;           // [kTR][d]   x - mu_k
    float *G = D + kTR * d;           // [kTR][d]   gradient accumulator
    float *M = G + kTR * d;           // [d][d]     inv_cov[k]
    const int64_t r0 = (int64_t)blockIdx.x * kTR;
    const int rows = (int)((a.V - r0) < kTR ? (a.V - r0) : kTR);
    const int n = kTR * d;
    for (int o = threadIdx.x; o < n; o += kThreads) {
        const int r = o / d;
        X[o] = r < rows ? a.x[(r0 + r) * d + (o % d)] : 0.0f;
    }
    for (int it = 0; it < a.iters; ++it) {
        for (int o = threadIdx.x; o < n; o += kThreads) G[o] = 0.0f;
        for (int k = 0; k < a.K; ++k) {
            __syncthreads();
            for (int o = threadIdx.x; o < d * d; o += kThreads) M[o] = a.inv_cov[(int64_t)k * d * d + o];
            for (int o = threadIdx.x; o < n; o += kThreads) D[o] = X[o] - a.mu[k * d + (o % d)];
            __syncthreads();
            for (int o = threadIdx.x; o < n; o += kThreads) {
                const int r = o / d, c = o % d;
                if (r >= rows) continue;
                const float p = a.pi[(r0 + r) * a.K + k];
                G[o] = __builtin_fmaf(p, tile_dot<false>(D, M, r, c, d), G[o]);
            }
        }
        __syncthreads();
        for (int o = threadIdx.x; o < n; o += kThreads) {
            float g = G[o] * a.coef;
            g = g < -5.0f ? -5.0f : (g > 5.0f ? 5.0f : g);  // clip(min=-5, max=5), :79
            X[o] = X[o] - g * a.lr;
        }
        __syncthreads();
    }
    for (int o = threadIdx.x; o < n; o += kThreads) {
        const int r = o / d;
        if (r < rows) a.x[(r0 + r) * d + (o % d)] = X[o];
    }
}

struct RespArgs {
    const float *x;
    const float *prec_chol;
    const float *mu_prec;
    const float *log_norm;
    float *resp;
    float *lse;  // optional [V]: log sum_k exp(weighted log prob) per row (EM's log-likelihood)
    int64_t V;
    int d;
    int K;
    const int *lower;  // MFMA path: [K], 1 if prec_chol[k] has a non-zero below the diagonal
    const float *prec_t;  // MFMA path: [K][d][d] prec_chol[k] transposed (k_transpose_sq)
    const float *prec_full;  // k_gmm_resp16t: P^T for the FULL body (prec_t = packed blocks)
};

__global__ void __launch_bounds__(kThreads) k_gmm_resp(RespArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int d = a.d;
    float *X = smem;              // [kTR][d]
    float *M = X + kTR * d;       // [d][d] prec_chol[k]
    float *LP = M + d * d;        // [kTR][64] log prob per component
    float *SQ = LP + kTR * 64;    // [kTR] squared norm accumulator
    const int64_t r0 = (int64_t)blockIdx.x * kTR;
    const int rows = (int)((a.V - r0) < kTR ? (a.V - r0) : kTR);
    const int n = kTR * d;
    for (int o = threadIdx.x; o < n; o += kThreads) {
        const int r = o / d;
        X[o] = r < rows ? a.x[(r0 + r) * d + (o % d)] : 0.0f;
    }
    for (int k = 0; k < a.K; ++k) {
        __syncthreads();
        for (int o = threadIdx.x; o < d * d; o += kThreads) M[o] = a.prec_chol[(int64_t)k * d * d + o];
        if (threadIdx.x < kTR) SQ[threadIdx.x] = 0.0f;
        __syncthreads();
        for (int o = threadIdx.x; o < n; o += kThreads) {
            const int r = o / d, c = o % d;
            const float y = tile_dot<true>(X, M, r, c, d) - a.mu_prec[k * d + c];
            atomicAdd(&SQ[r], y * y);
        }
        __syncthreads();
        if (threadIdx.x < kTR) LP[threadIdx.x * 64 + k] = a.log_norm[k] - 0.5f * SQ[threadIdx.x];
    }
    __syncthreads();
    if (threadIdx.x < kTR && threadIdx.x < rows) {
        const int r = threadIdx.x;
        float m = -INFINITY;
        for (int k = 0; k < a.K; ++k) m = fmaxf(m, LP[r * 64 + k]);
        float s = 0.0f;
        for (int k = 0; k < a.K; ++k) s += expf(LP[r * 64 + k] - m);
        const float lse = m + logf(s);
        for (int k = 0; k < a.K; ++k) a.resp[(r0 + r) * a.K + k] = expf(LP[r * 64 + k] - lse);
        if (a.lse) a.lse[r0 + r] = lse;
    }
}

// ---- MFMA community gradient (d in {64, 128}) ------------------------------------------------
//
// G = sum_k A_k M_k^T with A_k[i, :] = pi[i,k] (x_i - mu_k): one GEMM with a reduction of length
// K*d whose A operand is generated on the fly (exact fp32 fmas on the matrix cores).  A workgroup
// owns 128 rows; the `iters` loop runs in-kernel on the register-resident rows and x is written
// back once.

// ---- community gradient on 16x16x4 MFMAs, one 16-row tile per wavefront (community_async = 2) --
//
// Staging in two half images of M_k = Sigma_k^-1 (set A = columns s < D/2 and
// set B = the rest, each half staged while the other is multiplied; mu_k double-buffered), with
// the E-step's wave shape: 8 wavefronts x 16 rows per 128-row workgroup, about 90 VGPRs, so the
// two workgroups the LDS holds per CU give 4 waves per SIMD instead of 2.  MFMA (column tile ct,
// feature quad q; 4 k-steps t): A[i][k] = M_k[16 ct + i][16 q + 4 k + t] (one ds_read_b128 of
// the swizzled half image per block), B[k][j] = pi_jk (x_j - mu_k)[16 q + 4 k + t] (registers:
// the lane's row j = lane % 16 holds features 16 q + 4 (lane / 16) .. + 3 of every quad), so the
// output D[i][j] = G[row j][16 ct + i] lands in the layout x is held in: the update x -= lr *
// clip(coef G, -5, 5) happens in registers.  pi[row, k + 1] is prefetched into a register during
// component k.
template <int D>
struct Comm16 {
    static constexpr int NQ = D / 16;               // feature quads = column tiles
    static constexpr int RL = D / 8;                // 16-B granules per half-image row
    static constexpr int RPB = 16 / RL;             // rows per 256-B bank row
    static constexpr int SET = D * D / 2;           // floats per half image
    static constexpr int MUS = D * D;               // 2 x 256 floats: mu_k, double-buffered (a
                                                    // 64-lane copy writes 256 floats)
    static constexpr int LDS_FLOATS = D * D + 512;
    static constexpr int NW = 8;                    // wavefronts per workgroup
    // float offset of (row c, logical granule g of the full row) in half image g / RL
    __host__ __device__ static constexpr int at(int c, int g) {
        return (g / RL) * SET + c * RL * 4 + (((g % RL) ^ ((c / RPB) & (RL - 1))) * 4);
    }
};

// Piece i (1 KiB = ROWS rows) of half image SETI, i = wid + NW j: lane l fills row c = ROWS i + l / RL,
// physical granule l % RL, from the logical granule the swizzle puts there.  The swizzle key of
// c is the same for every j of a wavefront (NW ROWS / RPB is a multiple of RL), so one lane offset
// serves all its pieces.
template <int D, int SETI>
__device__ __forceinline__ void comm16_stage_set(const float *Mk, float *sm, int wid, int lane) {
    using C = Comm16<D>;
    constexpr int PIECES = C::SET / 256;
    constexpr int ROWS = 256 / (C::RL * 4);  // rows per 1 KiB piece
    static_assert((C::NW * ROWS / C::RPB) % C::RL == 0, "one swizzle key per wavefront");
    int ln = lane;
    asm volatile("" : "+v"(ln));  // recompute the offsets per call: hoisted, they cost 16 VGPRs
    const int c0 = wid * ROWS + ln / C::RL, pg = ln % C::RL;
    // bytes from a wavefront-uniform base: the saddr form, one VGPR for every piece
    const uint32_t loff =
        4u * (uint32_t)(c0 * D + 4 * (SETI * C::RL + (pg ^ ((c0 / C::RPB) & (C::RL - 1)))));
#pragma unroll
    for (int j = 0; j < (PIECES + C::NW - 1) / C::NW; ++j) {
        const int i = wid + C::NW * j;
        if (i >= PIECES) break;  // wavefront-uniform
        const char *base = reinterpret_cast<const char *>(Mk + j * C::NW * ROWS * D);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const float *>(base + loff),
                                         sm + SETI * C::SET + i * 256, 16, 0, 0);
    }
}

template <int D>
__device__ __forceinline__ void comm16_stage_mu(const float *mu, float *sm, int buf, int wid,
                                                int lane) {
    if (wid == 0) {
        const int src = lane * 4 < D ? lane * 4 : D - 4;
        __builtin_amdgcn_global_load_lds(mu + src, sm + Comm16<D>::MUS + buf * 256, 16, 0, 0);
    }
}

// the blocks of half H (quads q in [H NQ/2, (H+1) NQ/2), every column tile) into acc
// abase[a]: the lane's offset (floats) of granule 4 a + kg of its row j16 in column tile 0 of a
// half image; block (q, ct) adds the compile-time (q / (RL/4)) SET + 16 ct RL 4 (the swizzle depends
// on the row only through j16).
template <int D, int H>
__device__ __forceinline__ void comm16_phase(const __attribute__((ext_vector_type(4))) float (&xb)[D / 16],
                                             const float *sm, const float *mus, float p,
                                             const int (&abase)[D / 32], int kg,
                                             __attribute__((ext_vector_type(4))) float (&acc)[D / 16]) {
    using C = Comm16<D>;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    constexpr int NQ = C::NQ, HQ = NQ / 2, NB = HQ * NQ;
    f32x4 bq[HQ];
#pragma unroll
    for (int qq = 0; qq < HQ; ++qq) {
        const int q = H * HQ + qq;
        const f32x4 m = *reinterpret_cast<const f32x4 *>(mus + 16 * q + 4 * kg);
#pragma unroll
        for (int t = 0; t < 4; ++t) bq[qq][t] = p * (xb[q][t] - m[t]);
    }
    auto fetch = [&](int n) {  // block n = (qq, ct), qq-major
        const int q = H * HQ + n / NQ, ct = n % NQ;
        return *reinterpret_cast<const f32x4 *>(sm + (q / (C::RL / 4)) * C::SET +
                                                ct * 16 * C::RL * 4 + abase[q % (C::RL / 4)]);
    };
    f32x4 av[3];
    av[0] = fetch(0);
    av[1] = fetch(1);
    COME_PRIO(1);
#pragma unroll
    for (int n = 0; n < NB; ++n) {
        if (n + 2 < NB) av[(n + 2) % 3] = fetch(n + 2);
        const int qq = n / NQ, ct = n % NQ;
#pragma unroll
        for (int t = 0; t < 4; ++t)
            acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[n % 3][t], bq[qq][t], acc[ct], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    COME_PRIO(0);
}

template <int D>
__global__ void __launch_bounds__(512, 4) k_community16(CommArgs a) {
    using C = Comm16<D>;
    constexpr int NQ = C::NQ;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int tid = threadIdx.x;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int j16 = lane & 15, kg = lane >> 4;
    const int64_t row = (int64_t)blockIdx.x * 128 + wid * 16 + j16;
    const bool rowok = row < a.V;
    f32x4 xb[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q)
        xb[q] = rowok ? *reinterpret_cast<const f32x4 *>(a.x + row * D + 16 * q + 4 * kg)
                      : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    int abase[C::RL / 4];
#pragma unroll
    for (int q4 = 0; q4 < C::RL / 4; ++q4)
        abase[q4] = j16 * C::RL * 4 + 4 * ((4 * q4 + kg) ^ ((j16 / C::RPB) & (C::RL - 1)));
    for (int it = 0; it < a.iters; ++it) {
        __syncthreads();  // the previous iteration's last half image is free
        comm16_stage_set<D, 0>(a.inv_cov, sm, wid, lane);
        comm16_stage_set<D, 1>(a.inv_cov, sm, wid, lane);
        comm16_stage_mu<D>(a.mu, sm, 0, wid, lane);
        float pn = rowok ? a.pi[row * a.K] : 0.0f;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        f32x4 acc[NQ];
#pragma unroll
        for (int ct = 0; ct < NQ; ++ct) acc[ct] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        for (int k = 0; k < a.K; ++k) {
            const float p = pn;
            const float *mus = sm + C::MUS + (k & 1) * 256;
            const float *Mn = a.inv_cov + (int64_t)(k + 1) * D * D;
            comm16_phase<D, 0>(xb, sm, mus, p, abase, kg, acc);  // set A of M_k
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();  // set A free; set B of M_k in LDS
            if (k + 1 < a.K) {
                comm16_stage_set<D, 0>(Mn, sm, wid, lane);
                comm16_stage_mu<D>(a.mu + (int64_t)(k + 1) * D, sm, (k + 1) & 1, wid, lane);
                pn = rowok ? a.pi[row * a.K + k + 1] : 0.0f;
            }
            comm16_phase<D, 1>(xb, sm, mus, p, abase, kg, acc);  // set B of M_k
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();  // set B free; set A and mu of k + 1 in LDS
            if (k + 1 < a.K) comm16_stage_set<D, 1>(Mn, sm, wid, lane);
        }
        // x -= lr * clip(coef * G, -5, 5), in registers (lane: row j16, columns 16 ct + 4 kg + e)
#pragma unroll
        for (int ct = 0; ct < NQ; ++ct)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float g = acc[ct][e] * a.coef;
                g = g < -5.0f ? -5.0f : (g > 5.0f ? 5.0f : g);
                xb[ct][e] = xb[ct][e] - g * a.lr;
            }
    }
    if (rowok) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) *reinterpret_cast<f32x4 *>(a.x + row * D + 16 * q + 4 * kg) = xb[q];
    }
}

// ---- fp32 operands as bf16 parts: the arithmetic of the C4 default kernels --------------------
//
// Every fp32 operand v is carried as three bf16 parts, v1 = bf16(v), v2 = bf16(v - v1), v3 =
// bf16(v - v1 - v2): each difference is exact in fp32 and |v - v1 - v2 - v3| <= 2^-27 |v|.  A
// product a b is taken as its six part products of order <= 2 (a3 b1 + a2 b2 + a1 b3 + a2 b1 +
// a1 b2 + a1 b1; the three dropped are below 2^-26 |a b|), each exact in fp32, summed by the MFMA
// in fp32: the result carries fp32-level error (tests hold it to the fp32 kernels' tolerances),
// not a reduced-precision one.  A 16x16x32 block costs six v_mfma_f32_16x16x32_bf16 (6 x 16
// cycles) instead of eight v_mfma_f32_16x16x4_f32 (8 x 32): 2.67x the fp32 MFMA rate.
// bf16 part arithmetic on packed pairs (element 0 in the low half)
__device__ __forceinline__ uint32_t bf16_pk(float lo, float hi) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const bf16x2 v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
// (lo, hi) -> the packed first, second and third parts
__device__ __forceinline__ void bf16_split3(float lo, float hi, uint32_t &p1, uint32_t &p2,
                                            uint32_t &p3) {
    // (the empty asm hides where p1 and p2 came from: otherwise the compiler recomputes their
    // low halves with another v_cvt_pk_bf16_f32 instead of one shift)
    p1 = bf16_pk(lo, hi);
    asm("" : "+v"(p1));
    const float l2 = lo - bf16_lo(p1), h2 = hi - bf16_hi(p1);
    p2 = bf16_pk(l2, h2);
    asm("" : "+v"(p2));
    p3 = bf16_pk(l2 - bf16_lo(p2), h2 - bf16_hi(p2));
}

// ---- community gradient on bf16 parts, 16x16x32 MFMAs (k_community_b16, community_async = 3) ---
//
// One 16-row tile per wavefront, 8 wavefronts per 128-row workgroup: the fp32 kernel's wave shape
// (128 VGPRs: 4 waves per SIMD) on v_mfma_f32_16x16x32_bf16 (16 cycles).  M_k is split once per
// call (k_comm_split16); the row side pi_ik (x_i - mu_k) is split in registers at each step's head
// (the other three waves of the SIMD cover that VALU).  6.75 ms at C4 against 7.54 for the round-5
// first form (32x32x16 tiles, 32 rows per wavefront, ~216 VGPRs: 2 waves per SIMD, the next step's
// split software-pipelined), profiles/r06_ab_community_bf3.txt.  Lane (row j = lane % 16, group
// kg = lane / 16) holds features 32 s + 8 kg .. + 7 of its row for each 32-feature step s; image
// row 16 ct + i of M_k is output feature feat(), so accumulator register r of tile ct (row
// 4 kg + r) is the lane's own x[ct / 2][ct % 2][r].  One step (3 parts x D rows x 64 B, 24 KB at
// d = 128) is one staging unit, two buffers, one barrier per unit.
template <int D>
struct CommB16 {
    static constexpr int NS = D / 32;            // k-steps of 32 features = staging units
    static constexpr int CT = D / 16;            // 16-wide output column tiles
    static constexpr int PART = D * 64;          // bytes per part of a step
    static constexpr int UBYTES = 3 * PART;
    static constexpr int NW = 8;
    static constexpr int MUS = 2 * UBYTES;       // mu[2][256] after the two unit buffers
    static constexpr int LDS_BYTES = MUS + 2 * 1024;
    static constexpr int PIECES = UBYTES / 1024;
    __host__ __device__ static constexpr int feat(int rho) {
        const int ct = rho >> 4, i = rho & 15;
        return 32 * (ct >> 1) + 8 * (i >> 2) + 4 * (ct & 1) + (i & 3);
    }
    // (part P, image row rho, 16-B granule g of the step): granules swizzled by bit 2 of the row
    // (exhaustive search: conflict-free for the four 16-lane ds_read_b128 groups)
    __host__ __device__ static constexpr int at(int P, int rho, int g) {
        return P * PART + rho * 64 + 16 * (g ^ (((rho >> 2) & 1) << 1));
    }
};

template <int D>
__global__ void __launch_bounds__(256) k_comm_split16(const float *__restrict__ M,
                                                      char *__restrict__ img, int K) {
    using C = CommB16<D>;
    const int64_t n = (int64_t)K * C::NS * D * 4;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n;
         t += (int64_t)gridDim.x * 256) {
        const int g = (int)(t & 3);
        const int rho = (int)((t >> 2) % D);
        const int64_t ks = (t >> 2) / D;  // k * NS + s
        const int st = (int)(ks % C::NS);
        const int64_t k = ks / C::NS;
        const float *src = M + (k * D + C::feat(rho)) * D + 32 * st + 8 * g;
        uint4 w[3];
        uint32_t *w1 = &w[0].x, *w2 = &w[1].x, *w3 = &w[2].x;
#pragma unroll
        for (int e = 0; e < 4; ++e) bf16_split3(src[2 * e], src[2 * e + 1], w1[e], w2[e], w3[e]);
        char *ub = img + ks * C::UBYTES;
#pragma unroll
        for (int P = 0; P < 3; ++P) *reinterpret_cast<uint4 *>(ub + C::at(P, rho, g)) = w[P];
    }
}

template <int D>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
    k_community_b16(CommArgs a) {
    using C = CommB16<D>;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
    extern __shared__ __attribute__((aligned(16))) char smb[];
    const char *gimg = reinterpret_cast<const char *>(a.img);
    const int tid = threadIdx.x;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int j = lane & 15, kg = lane >> 4;
    const int64_t row = (int64_t)blockIdx.x * 128 + wid * 16 + j;
    const bool rowok = row < a.V;
    const int64_t prow = rowok ? row : a.V - 1;
    f32x4 xv[C::NS][2];  // features 32 s + 8 kg + 4 u + 0..3
#pragma unroll
    for (int s = 0; s < C::NS; ++s)
#pragma unroll
        for (int u = 0; u < 2; ++u)
            xv[s][u] = rowok ? *reinterpret_cast<const f32x4 *>(a.x + row * D + 32 * s + 8 * kg + 4 * u)
                             : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    auto stage = [&](int64_t t, int b) {
        const char *src = gimg + t * C::UBYTES + 16 * lane;
#pragma unroll
        for (int q = 0; q < (C::PIECES + C::NW - 1) / C::NW; ++q) {
            const int i = wid + C::NW * q;
            if (C::PIECES % C::NW != 0 && i >= C::PIECES) break;  // wavefront-uniform
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const float *>(src + i * 1024),
                                             reinterpret_cast<float *>(smb + b * C::UBYTES + i * 1024),
                                             16, 0, 0);
        }
    };
    auto stage_mu = [&](int c, int b) {
        if (wid == 0) {
            const int src = lane * 4 < D ? lane * 4 : D - 4;
            __builtin_amdgcn_global_load_lds(a.mu + (int64_t)c * D + src,
                                             reinterpret_cast<float *>(smb + C::MUS + b * 1024), 16,
                                             0, 0);
        }
    };
    auto mus_of = [&](int k) {
        return reinterpret_cast<const float *>(smb + C::MUS + (k & 1) * 1024);
    };
    auto split = [&](int s, const float *mus, float p, bf16x8 (&B)[3]) {
        uint32_t bw[3][4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const f32x4 m = *reinterpret_cast<const f32x4 *>(mus + 32 * s + 8 * kg + 4 * u);
            float b[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) b[e] = p * (xv[s][u][e] - m[e]);
            bf16_split3(b[0], b[1], bw[0][2 * u], bw[1][2 * u], bw[2][2 * u]);
            bf16_split3(b[2], b[3], bw[0][2 * u + 1], bw[1][2 * u + 1], bw[2][2 * u + 1]);
        }
#pragma unroll
        for (int P = 0; P < 3; ++P)
            B[P] = __builtin_bit_cast(bf16x8, uint4{bw[P][0], bw[P][1], bw[P][2], bw[P][3]});
    };
    const int aoff = C::at(0, j, kg);  // + C::at(0, 16 ct, 0): bit 2 of 16 ct + j is j's
    const int nt = a.K * C::NS;
    for (int it = 0; it < a.iters; ++it) {
        __syncthreads();  // the previous iteration's buffers are free
        stage(0, 0);
        stage(1, 1);
        stage_mu(0, 0);
        const float p0 = a.pi[prow * a.K];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        f32x4 acc[C::CT];
#pragma unroll
        for (int ct = 0; ct < C::CT; ++ct) acc[ct] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        float pn = p0;
        for (int k = 0; k < a.K; ++k) {
          const float pc = rowok ? pn : 0.0f;
          pn = a.pi[prow * a.K + min(k + 1, a.K - 1)];
#pragma unroll
          for (int s = 0; s < C::NS; ++s) {
            const int t = k * C::NS + s;
            const char *ub = smb + (s & 1) * C::UBYTES;  // t & 1 (NS is even)
            // B parts at the step's head (4 waves per SIMD cover the VALU; no second register set)
            bf16x8 Bc[3];
            split(s, mus_of(k), pc, Bc);
#pragma unroll
            for (int ct = 0; ct < C::CT; ++ct) {
                const char *base = ub + C::at(0, 16 * ct, 0) + aoff;
                bf16x8 A[3];
#pragma unroll
                for (int P = 0; P < 3; ++P) A[P] = *reinterpret_cast<const bf16x8 *>(base + P * C::PART);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2], Bc[0], acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], Bc[1], acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], Bc[2], acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], Bc[0], acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], Bc[1], acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], Bc[0], acc[ct], 0, 0, 0);
            }
            if (t + 1 < nt) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();  // buffer t & 1 free; unit t + 1 in LDS
                if (t + 2 < nt) stage(t + 2, s & 1);
                // mu_{k+1} into buffer (k + 1) & 1 (component k - 1's, done) with the unit that
                // opens component k + 1; it lands by that unit's barrier
                if (s + 2 == C::NS && k + 1 < a.K) stage_mu(k + 1, (k + 1) & 1);
            }
          }
        }
        // x -= lr * clip(coef * G, -5, 5): register r of tile ct is x[ct / 2][ct % 2][r]
#pragma unroll
        for (int ct = 0; ct < C::CT; ++ct)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float g = acc[ct][r] * a.coef;
                g = g < -5.0f ? -5.0f : (g > 5.0f ? 5.0f : g);
                xv[ct >> 1][ct & 1][r] -= g * a.lr;
            }
    }
    if (rowok) {
#pragma unroll
        for (int s = 0; s < C::NS; ++s)
#pragma unroll
            for (int u = 0; u < 2; ++u)
                *reinterpret_cast<f32x4 *>(a.x + row * D + 32 * s + 8 * kg + 4 * u) = xv[s][u];
    }
}

// GMM responsibilities, shared steps.  Triangular skip: sklearn's precisions_cholesky_ after an
// M-step is UPPER triangular (solve_triangular(chol(cov), I, lower=True).T), so a column tile of
// Y = X P_k only needs the features up to its last column.  k_gmm_lower_flags marks the components
// with a non-zero below the diagonal (a lower factor, e.g. sklearn's cholesky(precisions_init,
// lower=True)) and ORs them into flags[K]; a launch holding one runs the full-body kernel
// (k_gmm_resp16_full) instead of the skipping one.  The skipped MFMAs would only add exact zeros.
__global__ void __launch_bounds__(256) k_gmm_lower_flags(const float *__restrict__ P, int D,
                                                         int *__restrict__ flags, int K) {
    const float *Pk = P + (int64_t)blockIdx.x * D * D;
    int nz = 0;
    for (int o = threadIdx.x; o < D * D; o += 256) nz |= (o / D > o % D) && Pk[o] != 0.0f;
    nz = __syncthreads_or(nz);
    if (threadIdx.x == 0) {
        flags[blockIdx.x] = nz ? 1 : 0;
        if (nz) atomicOr(flags + K, 1);  // flags[K]: some component is not upper-triangular
    }
}

// Pt[k][c][s] = P[k][s][c] (one D x D matrix per blockIdx.y, 32 x 32 tiles through LDS)
__global__ void __launch_bounds__(256) k_transpose_sq(const float *__restrict__ P, int D,
                                                      float *__restrict__ Pt) {
    __shared__ float t[32][33];
    const int tiles = D / 32;
    const int tr = blockIdx.x / tiles, tc = blockIdx.x % tiles;
    const float *src = P + (int64_t)blockIdx.y * D * D;
    float *dst = Pt + (int64_t)blockIdx.y * D * D;
    const int x = threadIdx.x & 31, y0 = threadIdx.x >> 5;
    for (int y = y0; y < 32; y += 8) t[y][x] = src[(int64_t)(tr * 32 + y) * D + tc * 32 + x];
    __syncthreads();
    for (int y = y0; y < 32; y += 8) dst[(int64_t)(tc * 32 + y) * D + tr * 32 + x] = t[x][y];
}

// ---- E-step on v_mfma_f32_16x16x4_f32: the FULL body (k_gmm_resp16_full) ------------------
//
// Y^T = P_k^T X^T per 16 x 16 tile: A = P_k^T (lane: column c = ct*16 + lane%16, features
// 16q + 4 (lane/16) + t), B = X^T (lane: row = rt*16 + lane%16, the same features), so the four
// k-slots of an MFMA step t are features 16q + {0, 4, 8, 12} + t and each lane's A operands for
// the four steps of quad q are ONE ds_read_b128 (its B operands one f32x4 register).  The output
// lane holds column 4 (lane/16) + e of row lane%16, so a row's sum of squares is the lane's own
// 4 x CT values plus two cross-lane adds (lane ^ 16, lane ^ 32) -- no reduce-scatter.
// 16-wide blocks skip more of sklearn's upper precision factor than 32-wide ones: block (quad q,
// column tile ct) is non-zero iff q <= ct, 36 of 64 blocks at d = 128 (0.5625 of the dense MFMA
// cycles; 32-wide blocks: 10 of 16 = 0.625), at the same fp32 rate (32 cycles per
// 16x16x4 MFMA = 64 per 32x32x2, half the flops).
// A workgroup = 4 wavefronts x 32 rows (RT = 2 row tiles), two workgroups per CU.  P_k^T lives in
// LDS as two half images of D rows x D/2 features; half 0 holds quads {0 .. NQ/4-1} and
// {3NQ/4 .. NQ-1}, half 1 the middle ones, so both phases of a component run the same number of
// MFMAs (18 + 18 (quad, tile) blocks at d = 128; a plain split of the features: 112 vs 48 MFMAs).
// The next component's half is copied global -> LDS (global_load_lds) while the other half
// computes.  Rows of an image are 16-B granules XOR-swizzled by the row
// (granule g of row r at g ^ (r % granules)): conflict-free ds_read_b128 without padding.
template <int D>
struct Resp16Shape {
    static constexpr int NQ = D / 16;        // feature quads = column tiles
    static constexpr int HQ = NQ / 2;        // quads per half image
    static constexpr int GR = HQ * 4;        // 16-B granules per half-image row
    static constexpr int HIMG = D * GR * 4;  // floats per half image
    static constexpr int MP = 2 * HIMG;      // mu_k P_k (D floats, 256 reserved)
    static constexpr int PARAMS = MP + 256;  // lower flag, log_norm (64 reserved)
    static constexpr int LDS = PARAMS + 64;  // floats
    static_assert(HIMG % 256 == 0, "a half image is a whole number of 1 KiB copies");
};

// the quad held at position p of half image h
template <int D>
__host__ __device__ constexpr int r16_quad(int h, int p) {
    return h == 0 ? (p < D / 64 ? p : p + D / 32) : p + D / 64;
}

// Per-lane source offsets (floats, within one D x D matrix) of the 1 KiB pieces wavefront `wid`
// copies for half image h: piece i = wid + 4 j holds granules 64 i .. 64 i + 63 of the image.
template <int D>
struct R16Stage {
    static constexpr int PIECES = Resp16Shape<D>::HIMG / 256;
    static constexpr int PER_WAVE = (PIECES + 3) / 4;
    uint32_t off[2][PER_WAVE];  // bytes: a 32-bit vector offset from a scalar base
    __device__ __forceinline__ R16Stage(int wid, int lane) {
        using RS = Resp16Shape<D>;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < PER_WAVE; ++j) {
                const int g = (wid + 4 * j) * 64 + lane;
                const int r = g / RS::GR, logical = (g % RS::GR) ^ (r & (RS::GR - 1));
                off[h][j] = 4u * (uint32_t)(r * D + 16 * r16_quad<D>(h, logical >> 2) +
                                            4 * (logical & 3));
            }
    }
    // copy half image h of P_k^T (4 wavefronts, 1 KiB per instruction)
    __device__ __forceinline__ void half(const float *Ptk, float *sm, int h, int wid) const {
#pragma unroll
        for (int j = 0; j < PER_WAVE; ++j) {
            const int i = wid + 4 * j;
            if (i >= PIECES) break;  // wavefront-uniform
            __builtin_amdgcn_global_load_lds(
                reinterpret_cast<const float *>(reinterpret_cast<const char *>(Ptk) + off[h][j]),
                sm + h * Resp16Shape<D>::HIMG + i * 256, 16, 0, 0);
        }
    }
};

// F: the calling body's FULL (one instantiation per body: the host pass of hipcc rejects a
// second host-side use of a device template holding global_load_lds)
template <int D, bool F>
__device__ __forceinline__ void r16_stage_mp(const float *mp, float *sm, int wid, int lane) {
    if (wid == 0) {
        const int src = lane * 4 < D ? lane * 4 : D - 4;
        __builtin_amdgcn_global_load_lds(mp + src, sm + Resp16Shape<D>::MP, 16, 0, 0);
    }
}

template <int D, bool F>
__device__ __forceinline__ void r16_stage_params(const RespArgs &a, int k, float *sm, int wid,
                                                 int lane) {
    if (wid == 0) {
        const float *src = lane == 0 ? reinterpret_cast<const float *>(a.lower + k)
                                     : a.log_norm + k;
        __builtin_amdgcn_global_load_lds(src, sm + Resp16Shape<D>::PARAMS, 4, 0, 0);
    }
}

// Blocks (position p in half image H, column tile ct) of one phase in issue order: every tile
// of a quad (FULL: a lower or dense factor) or only ct >= q (upper factor).
template <int D>
constexpr int r16_nblk(int H, bool full) {
    int n = 0;
    for (int p = 0; p < D / 32; ++p) n += full ? D / 16 : D / 16 - r16_quad<D>(H, p);
    return n;
}
template <int D>
constexpr int r16_blk(int H, bool full, int n, bool want_ct) {
    for (int p = 0; p < D / 32; ++p)
        for (int ct = full ? 0 : r16_quad<D>(H, p); ct < D / 16; ++ct)
            if (n-- == 0) return want_ct ? ct : p;
    return 0;
}

// One phase: the blocks of half image H on both row tiles.  Per block one ds_read_b128 of A
// operands (four k-steps) feeds 8 MFMAs (4 steps x 2 row tiles, two independent accumulation
// chains); A operands are read two blocks ahead (a 3-slot ring: few VGPRs).
// abase[p] = the lane's offset (floats) of its A operands for position p in an image's first
// column tile; tile ct adds ct * 16 rows (a compile-time immediate: the XOR swizzle depends on
// the row only through row % granules = j16 % granules).
template <int D, bool FULL, int H>
__device__ __forceinline__ void r16_phase(
    const __attribute__((ext_vector_type(4))) float (&xb)[2][D / 16], const float *sm,
    const int (&abase)[D / 32], __attribute__((ext_vector_type(4))) float (&acc)[2][D / 16]) {
    using RS = Resp16Shape<D>;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    constexpr int NB = r16_nblk<D>(H, FULL);
    const float *img = sm + H * RS::HIMG;
    auto fetch = [&](int n) {
        const int p = r16_blk<D>(H, FULL, n, false), ct = r16_blk<D>(H, FULL, n, true);
        return *reinterpret_cast<const f32x4 *>(img + abase[p] + ct * 16 * (RS::GR * 4));
    };
    f32x4 av[3];
    av[0] = fetch(0);
    if (NB > 1) av[1] = fetch(1);
#pragma unroll
    for (int n = 0; n < NB; ++n) {
        if (n + 2 < NB) av[(n + 2) % 3] = fetch(n + 2);
        const int ct = r16_blk<D>(H, FULL, n, true);
        const int q = r16_quad<D>(H, r16_blk<D>(H, FULL, n, false));
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
                acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[n % 3][t], xb[rt][q][t],
                                                                   acc[rt][ct], 0, 0, 0);
        // keep the ring: no A read hoisted above its block (the scheduler would otherwise
        // cluster every read of the phase at its head and spill)
        __builtin_amdgcn_sched_barrier(0);
    }
}

// FULL: every component runs every (quad, tile) block -- the launch holds some lower or dense
// factor (flags[K], k_gmm_lower_flags); else the upper-triangular skip for all components.
template <int D, bool FULL>
__device__ __forceinline__ void r16_body(const RespArgs &a, float *sm, int64_t blk) {
    using RS = Resp16Shape<D>;
    constexpr int NQ = RS::NQ;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    const int tid = threadIdx.x;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int j16 = lane & 15, kg = lane >> 4;
    const int64_t row0 = blk * 128 + wid * 32;
    f32x4 xb[2][NQ];  // xb[rt][q][t] = x[row0 + 16 rt + j16][16 q + 4 kg + t]
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
        const int64_t row = row0 + 16 * rt + j16;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            xb[rt][q] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
            if (row < a.V) xb[rt][q] = *reinterpret_cast<const f32x4 *>(a.x + row * D + 16 * q + 4 * kg);
        }
    }
    const R16Stage<D> stage(wid, lane);
    stage.half(a.prec_t, sm, 0, wid);
    stage.half(a.prec_t, sm, 1, wid);
    r16_stage_mp<D, FULL>(a.mu_prec, sm, wid, lane);
    r16_stage_params<D, FULL>(a, 0, sm, wid, lane);
    int abase[RS::HQ];
#pragma unroll
    for (int p = 0; p < RS::HQ; ++p)
        abase[p] = j16 * (RS::GR * 4) + 4 * ((4 * p + kg) ^ (j16 & (RS::GR - 1)));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // lanes 0-15 own row tile 0, lanes 16-31 row tile 1 (the others hold copies)
    const int64_t my_row = row0 + 16 * (kg & 1) + j16;
    const bool owner = kg < 2 && my_row < a.V;
    float run_max = -INFINITY, run_sum = 0.0f;
    for (int k = 0; k < a.K; ++k) {
        const int kn = k + 1;
        const float lnk = sm[RS::PARAMS + 1];
        const float *Pn = a.prec_t + (int64_t)kn * D * D;
        f32x4 acc[2][NQ];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int ct = 0; ct < NQ; ++ct) acc[rt][ct] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        r16_phase<D, FULL, 0>(xb, sm, abase, acc);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // half 0 and the params free; half 1 and mu_k P_k in LDS
        if (k + 1 < a.K) {
            stage.half(Pn, sm, 0, wid);
            r16_stage_params<D, FULL>(a, kn, sm, wid, lane);
        }
        r16_phase<D, FULL, 1>(xb, sm, abase, acc);
        float sq[2] = {0.0f, 0.0f};
#pragma unroll
        for (int ct = 0; ct < NQ; ++ct) {
            const f32x4 mp = *reinterpret_cast<const f32x4 *>(sm + RS::MP + ct * 16 + 4 * kg);
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float y = acc[rt][ct][e] - mp[e];
                    sq[rt] = __builtin_fmaf(y, y, sq[rt]);
                }
        }
        // each row's columns are spread over the 4 lane groups: sum them for both row tiles
        const float tot0 = reduce_stage<5>(reduce_stage<4>(sq[0]));
        const float tot1 = reduce_stage<5>(reduce_stage<4>(sq[1]));
        const float tot = (kg & 1) ? tot1 : tot0;
        const float lp = lnk - 0.5f * tot;
        if (owner) a.resp[my_row * a.K + k] = lp;
        if (lp > run_max) {  // online log-sum-exp of the row's components so far
            run_sum = run_sum * expf(run_max - lp) + 1.0f;
            run_max = lp;
        } else {
            run_sum += expf(lp - run_max);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // half 1 and mu_k P_k free; half 0 of P_{k+1} in LDS
        if (k + 1 < a.K) {
            stage.half(Pn, sm, 1, wid);
            r16_stage_mp<D, FULL>(a.mu_prec + (int64_t)kn * D, sm, wid, lane);
        }
    }
    if (owner) {
        float *lp = a.resp + my_row * a.K;
        const float lse = run_max + logf(run_sum);
        for (int k = 0; k < a.K; ++k) lp[k] = expf(lp[k] - lse);
        if (a.lse) a.lse[my_row] = lse;
    }
}

// ---- k_gmm_resp16 on packed upper factors: one barrier per component ---------------------------
//
// When every factor of the launch is upper-triangular (sklearn's precisions_cholesky_), only the
// 36 non-zero 16 x 16 blocks of P_k^T are kept (k_pack_upper16): per quad q the rows c >= 16 q,
// 16 features each -- 36 KB instead of 64 KB at d = 128 -- so a workgroup double-buffers WHOLE
// components (2 x 37.3 KB, two workgroups per CU): component k + 1 is copied global -> LDS while
// k computes, and each component ends with ONE barrier instead of two (k_gmm_resp16's half
// images).  The copy is a straight 1 KiB-per-instruction memcpy of the packed image (the swizzle
// is applied by the pack kernel): granule g of row c's 16 features sits at g ^ ((c >> 1) & 2),
// conflict-free for the A-operand ds_read_b128 (lane groups of 16 rows x one granule).
template <int D>
struct Resp16T {
    static constexpr int NQ = D / 16;
    static constexpr int TRI = 16 * 16 * NQ * (NQ + 1) / 2;  // floats of the packed blocks
    static constexpr int MP = 0;                              // in a slot: mu_k P_k (256 reserved)
    static constexpr int PAR = 256;                           // lower flag, log_norm (64 reserved)
    static constexpr int SLOT = 256 + 64;                     // floats per parameter slot
    static constexpr int LDS = 2 * (TRI + SLOT);              // two buffers
    __device__ static float *blocks(float *sm, int k) { return sm + (k & 1) * TRI; }
    __device__ static float *slot(float *sm, int k) { return sm + 2 * TRI + (k & 1) * SLOT; }
    static constexpr int PIECES = TRI / 256;
    static_assert(TRI % 256 == 0, "whole 1 KiB pieces");
    // offset of quad q's first row block: 16 floats x sum_{q' < q} (D - 16 q') rows
    static constexpr int off(int q) { return 16 * (16 * q * NQ - 8 * q * (q - 1)); }
};

// packed[k][off(q) + (c - 16q) * 16 + 4 (g ^ ((c >> 1) & 2)) + i] = P[k][16q + 4g + i][c], c >= 16q
template <int D>
__global__ void __launch_bounds__(256) k_pack_upper16(const float *__restrict__ P,
                                                      float *__restrict__ packed) {
    using T = Resp16T<D>;
    const float *Pk = P + (int64_t)blockIdx.y * D * D;
    float *out = packed + (int64_t)blockIdx.y * T::TRI;
    for (int o = blockIdx.x * 256 + threadIdx.x; o < T::TRI; o += gridDim.x * 256) {
        int q = 0;
        while (q + 1 < T::NQ && o >= T::off(q + 1)) ++q;
        const int rel = o - T::off(q);
        const int c = 16 * q + rel / 16, slot = rel % 16;
        const int g = (slot / 4) ^ ((c >> 1) & 2), i = slot % 4;
        out[o] = Pk[(16 * q + 4 * g + i) * D + c];
    }
}

// One 16-row tile per wavefront, 8 wavefronts per 128-row workgroup (91-95 VGPRs: 4 waves per
// SIMD -- the LDS holds two workgroups per CU either way); two row tiles per wavefront and 4
// wavefronts (216 VGPRs, 2 waves per SIMD) were bit-identical and 1.5% slower (7.10 vs 7.00 ms).
// (16 wavefronts = 256-row workgroups, one per CU, half the component copies per row: 7.37 vs
// 7.00 ms -- the second workgroup's cover at barriers is worth more; profiles/r05_ab_gmm_diag.txt)
struct R16tShape {
    static constexpr int NW = 8;                 // wavefronts per workgroup
    static constexpr int ROWS = 16 * NW;         // rows per workgroup (128)
    static constexpr int THREADS = 64 * NW;
    static constexpr int WPE = 4;                // waves per SIMD the registers must allow
};

// component k's packed blocks into `buf`, its mu_k P_k, lower flag and log_norm into `par` (NW
// wavefronts share the 1 KiB copies)
template <int D>
__device__ __forceinline__ void r16t_stage(const RespArgs &a, int k, float *buf, float *par,
                                           int wid, int lane) {
    using T = Resp16T<D>;
    constexpr int NW = R16tShape::NW;
    const float *src = a.prec_t + (int64_t)k * T::TRI;  // the packed blocks in this body
#pragma unroll
    for (int j = 0; j < (T::PIECES + NW - 1) / NW; ++j) {
        const int i = wid + NW * j;
        if (i >= T::PIECES) break;  // wavefront-uniform
        __builtin_amdgcn_global_load_lds(src + i * 256 + lane * 4, buf + i * 256, 16, 0, 0);
    }
    if (wid == 0) {
        const int s = lane * 4 < D ? lane * 4 : D - 4;
        __builtin_amdgcn_global_load_lds(a.mu_prec + (int64_t)k * D + s, par + T::MP, 16, 0, 0);
    } else if (wid == 1) {
        const float *p = lane == 0 ? reinterpret_cast<const float *>(a.lower + k)
                                   : a.log_norm + k;
        __builtin_amdgcn_global_load_lds(p, par + T::PAR, 4, 0, 0);
    }
}

// piece j of r16t_stage's copy (j = 0 also copies mu_k P_k and the parameters), for the copy
// spread over the MFMA stream (k_gmm_resp16t)
template <int D>
__device__ __forceinline__ void r16t_stage_piece(const RespArgs &a, int k, float *buf, float *par,
                                                 int wid, int lane, int j) {
    using T = Resp16T<D>;
    constexpr int NW = R16tShape::NW;
    const float *src = a.prec_t + (int64_t)k * T::TRI;
    const int i = wid + NW * j;
    if (i < T::PIECES)  // wavefront-uniform
        __builtin_amdgcn_global_load_lds(src + i * 256 + lane * 4, buf + i * 256, 16, 0, 0);
    if (j == 0 && wid == 0) {
        const int s = lane * 4 < D ? lane * 4 : D - 4;
        __builtin_amdgcn_global_load_lds(a.mu_prec + (int64_t)k * D + s, par + T::MP, 16, 0, 0);
    } else if (j == 0 && wid == 1) {
        const float *p = lane == 0 ? reinterpret_cast<const float *>(a.lower + k)
                                   : a.log_norm + k;
        __builtin_amdgcn_global_load_lds(p, par + T::PAR, 4, 0, 0);
    }
}

// Block n of the upper triangle in row-major order (q, ct >= q), as compile-time tables.
template <int NQ>
struct TriBlocks {
    static constexpr int NB = NQ * (NQ + 1) / 2;
    int q[NB], ct[NB];
    constexpr TriBlocks() : q(), ct() {
        int n = 0;
        for (int a = 0; a < NQ; ++a)
            for (int b = a; b < NQ; ++b) {
                q[n] = a;
                ct[n] = b;
                ++n;
            }
    }
};

// All 36 (d = 128) upper blocks of one component on the wavefront's row tile, in row-major order
// (q, ct >= q); A operands read two blocks ahead through a 3-slot ring.  (Measured and not kept:
// blocks in pairs with interleaved accumulation chains +0.5%; the next component's staging issued
// behind the first A reads 0; a packed-fp32 epilogue 0; the accumulators started at -mu_k P_k and
// the log-sum-exp after the loop: no gain -- profiles/r04_ab_estep16.txt.)
template <int D, typename Hook>
__device__ __forceinline__ void r16t_blocks(
    const __attribute__((ext_vector_type(4))) float (&xb)[D / 16], const float *buf, int abase,
    __attribute__((ext_vector_type(4))) float (&acc)[D / 16], Hook &&hook) {
    using T = Resp16T<D>;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    constexpr int NQ = T::NQ;
    constexpr int NB = NQ * (NQ + 1) / 2;
    constexpr TriBlocks<NQ> TB{};
    auto fetch = [&](int n) {
        return *reinterpret_cast<const f32x4 *>(buf + T::off(TB.q[n]) + (TB.ct[n] - TB.q[n]) * 256 +
                                                abase);
    };
    f32x4 av[3];
    av[0] = fetch(0);
    av[1] = fetch(1);
    COME_PRIO(1);
#pragma unroll
    for (int n = 0; n < NB; ++n) {
        if (n + 2 < NB) av[(n + 2) % 3] = fetch(n + 2);
        hook(n);  // other work placed beside this block's MFMAs
        const int q = TB.q[n], ct = TB.ct[n];
        // quad 0's blocks (n < NQ) start acc[ct] from zero: the accumulator is born here
        if (q == 0) acc[ct] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int t = 0; t < 4; ++t)
            acc[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[n % 3][t], xb[q][t], acc[ct], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    COME_PRIO(0);
}

// the epilogue of one component: sq += |acc[ct] - (mu_k P_k)[ct]|^2 over the column tiles ct in
// order, then log N(x_row; mu_k, P_k) = log_norm_k - sq / 2 summed over the lane groups
template <int D>
__device__ __forceinline__ void r16t_sq(const __attribute__((ext_vector_type(4))) float &acc,
                                        const float *par, int ct, int kg, float &sq) {
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    const f32x4 mp = *reinterpret_cast<const f32x4 *>(par + Resp16T<D>::MP + ct * 16 + 4 * kg);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float y = acc[e] - mp[e];
        sq = __builtin_fmaf(y, y, sq);
    }
}
template <int D>
__device__ __forceinline__ float r16t_lp_of(float sq, const float *par) {
    return par[Resp16T<D>::PAR + 1] - 0.5f * reduce_stage<5>(reduce_stage<4>(sq));
}

// online log-sum-exp step
__device__ __forceinline__ void lse_push(float lp, float &run_max, float &run_sum) {
    if (lp > run_max) {
        run_sum = run_sum * expf(run_max - lp) + 1.0f;
        run_max = lp;
    } else {
        run_sum += expf(lp - run_max);
    }
}

// The default E-step when every factor of the launch is upper-triangular (flags[K] == 0); a
// launch holding a lower or dense factor returns at once and k_gmm_resp16_full (launched after it)
// runs every block.  prec_t points to the packed blocks, prec_full to P^T.
template <int D>
__global__ void __launch_bounds__(R16tShape::THREADS, R16tShape::WPE) k_gmm_resp16t(RespArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    if (__builtin_amdgcn_readfirstlane(a.lower[a.K]) != 0) return;
    using T = Resp16T<D>;
    constexpr int NQ = T::NQ;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    const int tid = threadIdx.x;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int j16 = lane & 15, kg = lane >> 4;
    const int64_t row0 = (int64_t)blockIdx.x * R16tShape::ROWS + wid * 16;
    f32x4 xb[NQ];  // xb[q][t] = x[row0 + j16][16 q + 4 kg + t]
    {
        const int64_t row = row0 + j16;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            xb[q] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
            if (row < a.V) xb[q] = *reinterpret_cast<const f32x4 *>(a.x + row * D + 16 * q + 4 * kg);
        }
    }
    r16t_stage<D>(a, 0, T::blocks(sm, 0), T::slot(sm, 0), wid, lane);
    // the lane's A operands of block (q, ct): row ct*16 + j16 of quad q's row block
    const int abase = j16 * 16 + 4 * (kg ^ ((j16 >> 1) & 2));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int64_t my_row = row0 + j16;  // lanes 0-15 own the tile's rows
    const bool owner = kg == 0 && my_row < a.V;
    float run_max = -INFINITY, run_sum = 0.0f, lp_prev = 0.0f;
    for (int k = 0; k < a.K; ++k) {
        const int kb = COME_RESP_DIAG >= 3 ? 0 : k;  // the buffer read
        // component k - 1's log-probability is stored one component late: a store counts on the
        // vector-memory counter like the staging copies, so storing it right before the barrier's
        // vmcnt(0) made every wavefront wait out the store's round trip once per component
        if (k > 0 && owner) a.resp[my_row * a.K + k - 1] = lp_prev;
        const float *par = T::slot(sm, kb);
        f32x4 acc[NQ];
        // component k + 1's copy (4-5 1-KiB LDS-DMA pieces per wavefront at d = 128) issued one
        // piece every SP blocks from block 3 instead of all at the component's head, where they sat
        // on the MFMA ramp: 6.95 vs 7.01 ms at C4 (SP = 7) (spacing 2 / 4 / 8 / 6 from block 4: 7.01 / 6.99 / 6.99 /
        // 6.95; profiles/r05_ab_gmm_diag.txt)
        r16t_blocks<D>(xb, T::blocks(sm, kb), abase, acc, [&](int n) {
            constexpr int NB = T::NQ * (T::NQ + 1) / 2, OFF = 3;
            constexpr int PER = (T::PIECES + R16tShape::NW - 1) / R16tShape::NW;
            constexpr int SP = (NB - OFF + PER - 1) / PER;  // 7 at d = 128, 4 at d = 64
            static_assert(OFF + SP * (PER - 1) < NB, "every piece lands on a block");
            const int m = n - OFF;
            if (!COME_RESP_DIAG && m >= 0 && m % SP == 0 && m / SP < PER && k + 1 < a.K)
                r16t_stage_piece<D>(a, k + 1, T::blocks(sm, k + 1), T::slot(sm, k + 1), wid, lane,
                                    m / SP);
        });
        float sq = 0.0f;
#pragma unroll
        for (int ct = 0; ct < NQ; ++ct) r16t_sq<D>(acc[ct], par, ct, kg, sq);
        const float lp = r16t_lp_of<D>(sq, par);
        lse_push(lp, run_max, run_sum);
        lp_prev = lp;
#if COME_RESP_DIAG != 2 && COME_RESP_DIAG != 4
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // buffer k & 1 free; component k + 1 in the other buffer
#endif
    }
    if (owner) {
        float *lp = a.resp + my_row * a.K;
        lp[a.K - 1] = lp_prev;
        const float lse = run_max + logf(run_sum);
        for (int k = 0; k < a.K; ++k) lp[k] = expf(lp[k] - lse);
        if (a.lse) a.lse[my_row] = lse;
    }
}

// ---- E-step on bf16 parts, 16x16x32 MFMAs (k_gmm_resp_b16, gmm_resp16 = 3) -------------------
//
// The bf16-part arithmetic (fp32 operands as three bf16 parts, six exact part products per
// multiply-add, summed in fp32) on Y = X P_k: output D[i][j] = Y[row j][16 ct + i], A = P_k^T parts
// (LDS), B = the row's x parts -- x does not change over the components, so the row side is split
// ONCE per workgroup, not per component (the community step's VALU cost).  Upper factors only
// (sklearn's precisions_cholesky_); a launch holding a lower or dense factor returns at once and
// k_gmm_resp16_full runs it.  k_community_b16's wave shape: one 16-row tile per wavefront, 8
// wavefronts per 128-row workgroup, the row's parts (48 VGPRs) formed once, 128 VGPRs: 4 waves
// per SIMD.  A component is staged in two units of 10 blocks, mu_k P_k and log_norm_k beside the
// first; each tile's first MFMA starts from the constant 0 and its squared residuals are summed as
// soon as its last block completes.  4.12 ms at C4 against 4.54 for the round-5 first form
// (32x32x16 tiles, 32 rows per wavefront, 2 waves per SIMD, A parts read one block ahead; removed),
// profiles/r06_ab_estep_bf3.txt.
// Block (16-wide column tile ct, 32-feature step s) of P_k^T is non-zero iff s <= ct / 2: 20 of 32
// at d = 128 (6 of 8 at 64), each a 3 KiB image (3 parts x 16 rows x 64 B, granules swizzled by
// bit 2 of the row as CommB16::at).  Lane (row j, group kg) holds columns 16 ct + 4 kg .. + 3 of
// its row per tile: a row's sum of squares is 4 x (tiles) in-lane FMAs and two permlane swaps.
template <int D>
struct RespB16 {
    static constexpr int NS = D / 32, CT = D / 16;
    static constexpr int NB = CT == 8 ? 20 : 6;     // sum over ct of ct / 2 + 1
    static constexpr int BLK = 3 * 1024;
    static constexpr int NW = 8, NU = 2;
    static constexpr int UB = NB / NU, UBYTES = UB * BLK;
    static constexpr int PAR = 2 * UBYTES, PARF = 256 + 64;
    static constexpr int LDS_BYTES = PAR + 2 * PARF * 4;
    static constexpr int PIECES = UBYTES / 1024;
    int ct[NB], s[NB];
    constexpr RespB16() : ct(), s() {
        int n = 0;
        for (int c = 0; c < CT; ++c)
            for (int k = 0; k <= c / 2; ++k) {
                ct[n] = c;
                s[n] = k;
                ++n;
            }
    }
    __host__ __device__ static constexpr int at(int P, int i, int g) {
        return P * 1024 + i * 64 + 16 * (g ^ (((i >> 2) & 1) << 1));
    }
};

template <int D>
__global__ void __launch_bounds__(256) k_pack_upper_b16(const float *__restrict__ P,
                                                        char *__restrict__ img, int K) {
    using R = RespB16<D>;
    constexpr R TB{};
    const int64_t n = (int64_t)K * R::NB * 16 * 4;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n;
         t += (int64_t)gridDim.x * 256) {
        const int g = (int)(t & 3), i = (int)((t >> 2) & 15);
        const int64_t kb = t >> 6;  // k * NB + block
        const int b = (int)(kb % R::NB);
        const int64_t k = kb / R::NB;
        const int c = 16 * TB.ct[b] + i, f0 = 32 * TB.s[b] + 8 * g;
        const float *Pk = P + k * D * D;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = Pk[(int64_t)(f0 + e) * D + c];  // P^T[c][f] = P[f][c]
        uint4 w[3];
        uint32_t *w1 = &w[0].x, *w2 = &w[1].x, *w3 = &w[2].x;
#pragma unroll
        for (int e = 0; e < 4; ++e) bf16_split3(v[2 * e], v[2 * e + 1], w1[e], w2[e], w3[e]);
        char *blk = img + kb * R::BLK;
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<uint4 *>(blk + R::at(p, i, g)) = w[p];
    }
}

template <int D>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
    k_gmm_resp_b16(RespArgs a) {
    using R = RespB16<D>;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
    extern __shared__ __attribute__((aligned(16))) char smb[];
    if (__builtin_amdgcn_readfirstlane(a.lower[a.K]) != 0) return;
    constexpr R TB{};
    const char *gimg = reinterpret_cast<const char *>(a.prec_t);
    const int tid = threadIdx.x;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int j = lane & 15, kg = lane >> 4;
    const int64_t row = (int64_t)blockIdx.x * 128 + wid * 16 + j;
    const bool rowok = row < a.V;
    const int nt = a.K * R::NU;
    // unit t -> buffer b; a component's first unit also brings its mu_k P_k and log_norm_k
    auto stage = [&](int64_t t, int b) {
        const char *src = gimg + t * R::UBYTES + 16 * lane;
#pragma unroll
        for (int q = 0; q < (R::PIECES + R::NW - 1) / R::NW; ++q) {
            const int i = wid + R::NW * q;
            if (R::PIECES % R::NW != 0 && i >= R::PIECES) break;  // wavefront-uniform
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const float *>(src + i * 1024),
                                             reinterpret_cast<float *>(smb + b * R::UBYTES + i * 1024),
                                             16, 0, 0);
        }
        if (t % R::NU == 0) {
            const int64_t k = t / R::NU;
            float *par = reinterpret_cast<float *>(smb + R::PAR) + (k & 1) * R::PARF;
            if (wid == 0) {
                const int s = lane * 4 < D ? lane * 4 : D - 4;
                __builtin_amdgcn_global_load_lds(a.mu_prec + k * D + s, par, 16, 0, 0);
            } else if (wid == 1) {
                __builtin_amdgcn_global_load_lds(a.log_norm + k, par + 256, 4, 0, 0);
            }
        }
    };
    stage(0, 0);
    if (nt > 1) stage(1, 1);
    // the row's parts, once: xp[s][P] = part P of features 32 s + 8 kg .. + 7
    bf16x8 xp[R::NS][3];
#pragma unroll
    for (int s = 0; s < R::NS; ++s) {
        uint32_t w[3][4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            f32x4 v = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
            if (rowok) v = *reinterpret_cast<const f32x4 *>(a.x + row * D + 32 * s + 8 * kg + 4 * u);
            bf16_split3(v[0], v[1], w[0][2 * u], w[1][2 * u], w[2][2 * u]);
            bf16_split3(v[2], v[3], w[0][2 * u + 1], w[1][2 * u + 1], w[2][2 * u + 1]);
        }
#pragma unroll
        for (int P = 0; P < 3; ++P)
            xp[s][P] = __builtin_bit_cast(bf16x8, uint4{w[P][0], w[P][1], w[P][2], w[P][3]});
    }
    const int aoff = R::at(0, j, kg);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const bool owner = kg == 0 && rowok;
    float run_max = -INFINITY, run_sum = 0.0f, lp_prev = 0.0f;
    for (int k = 0; k < a.K; ++k) {
        if (k > 0 && owner) a.resp[row * a.K + k - 1] = lp_prev;  // one component late
        const float *par = reinterpret_cast<const float *>(smb + R::PAR) + (k & 1) * R::PARF;
        float sq = 0.0f;
        f32x4 acc[R::CT];
#pragma unroll
        for (int u = 0; u < R::NU; ++u) {
            const int t = k * R::NU + u;
            const char *ub = smb + (u & 1) * R::UBYTES;  // t & 1
#pragma unroll
            for (int bi = 0; bi < R::UB; ++bi) {
                const int b = u * R::UB + bi, ct = TB.ct[b], s = TB.s[b];
                const char *base = ub + bi * R::BLK + aoff;
                bf16x8 A[3];
#pragma unroll
                for (int P = 0; P < 3; ++P) A[P] = *reinterpret_cast<const bf16x8 *>(base + P * 1024);
                const f32x4 c0 = s == 0 ? f32x4{0.0f, 0.0f, 0.0f, 0.0f} : acc[ct];
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2], xp[s][0], c0, 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], xp[s][1], acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], xp[s][2], acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], xp[s][0], acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], xp[s][1], acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], xp[s][0], acc[ct], 0, 0, 0);
                if (s == ct / 2) {  // tile ct complete: columns 16 ct + 4 kg + r
                    const f32x4 mp = *reinterpret_cast<const f32x4 *>(par + 16 * ct + 4 * kg);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float y = acc[ct][r] - mp[r];
                        sq = __builtin_fmaf(y, y, sq);
                    }
                }
            }
            if (t + 1 < nt) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();  // buffer t & 1 free; unit t + 1 (and its parameters) in LDS
                if (t + 2 < nt) stage(t + 2, u & 1);
            }
        }
        const float lp = par[256] - 0.5f * reduce_stage<5>(reduce_stage<4>(sq));
        lse_push(lp, run_max, run_sum);
        lp_prev = lp;
    }
    if (owner) {
        float *lp = a.resp + row * a.K;
        lp[a.K - 1] = lp_prev;
        const float lse = run_max + logf(run_sum);
        for (int k = 0; k < a.K; ++k) lp[k] = expf(lp[k] - lse);
        if (a.lse) a.lse[row] = lse;
    }
}

// The FULL body (k_gmm_resp16t's registers cannot hold it), launched after it: a no-op unless the
// launch holds a lower or dense factor (flags[K]); row blocks grid-stride.
template <int D>
__global__ void __launch_bounds__(256, 2) k_gmm_resp16_full(RespArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    if (__builtin_amdgcn_readfirstlane(a.lower[a.K]) == 0) return;
    RespArgs b = a;
    b.prec_t = a.prec_full;
    for (int64_t blk = blockIdx.x; blk * 128 < a.V; blk += gridDim.x) r16_body<D, true>(b, sm, blk);
}

// ---- GMM M-step scatter matrices -------------------------------------------------------------
//
// S_k = sum_i resp[i,k] (x_i - mu_k)(x_i - mu_k)^T, the numerator of sklearn's full covariance
// (_estimate_gaussian_covariances_full: np.dot(resp[:, k] * diff.T, diff) / nk[k]), 2 V K d^2
// flops per M-step.  Workgroup (k, chunk): rows of the chunk are staged through LDS in blocks of
// kCovRB samples, centred on mu_k, with their weights; the reduction over samples is the MFMA
// k-dimension (v_mfma_f32_32x32x2_f32: lane (r, h) supplies A[c1 = rt*32 + r][sample s0 + h] =
// w * xc and B[sample s0 + h][c2 = ct*32 + r] = xc).  The D x D output is split into 32 x 32
// tiles over the 4 wavefronts.  Each chunk writes its own partial; k_gmm_cov_reduce sums the
// chunks in a fixed order (deterministic, no float atomics).  blockIdx.x = k varies fastest, so
// the K workgroups of one chunk run together and share its rows through L2 / MALL.
constexpr int kCovRB = 64;

struct CovArgs {
    const float *x;
    const float *resp;
    const float *means;
    float *out;  // [chunks][K][d][d] partials (or [K][d][d] when chunks == 1)
    int64_t V;
    int64_t rows_per_chunk;
    int d;
    int K;
};

// ---- M-step scatter on v_mfma_f32_16x16x4_f32 (k_gmm_cov16, gmm_cov_async = 3) ----------------
//
// 4 MFMA + 4 staging wavefronts, CPW components per workgroup, two image buffers, two workgroups
// per CU, on 16 x 16 output tiles (only rt <= ct; each off-diagonal tile also stored transposed,
// so S_k comes out exactly symmetric): the symmetric output needs the
// 36 upper tiles of 64 at d = 128 (0.5625 of the dense MFMA cycles) instead of 10 of 16 32-wide
// tiles (0.625).  MFMA (tile rt, ct; 4 samples): A[i][k] = w_s (x_s - mu)[rt*16 + i], B[k][j] =
// (x_s - mu)[ct*16 + j], lane l: i = j = l % 16, samples s = 16 g + 4 (l / 16) + t for the four
// steps t of a 16-sample group g, so each operand row of a group is ONE ds_read_b128 of the
// transposed image B[k][c][s] (rows of 32 samples, 16-byte granules XOR-swizzled by c % 8:
// conflict-free without padding).  A d = 128 component's 36 tiles split 18 / 18 over two
// wavefronts by tile rows {0, 1, 6, 7} and {2, 3, 4, 5}; a wavefront weights its 4 A rows once
// per group and streams the B rows column by column (few VGPRs at 4 waves per SIMD).
// (Twice the MFMA wavefronts with half the tiles each -- 4 MFMA waves per SIMD, the E-step /
// community lesson -- was bit-identical and no faster: 7.45 vs 7.35 ms, profiles/r04_ab_scatter16.txt.)
template <int D>
struct Cov16 {
    static constexpr int RB = 32;                 // samples per block
    static constexpr int LDT = RB;                // image row (swizzled, unpadded)
    static constexpr int IMG = D * LDT;
    static constexpr int CPW = D == 128 ? 2 : 4;  // components per workgroup
    static constexpr int WOFF = CPW * IMG;
    static constexpr int BUF = CPW * IMG + CPW * RB;
    static constexpr int NBUF = 2;
    static constexpr int NT16 = D / 16;
    static constexpr int WPC = D == 128 ? 2 : 1;                  // MFMA wavefronts per component
    static constexpr int NTW = NT16 * (NT16 + 1) / 2 / WPC;      // tiles per wavefront
    static constexpr int NR = 4;                                  // A rows per wavefront
    static constexpr int AW = CPW * WPC;                          // MFMA wavefronts
    static constexpr int THREADS = 64 * (AW + 4);                 // + 4 staging wavefronts
};

// Tiles of MFMA wavefront part p (0 / 1 at d = 128, 0 at d = 64) in issue order (column-major:
// B row ct once per column), with their A-row slot.
template <int D>
struct Cov16Tiles {
    using C = Cov16<D>;
    int rows[C::WPC][C::NR];
    int ct[C::WPC][C::NTW], slot[C::WPC][C::NTW];
    constexpr Cov16Tiles() : rows(), ct(), slot() {
        for (int p = 0; p < C::WPC; ++p) {
            for (int i = 0; i < C::NR; ++i)
                rows[p][i] = D == 64 ? i : (p == 0 ? (i < 2 ? i : i + 4) : i + 2);
            int n = 0;
            for (int c = 0; c < C::NT16; ++c)
                for (int i = 0; i < C::NR; ++i)
                    if (rows[p][i] <= c) {
                        ct[p][n] = c;
                        slot[p][n] = i;
                        ++n;
                    }
        }
    }
};

template <int D>
__device__ __forceinline__ int cov16_off(int c, int gran) {  // image offset of (row c, granule)
    return c * Cov16<D>::LDT + 4 * (gran ^ (c & 7));
}

template <int D, int P>
__device__ __forceinline__ void cov16_consume(const float *img, int nb, int tk, int lane,
                                              __attribute__((ext_vector_type(4)))
                                              float (&acc)[Cov16<D>::NTW]) {
    using C = Cov16<D>;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    constexpr Cov16Tiles<D> TT{};
    const int j16 = lane & 15, kg = lane >> 4;
#if COME_COV_DIAG == 2
    __syncthreads();
#endif
    for (int j = 0; j < nb; ++j) {
#if COME_COV_DIAG == 2
        asm volatile("" ::: "memory");  // keep the LDS reads in the loop
        const float *buf = img;
#else
        __syncthreads();  // barrier j: block j staged
        const float *buf = img + (j % C::NBUF) * C::BUF;
#endif
        COME_PRIO(1);
        const float *im = buf + tk * C::IMG;
#pragma unroll
        for (int g = 0; g < C::RB / 16; ++g) {
            const int gran = 4 * g + kg;
            const f32x4 w = *reinterpret_cast<const f32x4 *>(buf + C::WOFF + tk * C::RB + 4 * gran);
            f32x4 wa[C::NR];
#pragma unroll
            for (int i = 0; i < C::NR; ++i)
                wa[i] = w * *reinterpret_cast<const f32x4 *>(
                                im + cov16_off<D>(TT.rows[P][i] * 16 + j16, gran));
            f32x4 bv[2];
            bv[0] = *reinterpret_cast<const f32x4 *>(im + cov16_off<D>(TT.ct[P][0] * 16 + j16, gran));
            int cur = 0;
#pragma unroll
            for (int n = 0; n < C::NTW; ++n) {
                // the next column's B row, read while this column's MFMAs run
                if (n + 1 < C::NTW && TT.ct[P][n + 1] != TT.ct[P][n])
                    bv[cur ^ 1] = *reinterpret_cast<const f32x4 *>(
                        im + cov16_off<D>(TT.ct[P][n + 1] * 16 + j16, gran));
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[TT.slot[P][n]][t], bv[cur][t],
                                                                  acc[n], 0, 0, 0);
                if (n + 1 < C::NTW && TT.ct[P][n + 1] != TT.ct[P][n]) cur ^= 1;
            }
        }
        COME_PRIO(0);
    }
}

// the MFMA part of wavefront part P (compile-time tile tables): consume, then store the tiles
template <int D, int P>
__device__ __forceinline__ void cov16_part(const CovArgs &a, const float *img, int nb, int tk,
                                           int nk, int k0, int64_t chunk, int lane) {
    using C = Cov16<D>;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    f32x4 acc[C::NTW];
#pragma unroll
    for (int n = 0; n < C::NTW; ++n) acc[n] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if (nb > 0) cov16_consume<D, P>(img, nb, tk, lane, acc);
    if (tk >= nk) return;  // wavefront-uniform: K not a multiple of CPW
    constexpr Cov16Tiles<D> TT{};
    const int j16 = lane & 15, kg = lane >> 4;
    float *out = a.out + (chunk * a.K + k0 + tk) * D * D;
#pragma unroll
    for (int n = 0; n < C::NTW; ++n) {
        const int rt = TT.rows[P][TT.slot[P][n]], ct = TT.ct[P][n];
        const int jj = ct * 16 + j16;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int ii = rt * 16 + 4 * kg + e;
            out[(int64_t)ii * D + jj] = acc[n][e];
            if (rt != ct) out[(int64_t)jj * D + ii] = acc[n][e];
        }
    }
}

// k_gmm_cov16's staging wavefronts (256 threads, thread st): block blk of the chunk [c0, c1) goes
// global -> VGPR register set u (three sets: loads run 3 blocks ahead of the stage that consumes
// them, an HBM / MALL round trip under load exceeding one block period) -> centred, transposed
// LDS image per component (stage), with the weights beside it.
// d = 128: 16-byte loads.  Thread st < RB D / 16 owns feature quad fq = st / 8 (features 4 fq ..
// 4 fq + 3) of samples 4 sg .. 4 sg + 3, sg = st % 8: one dwordx4 per sample, 8 lanes reading one
// 128-B line; each feature's 4 samples become one b128 granule (8 consecutive lanes write the 8
// granules of one image row: conflict-free).  Thread st carries the weight of sample st % RB for
// component st % (CPW RB) / RB (four threads per weight, the same value: no branch).  (vs one dword per column and sample: 7.27 vs 7.40 ms at C4,
// bit-identical, profiles/r05_ab_gmm_diag.txt; the d = 64 form below needs too many registers this
// way: 16 means per thread.)
template <int D>
struct Cov16StageX4 {
    using C = Cov16<D>;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    static constexpr int RB = C::RB, CPW = C::CPW, NX = RB * D / 16;
    static_assert(RB == 32 && NX <= 256 && CPW * RB <= 256, "x4 staging layout");
    const CovArgs &a;
    const int sg, fq, wk, ws, k0, nk;
    const bool xl, wlane;
    const int64_t c0, c1;
    static constexpr int NS = COME_COV_NS;  // register sets: loads run NS blocks ahead
    float mu[CPW][4];
    f32x4 xv[NS][4];
    float wl[NS];
    __device__ __forceinline__ Cov16StageX4(const CovArgs &a_, int st, int k0_, int nk_, int64_t c0_,
                                            int64_t c1_)
        : a(a_), sg(st % 8), fq(st / 8), wk(st % (CPW * RB) / RB), ws(st % RB), k0(k0_), nk(nk_),
          xl(st < NX), wlane(true), c0(c0_), c1(c1_) {
#pragma unroll
        for (int kk = 0; kk < CPW; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                mu[kk][i] = xl && kk < nk ? a.means[(int64_t)(k0 + kk) * D + 4 * fq + i] : 0.0f;
    }
    // Loads are unconditional (rows past the chunk clamped to its last row, components past K
    // to K - 1) and the out-of-range values zeroed when staged: a load under a divergent branch
    // leaves the compiler unable to count the loads in flight, and it then waits for all of them
    // (vmcnt(0)) before every stage -- the three-block lookahead collapses to none.
    __device__ __forceinline__ void load(int u, int blk) {
        const int64_t b = c0 + (COME_COV_DIAG == 3 ? 0 : (int64_t)blk * RB);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int64_t r = min(b + 4 * sg + t, c1 - 1);
            xv[u][t] = *reinterpret_cast<const f32x4 *>(a.x + r * D + 4 * fq);
        }
        const int64_t wrow = min(b + ws, c1 - 1);
        wl[u] = a.resp[wrow * a.K + min(k0 + wk, a.K - 1)];
    }
    __device__ __forceinline__ void stage(float *img, int u, int blk) const {
        float *buf = img + (blk % C::NBUF) * C::BUF;
        const int64_t b = c0 + (COME_COV_DIAG == 3 ? 0 : (int64_t)blk * RB);
        // (the values are read outside any branch: a register read under a divergent branch
        // also makes the compiler drain every load in flight)
        const float w = wk < nk && b + ws < c1 ? wl[u] : 0.0f;
        if (NX == 256 || xl) {  // every thread holds samples at d = 128 (no branch)
#pragma unroll
            for (int kk = 0; kk < CPW; ++kk)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    f32x4 xb;
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        xb[t] = b + 4 * sg + t < c1 ? xv[u][t][i] - mu[kk][i] : 0.0f;
                    *reinterpret_cast<f32x4 *>(buf + kk * C::IMG + cov16_off<D>(4 * fq + i, sg)) = xb;
                }
        }
        buf[C::WOFF + wk * RB + ws] = w;  // (threads st, st + 64, ... write the same value)
    }
};

// d = 64: thread owns column sc and samples SPT sp .. SPT sp + SPT
// - 1 of a block; lane l also carries the weight of sample SPT sp + l % SPT for component
// l % (SPT CPW) / SPT
template <int D>
struct Cov16StageCol {
    using C = Cov16<D>;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    static constexpr int RB = C::RB, CPW = C::CPW, SPT = RB * D / 256;
    static_assert(SPT % 4 == 0 && SPT * CPW <= 64 && D % 64 == 0, "staging layout");
    const CovArgs &a;
    const int sc, sp, wk, ws, k0, nk;
    const bool wlane;
    const int64_t c0, c1;
    static constexpr int NS = 3;
    float mu[CPW];
    float xv[3][SPT];
    float wl[3];
    __device__ __forceinline__ Cov16StageCol(const CovArgs &a_, int st, int lane, int k0_, int nk_,
                                             int64_t c0_, int64_t c1_)
        : a(a_), sc(st % D), sp(st / D), wk(lane % (SPT * CPW) / SPT), ws(lane % SPT), k0(k0_),
          nk(nk_), wlane(true), c0(c0_), c1(c1_) {
#pragma unroll
        for (int kk = 0; kk < CPW; ++kk)
            mu[kk] = kk < nk ? a.means[(int64_t)(k0 + kk) * D + sc] : 0.0f;
    }
    // unconditional loads, out-of-range values zeroed when staged (as Cov16StageX4)
    __device__ __forceinline__ void load(int u, int blk) {
        const int64_t b = c0 + (COME_COV_DIAG == 3 ? 0 : (int64_t)blk * RB);
#pragma unroll
        for (int q = 0; q < SPT; ++q) xv[u][q] = a.x[min(b + SPT * sp + q, c1 - 1) * D + sc];
        const int64_t wrow = min(b + SPT * sp + ws, c1 - 1);
        wl[u] = a.resp[wrow * a.K + min(k0 + wk, a.K - 1)];
    }
    __device__ __forceinline__ void stage(float *img, int u, int blk) const {
        float *buf = img + (blk % C::NBUF) * C::BUF;
        const int64_t b = c0 + (COME_COV_DIAG == 3 ? 0 : (int64_t)blk * RB);
#pragma unroll
        for (int kk = 0; kk < CPW; ++kk)
#pragma unroll
            for (int j = 0; j < SPT / 4; ++j) {
                f32x4 xb;
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4)
                    xb[q4] = b + SPT * sp + 4 * j + q4 < c1 ? xv[u][4 * j + q4] - mu[kk] : 0.0f;
                *reinterpret_cast<f32x4 *>(buf + kk * C::IMG + cov16_off<D>(sc, (SPT * sp + 4 * j) / 4)) =
                    xb;
            }
        const float w = wk < nk && b + SPT * sp + ws < c1 ? wl[u] : 0.0f;
        buf[C::WOFF + wk * RB + SPT * sp + ws] = w;  // (lanes l, l + SPT CPW: the same value)
    }
};

// the staging pipeline: block j + 1 is staged while block j is multiplied (two image buffers, one
// barrier per block); register set (j + 1) % NS holds block j + 1, reloaded with block j + 1 + NS.
// Every load and stage is issued unconditionally (the block index clamped to nb - 1; a stage of
// block nb lands in a buffer nobody reads again, its values zeroed): with no branch around them
// the compiler counts the loads in flight exactly and each stage waits only for its own set
// (a conditional load made it drain all of them, vmcnt(0), at the loop head).
template <int D, typename S>
__device__ __forceinline__ void cov16_staging(float *img, S &sg, int nb) {
    if (nb == 0) return;
    constexpr int SD = Cov16<D>::NBUF - 1, NS = S::NS;
    const int last = nb - 1;
#pragma unroll
    for (int u = 0; u < NS; ++u) sg.load(u, min(u, last));
#if COME_COV_DIAG == 2
    sg.stage(img, 0, 0);
    __syncthreads();
    return;
#endif
    sg.stage(img, 0, 0);
    if (COME_COV_DIAG != 1) sg.load(0, min(NS, last));
    __syncthreads();  // barrier 0
    for (int j0 = 0; j0 < nb; j0 += NS) {
#pragma unroll
        for (int u = 0; u < NS; ++u) {  // j = j0 + u: register set (j + SD) % NS
            const int j = j0 + u;
            if (j >= nb) return;  // (not break: the loop head then sees one load order only)
            sg.stage(img, (u + SD) % NS, j + SD);
            if (COME_COV_DIAG != 1) sg.load((u + SD) % NS, min(j + SD + NS, last));
            if (j + 1 < nb) __syncthreads();  // barrier j + 1
        }
    }
}

template <int D>
__global__ void __launch_bounds__((Cov16<D>::THREADS))
    __attribute__((amdgpu_waves_per_eu(4))) k_gmm_cov16(CovArgs a) {
    using C = Cov16<D>;
    constexpr int CPW = C::CPW;
    constexpr int RB = C::RB;
    static_assert(C::NBUF * C::BUF * sizeof(float) * 2 <= 160 * 1024, "two workgroups per CU");
    __shared__ __attribute__((aligned(16))) float img[C::NBUF * C::BUF];
    const int64_t chunk = blockIdx.y;
    const int k0 = blockIdx.x * CPW;
    const int nk = a.K - k0 < CPW ? a.K - k0 : CPW;
    const int64_t c0 = chunk * a.rows_per_chunk;
    int64_t c1 = c0 + a.rows_per_chunk;
    if (c1 > a.V) c1 = a.V;
    const int nb = c1 > c0 ? (int)((c1 - c0 + RB - 1) / RB) : 0;
    const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    if (wid < C::AW) {
        // ---- MFMA wavefronts: component tk, tile part p ----
        const int tk = wid / C::WPC, p = wid % C::WPC;
        constexpr int P1 = C::WPC > 1 ? 1 : 0;
        if (p == 0) cov16_part<D, 0>(a, img, nb, tk, nk, k0, chunk, lane);
        else cov16_part<D, P1>(a, img, nb, tk, nk, k0, chunk, lane);
        return;
    }
    // ---- staging wavefronts: 16-byte loads at d = 128, one column per thread at d = 64 ----
    const int st = tid - 64 * C::AW;
    if constexpr (D == 128) {
        Cov16StageX4<D> sg(a, st, k0, nk, c0, c1);
        cov16_staging<D>(img, sg, nb);
    } else {
        Cov16StageCol<D> sg(a, st, lane, k0, nk, c0, c1);
        cov16_staging<D>(img, sg, nb);
    }
}

// ---- M-step scatter on bf16-part MFMAs (k_gmm_cov_bf3, gmm_cov_async = 4) --------------------
//
// S_k = sum_i r_ik d_i d_i^T (d_i = x_i - m_k) written as E^T E with E_ik = sqrt(r_ik) d_i: one
// operand image serves both sides of every MFMA.  E is formed and split into its three bf16 parts
// (the bf16-part arithmetic: six exact part products per multiply-add, summed in fp32) by 4
// staging wavefronts, ONCE per (sample, feature, component), into a feature-major LDS image (rows
// of 32 samples, 16-byte granules of 8 samples XOR-swizzled by CovBf3::swz: conflict-free
// ds_read_b128 fragments and ds_write_b128 stores).  The MFMA wavefronts take fragment a (32
// features x 16 samples, one ds_read_b128 per part) as the A operand of the tiles in row a and
// the B operand of the tiles in column a: the 10 upper 32x32 tiles of a d = 128 component (3 at
// d = 64) split 5 / 5 over two wavefronts.  sqrt(r) adds one rounding (1 ulp) to each weight
// against the fp32 kernels' r d: tests hold the result to their tolerances and error level.
// Grid and output as k_gmm_cov16 (components per workgroup x row chunks, [chunk][K][d][d]).
template <int D>
struct CovBf3 {
    static constexpr int RB = 32;                   // samples per block (2 k-steps)
    static constexpr int CPW = D == 128 ? 2 : 4;    // components per workgroup
    static constexpr int WPC = D == 128 ? COME_COV3_WPC : 1;  // MFMA wavefronts per component
    static constexpr int AW = CPW * WPC;            // MFMA wavefronts (4)
    static constexpr int SW = D == 128 ? COME_COV3_SW : 4;  // staging wavefronts
    static constexpr int THREADS = 64 * (AW + SW);
    static constexpr int NF = D / 32;               // fragments (32-feature row groups)
    static constexpr int PLANE = D * RB * 2;        // bytes per part image (D rows x 32 bf16)
    static constexpr int IMG = 3 * PLANE;           // per component (24 KB at d = 128)
    static constexpr int BUF = CPW * IMG;
    static constexpr int LDS_BYTES = 2 * BUF;       // 96 KB: one workgroup per CU
    static constexpr int SPT = RB * D / (64 * SW);  // samples per staging thread (16 / 8)
    static_assert(SPT % 8 == 0, "a staging thread fills whole 8-sample granules");
    // granule swizzle: bit 0 = bit 2 of the row, bit 1 = bit 1 ^ bit 3 -- distinct over the rows
    // of every 16-lane ds_read_b128 group (64 banks) and of every 8-lane ds_write_b128 group (32
    // banks: 8 consecutive rows) that share a bank column
    __host__ __device__ static constexpr int swz(int f) {
        return ((f >> 2) & 1) | ((((f >> 1) ^ (f >> 3)) & 1) << 1);
    }
    __host__ __device__ static constexpr int at(int P, int f, int g) {
        return P * PLANE + f * 64 + 16 * (g ^ swz(f));
    }
};

// tile n of MFMA part p: (row group ta, column group tb), ta <= tb
template <int D>
struct CovBf3Tiles {
    static constexpr int WPC = CovBf3<D>::WPC;
    int cnt[4], ta[4][5], tb[4][5];
    bool need[4][4];  // fragments a part reads
    constexpr CovBf3Tiles() : cnt(), ta(), tb(), need() {
        // d = 128: 10 upper tiles per component, 5 / 5 over 2 wavefronts or 3 / 3 / 2 / 2 over 4
        const int a2[2][5] = {{0, 0, 0, 0, 3}, {1, 1, 1, 2, 2}};
        const int b2[2][5] = {{0, 1, 2, 3, 3}, {1, 2, 3, 2, 3}};
        const int a4[4][3] = {{0, 0, 0}, {0, 1, 3}, {1, 1, 0}, {2, 2, 0}};
        const int b4[4][3] = {{0, 1, 2}, {3, 3, 3}, {1, 2, 0}, {2, 3, 0}};
        const int c4[4] = {3, 3, 2, 2};
        for (int p = 0; p < 4; ++p) {
            if (D == 128 && WPC == 2 && p < 2) {
                cnt[p] = 5;
                for (int n = 0; n < 5; ++n) {
                    ta[p][n] = a2[p][n];
                    tb[p][n] = b2[p][n];
                }
            } else if (D == 128 && WPC == 4) {
                cnt[p] = c4[p];
                for (int n = 0; n < c4[p]; ++n) {
                    ta[p][n] = a4[p][n];
                    tb[p][n] = b4[p][n];
                }
            } else if (D == 64 && p == 0) {
                const int a0[3] = {0, 0, 1}, b0[3] = {0, 1, 1};
                cnt[p] = 3;
                for (int n = 0; n < 3; ++n) {
                    ta[p][n] = a0[n];
                    tb[p][n] = b0[n];
                }
            }
            for (int n = 0; n < cnt[p]; ++n) need[p][ta[p][n]] = need[p][tb[p][n]] = true;
        }
    }
};

template <int D, int P>
__device__ __forceinline__ void covbf3_part(const CovArgs &a, const char *smb, int nb, int tk,
                                            int nk, int k0, int64_t chunk, int lane) {
    using C = CovBf3<D>;
    using f32x16 = __attribute__((ext_vector_type(16))) float;
    typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
    constexpr CovBf3Tiles<D> TT{};
    constexpr int NT = TT.cnt[P];
    const int i = lane & 31, h = lane >> 5;
    f32x16 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[n][e] = 0.0f;
    for (int j = 0; j < nb; ++j) {
        __syncthreads();  // barrier j: block j staged
        const char *im = smb + (j & 1) * C::BUF + tk * C::IMG;
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            bf16x8 F[C::NF][3];
#pragma unroll
            for (int f = 0; f < C::NF; ++f) {
                if (!TT.need[P][f]) continue;
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    F[f][p] = *reinterpret_cast<const bf16x8 *>(im + C::at(p, 32 * f + i, 2 * st + h));
            }
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                const int ta = TT.ta[P][n], tb = TT.tb[P][n];
                acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][2], F[tb][0], acc[n], 0, 0, 0);
                acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][1], F[tb][1], acc[n], 0, 0, 0);
                acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][0], F[tb][2], acc[n], 0, 0, 0);
                acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][1], F[tb][0], acc[n], 0, 0, 0);
                acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][0], F[tb][1], acc[n], 0, 0, 0);
                acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][0], F[tb][0], acc[n], 0, 0, 0);
            }
        }
    }
    if (tk >= nk) return;  // wavefront-uniform: K not a multiple of CPW
    float *out = a.out + (chunk * a.K + k0 + tk) * D * D;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int ta = TT.ta[P][n], tb = TT.tb[P][n];
        const int jj = 32 * tb + i;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int ii = 32 * ta + (r & 3) + 8 * (r >> 2) + 4 * h;
            out[(int64_t)ii * D + jj] = acc[n][r];
            if (ta != tb) out[(int64_t)jj * D + ii] = acc[n][r];
        }
    }
}

// staging thread st: feature f = st % D of samples SPT sg .. SPT sg + SPT - 1 (sg = st / D,
// uniform over a wavefront); lane l < CPW SPT of each wavefront also loads the weight r of its
// (component l / SPT, sample l % SPT), square-rooted at stage time and broadcast by readlane
// (a broadcast through a 128-byte LDS slot per wavefront instead -- one store, 8 ds_read_b128 --
// was 3% slower: 5.80-5.88 vs 5.64-5.71 ms at C4)
template <int D>
struct CovBf3Stage {
    using C = CovBf3<D>;
    static constexpr int SPT = C::SPT, CPW = C::CPW;
    static constexpr int NS = COME_COV3_NS;  // register sets: loads run NS blocks ahead
    const CovArgs &a;
    const int f, sg, k0, nk, lane;
    const int64_t c0, c1;
    float mu[CPW];
    float xv[NS][SPT];
    float wv[NS];
    __device__ __forceinline__ CovBf3Stage(const CovArgs &a_, int st, int lane_, int k0_, int nk_,
                                           int64_t c0_, int64_t c1_)
        : a(a_), f(st % D), sg(__builtin_amdgcn_readfirstlane(st / D)), k0(k0_), nk(nk_),
          lane(lane_), c0(c0_), c1(c1_) {
#pragma unroll
        for (int kk = 0; kk < CPW; ++kk)
            mu[kk] = kk < nk ? a.means[(int64_t)(k0 + kk) * D + f] : 0.0f;
    }
    // unconditional loads (rows clamped to the chunk, components to K - 1; zeroed when staged)
    __device__ __forceinline__ void load(int u, int blk) {
        const int64_t b = c0 + (int64_t)blk * C::RB + SPT * sg;
#pragma unroll
        for (int q = 0; q < SPT; ++q) xv[u][q] = a.x[min(b + q, c1 - 1) * D + f];
        const int l = lane % (CPW * SPT);
        wv[u] = a.resp[min(b + l % SPT, c1 - 1) * a.K + min(k0 + l / SPT, a.K - 1)];
    }
    // the weight of lane l's (component, sample): sqrt(r), 0 past the chunk or K (so every E
    // value of those is an exact 0 with no per-element select; x is finite, rows clamped)
    __device__ __forceinline__ float weight(int u, int blk) const {
        const int l = lane % (CPW * SPT);
        const int64_t row = c0 + (int64_t)blk * C::RB + SPT * sg + l % SPT;
        return (l / SPT < nk && row < c1) ? sqrtf(wv[u]) : 0.0f;
    }
    __device__ __forceinline__ void stage(float *img, int u, int blk) const {
        char *buf = reinterpret_cast<char *>(img) + (blk % 2) * C::BUF;
        const float w = weight(u, blk);
#pragma unroll
        for (int kk = 0; kk < CPW; ++kk) {
            char *im = buf + kk * C::IMG;
#pragma unroll
            for (int g = 0; g < SPT / 8; ++g) {
                uint32_t p1[4], p2[4], p3[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float v[2];
#pragma unroll
                    for (int z = 0; z < 2; ++z) {
                        const int q = 8 * g + 2 * e + z;
                        const float ws =
                            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), kk * SPT + q));
                        v[z] = ws * (xv[u][q] - mu[kk]);
                    }
                    bf16_split3(v[0], v[1], p1[e], p2[e], p3[e]);
                }
                const int gr = (SPT * sg) / 8 + g;  // granule of the 32-sample row
                *reinterpret_cast<uint4 *>(im + C::at(0, f, gr)) = uint4{p1[0], p1[1], p1[2], p1[3]};
                *reinterpret_cast<uint4 *>(im + C::at(1, f, gr)) = uint4{p2[0], p2[1], p2[2], p2[3]};
                *reinterpret_cast<uint4 *>(im + C::at(2, f, gr)) = uint4{p3[0], p3[1], p3[2], p3[3]};
            }
        }
    }
};

template <int D>
__global__ void __launch_bounds__(CovBf3<D>::THREADS) __attribute__((amdgpu_waves_per_eu(2)))
    k_gmm_cov_bf3(CovArgs a) {
    using C = CovBf3<D>;
    extern __shared__ __attribute__((aligned(16))) char smb[];
    const int64_t chunk = blockIdx.y;
    const int k0 = blockIdx.x * C::CPW;
    const int nk = a.K - k0 < C::CPW ? a.K - k0 : C::CPW;
    const int64_t c0 = chunk * a.rows_per_chunk;
    int64_t c1 = c0 + a.rows_per_chunk;
    if (c1 > a.V) c1 = a.V;
    const int nb = c1 > c0 ? (int)((c1 - c0 + C::RB - 1) / C::RB) : 0;
    const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    if (wid < C::AW) {
        // wavefronts w and w + 4 share a SIMD: with 4 parts per component, component 1's part
        // index is shifted by 2 so that each SIMD gets 3 + 2 tiles
        const int tk = wid / C::WPC;
        const int p = C::WPC == 4 ? (wid % 4 + 2 * tk) % 4 : wid % C::WPC;
        if (p == 0) covbf3_part<D, 0>(a, smb, nb, tk, nk, k0, chunk, lane);
        else if (p == 1) covbf3_part<D, (C::WPC > 1 ? 1 : 0)>(a, smb, nb, tk, nk, k0, chunk, lane);
        else if (p == 2) covbf3_part<D, (C::WPC > 2 ? 2 : 0)>(a, smb, nb, tk, nk, k0, chunk, lane);
        else covbf3_part<D, (C::WPC > 2 ? 3 : 0)>(a, smb, nb, tk, nk, k0, chunk, lane);
        return;
    }
    CovBf3Stage<D> sg(a, tid - 64 * C::AW, lane, k0, nk, c0, c1);
    cov16_staging<D>(reinterpret_cast<float *>(smb), sg, nb);
}

// Any d <= 128 on the VALU: thread owns entries tid + 256 q of the d x d output.
__global__ void __launch_bounds__(256) k_gmm_cov_valu(CovArgs a) {
    constexpr int MAXQ = 64;  // 128 * 128 / 256
    __shared__ float xs[kCovRB * 129];
    __shared__ float ws[kCovRB];
    const int d = a.d, k = blockIdx.x, tid = threadIdx.x;
    const int64_t c0 = (int64_t)blockIdx.y * a.rows_per_chunk;
    int64_t c1 = c0 + a.rows_per_chunk;
    if (c1 > a.V) c1 = a.V;
    const int ne = d * d;
    float acc[MAXQ];
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) acc[q] = 0.0f;
    for (int64_t b = c0; b < c1; b += kCovRB) {
        __syncthreads();
        for (int o = tid; o < kCovRB * d; o += 256) {
            const int s = o / d, c = o % d;
            xs[s * 129 + c] = b + s < c1 ? a.x[(b + s) * d + c] - a.means[k * d + c] : 0.0f;
        }
        if (tid < kCovRB) ws[tid] = b + tid < c1 ? a.resp[(b + tid) * a.K + k] : 0.0f;
        __syncthreads();
        const int nb = (int)((c1 - b) < kCovRB ? (c1 - b) : kCovRB);
        for (int s = 0; s < nb; ++s) {
            const float w = ws[s];
            const float *row = xs + s * 129;
#pragma unroll
            for (int q = 0; q < MAXQ; ++q) {
                const int e = tid + 256 * q;
                if (e < ne) acc[q] = __builtin_fmaf(w * row[e / d], row[e % d], acc[q]);
            }
        }
    }
    float *out = a.out + ((int64_t)blockIdx.y * a.K + k) * ne;
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) {
        const int e = tid + 256 * q;
        if (e < ne) out[e] = acc[q];
    }
}

// ---- wide rows (128 < d <= 512): VALU forms with the d x d matrices streamed in row chunks ----
// The MFMA kernels above keep a whole d x d matrix (or a 128-row tile of inputs) in LDS, which
// stops at d = 128.  These forms cover every d up to kMaxDim: kTRW rows per workgroup, each
// component's matrix staged kChunkRows(d) rows at a time (<= 64 KiB, rows padded by one float
// against bank conflicts).  Same arithmetic as k_community_grad / k_gmm_resp (fmaf chains in j
// order), a fraction of the MFMA rate: they exist so that every embedding size the SGNS kernels
// accept also trains through the community step (community_embeddings.py:61-78) and the GMM.
constexpr int kTRW = 8;
__host__ __device__ inline int chunk_rows(int d) { return 16384 / (d + 1); }

__global__ void __launch_bounds__(kThreads) k_community_grad_wide(CommArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int d = a.d, CH = chunk_rows(d), LDM = d + 1;
    float *X = smem;            // [kTRW][d]
    float *Dk = X + kTRW * d;   // [kTRW][d]  x - mu_k
    float *G = Dk + kTRW * d;   // [kTRW][d]
    float *M = G + kTRW * d;    // [CH][d + 1] rows c0 .. c0 + CH of inv_cov[k]
    float *P = M + CH * LDM;    // [kTRW] pi[:, k]
    const int64_t r0 = (int64_t)blockIdx.x * kTRW;
    const int rows = (int)((a.V - r0) < kTRW ? (a.V - r0) : kTRW);
    const int n = kTRW * d;
    for (int o = threadIdx.x; o < n; o += kThreads)
        X[o] = o / d < rows ? a.x[(r0 + o / d) * d + (o % d)] : 0.0f;
    for (int it = 0; it < a.iters; ++it) {
        for (int o = threadIdx.x; o < n; o += kThreads) G[o] = 0.0f;
        for (int k = 0; k < a.K; ++k) {
            __syncthreads();
            for (int o = threadIdx.x; o < n; o += kThreads) Dk[o] = X[o] - a.mu[k * d + (o % d)];
            if (threadIdx.x < kTRW)
                P[threadIdx.x] = threadIdx.x < rows ? a.pi[(r0 + threadIdx.x) * a.K + k] : 0.0f;
            for (int c0 = 0; c0 < d; c0 += CH) {
                const int cn = d - c0 < CH ? d - c0 : CH;
                __syncthreads();
                for (int o = threadIdx.x; o < cn * d; o += kThreads)
                    M[(o / d) * LDM + o % d] = a.inv_cov[(int64_t)k * d * d + (int64_t)c0 * d + o];
                __syncthreads();
                for (int o = threadIdx.x; o < kTRW * cn; o += kThreads) {
                    const int r = o / cn, c = o % cn;
                    if (r >= rows) continue;
                    float acc = 0.0f;
                    for (int j = 0; j < d; ++j) acc = __builtin_fmaf(Dk[r * d + j], M[c * LDM + j], acc);
                    G[r * d + c0 + c] = __builtin_fmaf(P[r], acc, G[r * d + c0 + c]);
                }
            }
        }
        __syncthreads();
        for (int o = threadIdx.x; o < n; o += kThreads) {
            float g = G[o] * a.coef;
            g = g < -5.0f ? -5.0f : (g > 5.0f ? 5.0f : g);  // clip(min=-5, max=5), :79
            X[o] = X[o] - g * a.lr;
        }
        __syncthreads();
    }
    for (int o = threadIdx.x; o < n; o += kThreads)
        if (o / d < rows) a.x[(r0 + o / d) * d + (o % d)] = X[o];
}

// log N(x; mu_k, P_k) + log w_k for every (row, k) into resp_out (any K), then the per-row
// softmax over k in place (the lse of each row optionally into a.lse).
__global__ void __launch_bounds__(kThreads) k_gmm_resp_wide(RespArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int d = a.d, CH = chunk_rows(d), LDM = d + 1;
    float *X = smem;            // [kTRW][d]
    float *Y = X + kTRW * d;    // [kTRW][d]  x P_k, accumulated over row chunks of P_k
    float *M = Y + kTRW * d;    // [CH][d + 1] rows j0 .. j0 + CH of prec_chol[k]
    float *SQ = M + CH * LDM;   // [kTRW]
    const int64_t r0 = (int64_t)blockIdx.x * kTRW;
    const int rows = (int)((a.V - r0) < kTRW ? (a.V - r0) : kTRW);
    const int n = kTRW * d;
    for (int o = threadIdx.x; o < n; o += kThreads)
        X[o] = o / d < rows ? a.x[(r0 + o / d) * d + (o % d)] : 0.0f;
    for (int k = 0; k < a.K; ++k) {
        __syncthreads();
        for (int o = threadIdx.x; o < n; o += kThreads) Y[o] = 0.0f;
        if (threadIdx.x < kTRW) SQ[threadIdx.x] = 0.0f;
        for (int j0 = 0; j0 < d; j0 += CH) {
            const int jn = d - j0 < CH ? d - j0 : CH;
            __syncthreads();
            for (int o = threadIdx.x; o < jn * d; o += kThreads)
                M[(o / d) * LDM + o % d] = a.prec_chol[(int64_t)k * d * d + (int64_t)j0 * d + o];
            __syncthreads();
            for (int o = threadIdx.x; o < n; o += kThreads) {
                const int r = o / d, c = o % d;
                float acc = Y[o];
                for (int j = 0; j < jn; ++j)
                    acc = __builtin_fmaf(X[r * d + j0 + j], M[j * LDM + c], acc);
                Y[o] = acc;
            }
        }
        __syncthreads();
        for (int o = threadIdx.x; o < n; o += kThreads) {
            const float y = Y[o] - a.mu_prec[k * d + (o % d)];
            atomicAdd(&SQ[o / d], y * y);
        }
        __syncthreads();
        if (threadIdx.x < rows) a.resp[(r0 + threadIdx.x) * a.K + k] =
            a.log_norm[k] - 0.5f * SQ[threadIdx.x];
    }
    __syncthreads();
    if (threadIdx.x < rows) {  // stores above came from this same thread: visible to it
        float *lp = a.resp + (r0 + threadIdx.x) * a.K;
        float m = -INFINITY;
        for (int k = 0; k < a.K; ++k) m = fmaxf(m, lp[k]);
        float s = 0.0f;
        for (int k = 0; k < a.K; ++k) s += expf(lp[k] - m);
        const float lse = m + logf(s);
        for (int k = 0; k < a.K; ++k) lp[k] = expf(lp[k] - lse);
        if (a.lse) a.lse[r0 + threadIdx.x] = lse;
    }
}

// Scatter matrices for any d <= kMaxDim: workgroup (k, chunk, tile) accumulates the 64 x 64
// output tile `tile` (row-major over (d/64 rounded up)^2 tiles) over the chunk's samples, staged
// 32 at a time centred on mu_k with their weights.
constexpr int kCovWideRB = 32;
__global__ void __launch_bounds__(kThreads) k_gmm_cov_wide(CovArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int d = a.d, k = blockIdx.x, tid = threadIdx.x;
    const int nt = (d + 63) / 64;
    const int ti = blockIdx.z / nt, tj = blockIdx.z % nt;
    float *xs = smem;                 // [kCovWideRB][d]
    float *ws = xs + kCovWideRB * d;  // [kCovWideRB]
    const int64_t c0 = (int64_t)blockIdx.y * a.rows_per_chunk;
    int64_t c1 = c0 + a.rows_per_chunk;
    if (c1 > a.V) c1 = a.V;
    float acc[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
    for (int64_t b = c0; b < c1; b += kCovWideRB) {
        __syncthreads();
        for (int o = tid; o < kCovWideRB * d; o += kThreads) {
            const int s = o / d, c = o % d;
            xs[o] = b + s < c1 ? a.x[(b + s) * d + c] - a.means[k * d + c] : 0.0f;
        }
        if (tid < kCovWideRB) ws[tid] = b + tid < c1 ? a.resp[(b + tid) * a.K + k] : 0.0f;
        __syncthreads();
        const int nb = (int)((c1 - b) < kCovWideRB ? (c1 - b) : kCovWideRB);
        for (int s = 0; s < nb; ++s) {
            const float w = ws[s];
            const float *row = xs + s * d;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int e = tid + 256 * q;  // (i, j) of the 64 x 64 tile
                const int i = ti * 64 + e / 64, j = tj * 64 + e % 64;
                if (i < d && j < d) acc[q] = __builtin_fmaf(w * row[i], row[j], acc[q]);
            }
        }
    }
    float *out = a.out + ((int64_t)blockIdx.y * a.K + k) * d * d;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int e = tid + 256 * q;
        const int i = ti * 64 + e / 64, j = tj * 64 + e % 64;
        if (i < d && j < d) out[(int64_t)i * d + j] = acc[q];
    }
}

// out[i] = sum_c part[c][i] in chunk order (deterministic), i over K d^2 entries.
__global__ void __launch_bounds__(256) k_gmm_cov_reduce(const float *part, float *out, int64_t n,
                                                        int chunks) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float s = 0.0f;
    for (int c = 0; c < chunks; ++c) s += part[(int64_t)c * n + i];
    out[i] = s;
}

}  // namespace come

using namespace come;

extern "C" int come_community_grad(float *x, int64_t V, int d, const float *pi, const float *mu,
                                   const float *inv_cov, int K, float beta, float lr, int iters,
                                   void *stream) {
    if (V < 0 || d < 1 || d > kMaxDim || K < 1 || iters < 0)
        return set_error(COME_E_INVALID, "community_grad: need V>=0, 1<=d<=%d, K>=1, iters>=0",
                         kMaxDim);
    if (V == 0 || iters == 0) return COME_OK;
    if (!x || !pi || !mu || !inv_cov) return set_error(COME_E_INVALID, "null pointer");
    int dev;
    int rc = ensure_init(&dev);
    if (rc) return rc;
    CommArgs a{x, pi, mu, inv_cov, V, d, K, (float)((double)beta / (double)K), lr, iters};
    const int variant = current_opts().community_async;
    if (variant != 2 && variant != 3)
        return set_error(COME_E_INVALID, "community_async must be 2 or 3 (got %d)", variant);
    if ((d == 64 || d == 128) && ((uintptr_t)inv_cov % 16) == 0 && ((uintptr_t)mu % 16) == 0 &&
        variant == 3) {
        // k_comm_split16 (the bf16 part images of every inv_cov[k], once per call) + k_community_b16
        const size_t ub = d == 64 ? CommB16<64>::UBYTES : CommB16<128>::UBYTES;
        char *img = (char *)stream_scratch(dev, stream, kScratchCommSplit, (size_t)K * (d / 32) * ub);
        if (!img) return scratch_failed();
        const int64_t work = (int64_t)K * (d / 32) * d * 4;
        hipLaunchKernelGGL(d == 64 ? k_comm_split16<64> : k_comm_split16<128>,
                           dim3((unsigned)std::min<int64_t>((work + 255) / 256, 4096)), dim3(256), 0,
                           (hipStream_t)stream, inv_cov, img, K);
        rc = hip_error(hipGetLastError(), "k_comm_split16 launch");
        if (rc) return rc;
        a.img = img;
        static bool attr3 = false;
        if (!attr3) {
            for (void (*f)(CommArgs) : {k_community_b16<64>, k_community_b16<128>})
                (void)hipFuncSetAttribute((const void *)f,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr3 = true;
        }
        hipLaunchKernelGGL(d == 64 ? k_community_b16<64> : k_community_b16<128>,
                           dim3((unsigned)((V + 127) / 128)), dim3(512),
                           d == 64 ? CommB16<64>::LDS_BYTES : CommB16<128>::LDS_BYTES,
                           (hipStream_t)stream, a);
        return hip_error(hipGetLastError(), "k_community_b16 launch");
    }
    if ((d == 64 || d == 128) && ((uintptr_t)inv_cov % 16) == 0 && ((uintptr_t)mu % 16) == 0) {
        // 2: the fp32 form k_community16
        void (*kern)(CommArgs) = d == 64 ? k_community16<64> : k_community16<128>;
        const size_t lds =
            sizeof(float) * (size_t)(d == 64 ? Comm16<64>::LDS_FLOATS : Comm16<128>::LDS_FLOATS);
        static bool attr = false;
        if (!attr) {
            for (void (*f)(CommArgs) : {k_community16<64>, k_community16<128>})
                (void)hipFuncSetAttribute((const void *)f,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr = true;
        }
        hipLaunchKernelGGL(kern, dim3((unsigned)((V + 127) / 128)), dim3(512), lds,
                           (hipStream_t)stream, a);
        return hip_error(hipGetLastError(), "community MFMA launch");
    }
    if (d > 128) {
        const size_t lds = sizeof(float) * ((size_t)3 * kTRW * d +
                                            (size_t)chunk_rows(d) * (d + 1) + kTRW);
        static bool attr_w = false;
        if (!attr_w) {
            (void)hipFuncSetAttribute((const void *)k_community_grad_wide,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr_w = true;
        }
        hipLaunchKernelGGL(k_community_grad_wide, dim3((unsigned)((V + kTRW - 1) / kTRW)),
                           dim3(kThreads), lds, (hipStream_t)stream, a);
        return hip_error(hipGetLastError(), "k_community_grad_wide launch");
    }
    const size_t lds = sizeof(float) * ((size_t)3 * kTR * d + (size_t)d * d);
    const unsigned grid = (unsigned)((V + kTR - 1) / kTR);
    static bool attr_v = false;
    if (!attr_v) {
        (void)hipFuncSetAttribute((const void *)k_community_grad,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_v = true;
    }
    hipLaunchKernelGGL(k_community_grad, dim3(grid), dim3(kThreads), lds, (hipStream_t)stream, a);
    return hip_error(hipGetLastError(), "k_community_grad launch");
}

extern "C" int come_gmm_resp(const float *x, int64_t V, int d, const float *prec_chol,
                             const float *mu_prec, const float *log_norm, int K, float *resp_out,
                             void *stream) {
    return come_gmm_estep(x, V, d, prec_chol, mu_prec, log_norm, K, resp_out, nullptr, stream);
}

extern "C" int come_gmm_estep(const float *x, int64_t V, int d, const float *prec_chol,
                              const float *mu_prec, const float *log_norm, int K, float *resp_out,
                              float *lse_out, void *stream) {
    const bool mfma = (d == 64 || d == 128) && ((uintptr_t)prec_chol % 16) == 0 &&
                      ((uintptr_t)mu_prec % 16) == 0;
    if (V < 0 || d < 1 || d > kMaxDim || K < 1 || K > 4096 || (!mfma && d <= 128 && K > 64))
        return set_error(COME_E_INVALID, "gmm_resp: need V>=0, 1<=d<=%d, 1<=K<=4096 (K<=64 for "
                                         "d <= 128 other than 64, 128)", kMaxDim);
    if (V == 0) return COME_OK;
    if (!x || !prec_chol || !mu_prec || !log_norm || !resp_out)
        return set_error(COME_E_INVALID, "null pointer");
    int dev;
    int rc = ensure_init(&dev);
    if (rc) return rc;
    RespArgs a{x, prec_chol, mu_prec, log_norm, resp_out, lse_out, V, d, K, nullptr};
    if (mfma) {
        int *flags = (int *)stream_scratch(dev, stream, kScratchGmmFlags, sizeof(int) * (K + 1));
        if (!flags) return scratch_failed();
        rc = hip_error(hipMemsetAsync(flags + K, 0, sizeof(int), (hipStream_t)stream),
                       "gmm_resp: flag reset");
        if (rc) return rc;
        hipLaunchKernelGGL(k_gmm_lower_flags, dim3(K), dim3(256), 0, (hipStream_t)stream,
                           prec_chol, d, flags, K);
        rc = hip_error(hipGetLastError(), "k_gmm_lower_flags launch");
        if (rc) return rc;
        a.lower = flags;
        float *pt = stream_scratch(dev, stream, kScratchGmmPt, sizeof(float) * (size_t)K * d * d);
        if (!pt) return scratch_failed();
        hipLaunchKernelGGL(k_transpose_sq, dim3((d / 32) * (d / 32), K), dim3(256), 0,
                           (hipStream_t)stream, prec_chol, d, pt);
        rc = hip_error(hipGetLastError(), "k_transpose_sq launch");
        if (rc) return rc;
        a.prec_t = pt;
        const int r16 = current_opts().gmm_resp16;
        if (r16 == 3) {
            // default: k_gmm_resp_b16 over the bf16-part images of the upper factors, then
            // k_gmm_resp16_full (a no-op unless some factor is lower or dense)
            const size_t img_bytes =
                (size_t)K * (d == 64 ? RespB16<64>::NB : RespB16<128>::NB) * RespB16<64>::BLK;
            char *img = (char *)stream_scratch(dev, stream, kScratchRespSplit, img_bytes);
            if (!img) return scratch_failed();
            const int64_t work = (int64_t)K * (d == 64 ? RespB16<64>::NB : RespB16<128>::NB) * 64;
            hipLaunchKernelGGL(d == 64 ? k_pack_upper_b16<64> : k_pack_upper_b16<128>,
                               dim3((unsigned)std::min<int64_t>((work + 255) / 256, 4096)),
                               dim3(256), 0, (hipStream_t)stream, prec_chol, img, K);
            rc = hip_error(hipGetLastError(), "k_pack_upper_b16 launch");
            if (rc) return rc;
            RespArgs b = a;
            b.prec_full = a.prec_t;
            b.prec_t = reinterpret_cast<const float *>(img);
            static bool attr3 = false;
            if (!attr3) {
                for (void (*f)(RespArgs) : {k_gmm_resp_b16<64>, k_gmm_resp_b16<128>,
                                            k_gmm_resp16_full<64>, k_gmm_resp16_full<128>})
                    (void)hipFuncSetAttribute((const void *)f,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                attr3 = true;
            }
            hipLaunchKernelGGL(d == 64 ? k_gmm_resp_b16<64> : k_gmm_resp_b16<128>,
                               dim3((unsigned)((V + 127) / 128)), dim3(512),
                               d == 64 ? RespB16<64>::LDS_BYTES : RespB16<128>::LDS_BYTES,
                               (hipStream_t)stream, b);
            rc = hip_error(hipGetLastError(), "k_gmm_resp_b16 launch");
            if (rc) return rc;
            const size_t lds16 = sizeof(float) * (size_t)(d == 64 ? Resp16Shape<64>::LDS
                                                                   : Resp16Shape<128>::LDS);
            const int64_t blks = (V + 127) / 128;
            hipLaunchKernelGGL(d == 64 ? k_gmm_resp16_full<64> : k_gmm_resp16_full<128>,
                               dim3((unsigned)std::min<int64_t>(blks, 2 * (int64_t)num_cus(dev))),
                               dim3(256), lds16, (hipStream_t)stream, b);
            return hip_error(hipGetLastError(), "k_gmm_resp16_full launch");
        }
        if (r16 == 2) {
            // default: k_gmm_resp16t over the packed non-zero blocks (every factor upper-
            // triangular), then k_gmm_resp16_full (a no-op unless some factor is lower or dense)
            const int tri = d == 64 ? Resp16T<64>::TRI : Resp16T<128>::TRI;
            float *packed = stream_scratch(dev, stream, kScratchGmmTri, sizeof(float) * (size_t)K * tri);
            if (!packed) return scratch_failed();
            hipLaunchKernelGGL(d == 64 ? k_pack_upper16<64> : k_pack_upper16<128>,
                               dim3((unsigned)((tri + 255) / 256), K), dim3(256), 0,
                               (hipStream_t)stream, prec_chol, packed);
            rc = hip_error(hipGetLastError(), "k_pack_upper16 launch");
            if (rc) return rc;
            RespArgs b = a;
            b.prec_full = a.prec_t;
            b.prec_t = packed;
            const size_t ldst = sizeof(float) * (size_t)(d == 64 ? Resp16T<64>::LDS : Resp16T<128>::LDS);
            const size_t lds16 = sizeof(float) * (size_t)(d == 64 ? Resp16Shape<64>::LDS
                                                                   : Resp16Shape<128>::LDS);
            static bool attr16t = false;
            if (!attr16t) {
                for (void (*f)(RespArgs) : {k_gmm_resp16t<64>, k_gmm_resp16t<128>,
                                            k_gmm_resp16_full<64>, k_gmm_resp16_full<128>})
                    (void)hipFuncSetAttribute((const void *)f,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                attr16t = true;
            }
            hipLaunchKernelGGL(d == 64 ? k_gmm_resp16t<64> : k_gmm_resp16t<128>,
                               dim3((unsigned)((V + R16tShape::ROWS - 1) / R16tShape::ROWS)),
                               dim3(R16tShape::THREADS), ldst,
                               (hipStream_t)stream, b);
            rc = hip_error(hipGetLastError(), "k_gmm_resp16t launch");
            if (rc) return rc;
            const int64_t blks = (V + 127) / 128;
            hipLaunchKernelGGL(d == 64 ? k_gmm_resp16_full<64> : k_gmm_resp16_full<128>,
                               dim3((unsigned)std::min<int64_t>(blks, 2 * (int64_t)num_cus(dev))),
                               dim3(256), lds16, (hipStream_t)stream, b);
            return hip_error(hipGetLastError(), "k_gmm_resp16_full launch");
        }
        return set_error(COME_E_INVALID, "gmm_resp16 must be 2 or 3 (got %d)", r16);
    }
    if (d > 128) {
        const size_t lds = sizeof(float) * ((size_t)2 * kTRW * d +
                                            (size_t)chunk_rows(d) * (d + 1) + kTRW);
        static bool attr_w = false;
        if (!attr_w) {
            (void)hipFuncSetAttribute((const void *)k_gmm_resp_wide,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr_w = true;
        }
        hipLaunchKernelGGL(k_gmm_resp_wide, dim3((unsigned)((V + kTRW - 1) / kTRW)),
                           dim3(kThreads), lds, (hipStream_t)stream, a);
        return hip_error(hipGetLastError(), "k_gmm_resp_wide launch");
    }
    const size_t lds = sizeof(float) * ((size_t)kTR * d + (size_t)d * d + kTR * 64 + kTR);
    const unsigned grid = (unsigned)((V + kTR - 1) / kTR);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)k_gmm_resp,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k_gmm_resp, dim3(grid), dim3(kThreads), lds, (hipStream_t)stream, a);
    return hip_error(hipGetLastError(), "k_gmm_resp launch");
}

extern "C" int come_gmm_scatter(const float *x, int64_t V, int d, const float *resp,
                                const float *means, int K, int chunks, float *scratch,
                                float *scatter_out, void *stream) {
    if (V < 0 || d < 1 || d > kMaxDim || K < 1 || chunks < 1 || chunks > 65535)
        return set_error(COME_E_INVALID, "gmm_scatter: need V>=0, 1<=d<=%d, K>=1, "
                                         "1<=chunks<=65535", kMaxDim);
    if (!x || !resp || !means || !scatter_out || (chunks > 1 && !scratch))
        return set_error(COME_E_INVALID, "null pointer");
    int dev;
    int rc = ensure_init(&dev);
    if (rc) return rc;
    const int64_t n = (int64_t)K * d * d;
    int64_t per = (V + chunks - 1) / chunks;
    per = (per + kCovRB - 1) / kCovRB * kCovRB;
    if (per < kCovRB) per = kCovRB;
    const int used = V == 0 ? 1 : (int)((V + per - 1) / per);
    CovArgs a{x, resp, means, used > 1 ? scratch : scatter_out, V, per, d, K};
    const bool mfma = (d == 64 || d == 128) && ((uintptr_t)x % 16) == 0;
    if (d > 128) {
        const int nt = (d + 63) / 64;
        const size_t lds = sizeof(float) * ((size_t)kCovWideRB * d + kCovWideRB);
        static bool attr_w = false;
        if (!attr_w) {
            (void)hipFuncSetAttribute((const void *)k_gmm_cov_wide,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr_w = true;
        }
        hipLaunchKernelGGL(k_gmm_cov_wide, dim3(K, used, nt * nt), dim3(kThreads), lds,
                           (hipStream_t)stream, a);
        rc = hip_error(hipGetLastError(), "k_gmm_cov_wide launch");
        if (rc || used == 1) return rc;
        hipLaunchKernelGGL(k_gmm_cov_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                           (hipStream_t)stream, (const float *)scratch, scatter_out, n, used);
        return hip_error(hipGetLastError(), "k_gmm_cov_reduce launch");
    }
    // gmm_cov_async: 4 (default) = k_gmm_cov_bf3 (bf16 parts), 3 = k_gmm_cov16 (fp32 16x16x4)
    const int cv = current_opts().gmm_cov_async;
    if (cv != 3 && cv != 4)
        return set_error(COME_E_INVALID, "gmm_cov_async must be 3 or 4 (got %d)", cv);
    if (mfma && cv == 4) {
        static bool attr4 = false;
        if (!attr4) {
            for (void (*f)(CovArgs) : {k_gmm_cov_bf3<64>, k_gmm_cov_bf3<128>})
                (void)hipFuncSetAttribute((const void *)f,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr4 = true;
        }
        const int cpw = d == 64 ? CovBf3<64>::CPW : CovBf3<128>::CPW;
        hipLaunchKernelGGL(d == 64 ? k_gmm_cov_bf3<64> : k_gmm_cov_bf3<128>,
                           dim3((K + cpw - 1) / cpw, used),
                           dim3(d == 64 ? CovBf3<64>::THREADS : CovBf3<128>::THREADS),
                           d == 64 ? CovBf3<64>::LDS_BYTES : CovBf3<128>::LDS_BYTES,
                           (hipStream_t)stream, a);
        rc = hip_error(hipGetLastError(), "k_gmm_cov_bf3 launch");
        if (rc || used == 1) return rc;
        hipLaunchKernelGGL(k_gmm_cov_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                           (hipStream_t)stream, (const float *)scratch, scatter_out, n, used);
        return hip_error(hipGetLastError(), "k_gmm_cov_reduce launch");
    }
    void (*kern)(CovArgs) = !mfma ? k_gmm_cov_valu : (d == 64 ? k_gmm_cov16<64> : k_gmm_cov16<128>);
    const int threads = !mfma ? 256 : (d == 64 ? Cov16<64>::THREADS : Cov16<128>::THREADS);
    const int cpw = !mfma ? 1 : (d == 64 ? Cov16<64>::CPW : Cov16<128>::CPW);
    hipLaunchKernelGGL(kern, dim3((K + cpw - 1) / cpw, used), dim3(threads), 0,
                       (hipStream_t)stream, a);
    rc = hip_error(hipGetLastError(), "k_gmm_cov launch");
    if (rc || used == 1) return rc;
    hipLaunchKernelGGL(k_gmm_cov_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, (const float *)scratch, scatter_out, n, used);
    return hip_error(hipGetLastError(), "k_gmm_cov_reduce launch");
}
