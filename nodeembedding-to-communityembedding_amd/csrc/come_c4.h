// come_c4.h -- what the C4 kernels share (gfx950): argument blocks, the bf16-part arithmetic,
// launch constants and A/B hooks.  Included by come_community.hip (community step),
// come_gmm_estep.hip (GMM responsibilities) and come_gmm_scatter.hip (M-step scatter matrices).
#pragma once

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
// k_gmm_cov_fb3 (A/B hooks): staging register sets (loads NS blocks ahead; 2: 4.64 vs 4.84 ms with
// 3 at C4 with SYMU, which at 3 sets needs all 256 VGPRs) and the diagonal tiles' cross terms as
// U + U^T (0: six MFMAs per diagonal tile as k_gmm_cov_bf3, bit-identical to it; 1: four, 3-5%
// faster)
#ifndef COME_COVF_NS
#define COME_COVF_NS 2
#endif
#ifndef COME_COVF_SYMU
#define COME_COVF_SYMU 1
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

// ---- wide rows (128 < d <= 512): VALU forms with the d x d matrices streamed in row chunks ----
// The MFMA kernels above keep a whole d x d matrix (or a 128-row tile of inputs) in LDS, which
// stops at d = 128.  These forms cover every d up to kMaxDim: kTRW rows per workgroup, each
// component's matrix staged kChunkRows(d) rows at a time (<= 64 KiB, rows padded by one float
// against bank conflicts).  Same arithmetic as k_community_grad / k_gmm_resp (fmaf chains in j
// order), a fraction of the MFMA rate: they exist so that every embedding size the SGNS kernels
// accept also trains through the community step (community_embeddings.py:61-78) and the GMM.
constexpr int kTRW = 8;
__host__ __device__ inline int chunk_rows(int d) { return 16384 / (d + 1); }

}  // namespace come
