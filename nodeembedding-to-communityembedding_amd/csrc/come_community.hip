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
#include <math.h>
#include <stdint.h>

#include "come_internal.h"

namespace come {

constexpr int kTR = 16;        // rows per workgroup tile
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
    int64_t V;
    int d;
    int K;
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
    }
}

}  // namespace come

using namespace come;

extern "C" int come_community_grad(float *x, int64_t V, int d, const float *pi, const float *mu,
                                   const float *inv_cov, int K, float beta, float lr, int iters,
                                   void *stream) {
    if (V < 0 || d < 1 || d > 128 || K < 1 || iters < 0)
        return set_error(COME_E_INVALID, "community_grad: need V>=0, 1<=d<=128, K>=1, iters>=0");
    if (V == 0 || iters == 0) return COME_OK;
    if (!x || !pi || !mu || !inv_cov) return set_error(COME_E_INVALID, "null pointer");
    int dev;
    int rc = ensure_init(&dev);
    if (rc) return rc;
    CommArgs a{x, pi, mu, inv_cov, V, d, K, (float)((double)beta / (double)K), lr, iters};
    const size_t lds = sizeof(float) * ((size_t)3 * kTR * d + (size_t)d * d);
    const unsigned grid = (unsigned)((V + kTR - 1) / kTR);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)k_community_grad,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k_community_grad, dim3(grid), dim3(kThreads), lds, (hipStream_t)stream, a);
    return hip_error(hipGetLastError(), "k_community_grad launch");
}

extern "C" int come_gmm_resp(const float *x, int64_t V, int d, const float *prec_chol,
                             const float *mu_prec, const float *log_norm, int K, float *resp_out,
                             void *stream) {
    if (V < 0 || d < 1 || d > 128 || K < 1 || K > 64)
        return set_error(COME_E_INVALID, "gmm_resp: need V>=0, 1<=d<=128, 1<=K<=64");
    if (V == 0) return COME_OK;
    if (!x || !prec_chol || !mu_prec || !log_norm || !resp_out)
        return set_error(COME_E_INVALID, "null pointer");
    int dev;
    int rc = ensure_init(&dev);
    if (rc) return rc;
    RespArgs a{x, prec_chol, mu_prec, log_norm, resp_out, V, d, K};
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
