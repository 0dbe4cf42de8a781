// come_community.hip -- community-embedding step (gfx950).
//
// Replaces /root/reference/ADSCModel/community_embeddings.py:
//   Community2Vec.train (:61-78)  -> come_community_grad: k_community_b16 (default, fp32 operands as
//   bf16 parts), k_community16 (fp32 MFMA), k_community_grad / k_community_grad_wide (VALU, any d)
//
// A dense contraction, 2*V*K*d^2 flops per pass: each component's d x d matrix streams through LDS
// and the per-component matrix-vector products accumulate in registers.  Rows are independent
// (community_embeddings.py:65 takes a snapshot per iteration and every row's gradient reads only
// its own row), so the `iters` loop runs inside the kernel and x is written back once.

#include "come_c4.h"

namespace come {

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
