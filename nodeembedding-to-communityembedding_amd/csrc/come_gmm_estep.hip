// come_gmm_estep.hip -- GMM responsibilities, the E-step (gfx950).
//
// Replaces GaussianMixture.predict_proba / _e_step (community_embeddings.py:27,37,
// covariance_type='full'): come_gmm_estep / come_gmm_resp -> k_gmm_resp_b16 (default, fp32 operands
// as bf16 parts), k_gmm_resp16t (fp32 MFMA), k_gmm_resp16_full (lower or dense factors),
// k_gmm_resp / k_gmm_resp_wide (VALU, any d).  2*V*K*d^2 flops per pass (half of it skipped on the
// upper-triangular precision factors sklearn keeps).

#include "come_c4.h"

namespace come {

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

// GMM responsibilities, shared steps.  Triangular skip: sklearn's precisions_cholesky_ after an
// M-step is UPPER triangular (solve_triangular(chol(cov), I, lower=True).T), so a column tile of
// Y = X P_k only needs the features up to its last column.  k_gmm_lower_flags marks the components
// with a non-zero below the diagonal (a lower factor, e.g. sklearn's cholesky(precisions_init,
// lower=True)) and ORs them into flags[K]; a launch holding one runs the full-body kernel
// (k_gmm_resp16_full) instead of the skipping one.  The skipped MFMAs would only add exact zeros.
__global__ void __launch_bounds__(256) k_gmm_lower_flags(const float *__restrict__ P, int D,
                                                         int *__restrict__ flags, int K) {
    const float *Pk = P + (int64_t)blockIdx.x * D * D;
    // the strictly lower triangle only, 16 lanes per row segment (no per-element division)
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    int nz = 0;
    for (int r = 1 + ty; r < D; r += 16)
        for (int c = tx; c < r; c += 16) nz |= Pk[(int64_t)r * D + c] != 0.0f;
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
// A row's responsibilities from its stored log-probabilities: the row's four lanes (group kg)
// take components k = kg, kg + 4, ..., each lane's loads issued as a batch of up to 16 before any
// exp or store (one memory round trip where one lane walking all K took K); the last component's
// value comes from the register that would have stored it.
__device__ __forceinline__ void resp_normalize(float *lp, int K, float lp_last, float lse, int kg) {
    for (int k0 = kg; k0 < K; k0 += 64) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int k = k0 + 4 * u;
            v[u] = k < K - 1 ? lp[k] : lp_last;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int k = k0 + 4 * u;
            if (k < K) lp[k] = expf(v[u] - lse);
        }
    }
}

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
    if (rowok) {  // the row's four lanes (the reduction left the sums in all of them)
        const float lse = run_max + logf(run_sum);
        resp_normalize(a.resp + row * a.K, a.K, lp_prev, lse, kg);
        if (a.lse && kg == 0) a.lse[row] = lse;
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

}  // namespace come

using namespace come;

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
