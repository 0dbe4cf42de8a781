// come_gmm_scatter.hip -- GMM M-step scatter matrices (gfx950).
//
// Replaces the numerator of sklearn's _estimate_gaussian_covariances_full (community_embeddings.py
// :27 fit): come_gmm_scatter -> k_gmm_cov_fb3 (default at d = 128) and k_gmm_cov_bf3 (d = 64; fp32
// operands as bf16 parts), k_gmm_cov16 (fp32 MFMA), k_gmm_cov_valu / k_gmm_cov_wide (VALU, any d),
// k_gmm_cov_reduce (chunk partials in a fixed order).

#include "come_c4.h"

namespace come {

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
    int upper_only;  // 32-wide-tile kernels writing chunk partials: only the upper tiles (the
                     // reduction mirrors them), no transposed (uncoalesced) stores
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
    // index of tile n of part p among that part's diagonal tiles
    constexpr int dslot(int p, int n) const {
        int c = 0;
        for (int m = 0; m < n; ++m) c += ta[p][m] == tb[p][m];
        return c;
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
            if (ta != tb && !a.upper_only) out[(int64_t)jj * D + ii] = acc[n][r];
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
    // cov16_staging's look-ahead is Cov16<D>::NBUF - 1 blocks, while CovBf3Stage::stage and
    // covbf3_part index the image buffers by blk % 2 / j & 1: the two must agree
    static_assert(Cov16<D>::NBUF == 2, "k_gmm_cov_bf3 assumes two image buffers");
    CovBf3Stage<D> sg(a, tid - 64 * C::AW, lane, k0, nk, c0, c1);
    cov16_staging<D>(reinterpret_cast<float *>(smb), sg, nb);
}

// ---- M-step scatter with the staging inside the MFMA wavefronts (k_gmm_cov_fb3, d = 128) -------
//
// k_gmm_cov_bf3's arithmetic (E = sqrt(r) (x - m) as three bf16 parts, six exact part products per
// multiply-add on 32x32x16 bf16 MFMAs, the 10 upper 32x32 tiles) without specialised wavefronts:
// each of the 4 wavefronts (one per SIMD) owns 5 tiles of one of the workgroup's 2 components AND
// stages one sample x 8 features of the next block for both components, so a SIMD's staging VALU
// issues in the gaps of its own MFMA stream (a 32x32x16 MFMA holds the SIMD's vector issue for 8
// of its 32 cycles) instead of competing with it from other wavefronts.  Blocks are 16 samples
// (one k-step), so a workgroup holds 48 KB of LDS and two run per CU: one's barrier waits fill
// with the other's MFMAs.  The images are sample-major (row = sample: 128 features x 2 B per part)
// and the MFMA fragments are read with ds_read_b64_tr_b16 (a 16-lane group receives a 4-sample x
// 16-feature block transposed: lane i gets feature i of the 4 samples), so a staging lane's weight
// is its own sample's (no broadcast) and its x is two 16-byte loads.  Diagonal tiles take their
// cross terms a1 b2 + a2 b1 + a1 b3 + a3 b1 as U + U^T, U = a1 b2 + a1 b3: four MFMAs instead of six,
// U^T added once at the end (COME_COVF_SYMU).
template <int D>
struct CovFb3 {
    static_assert(D == 128, "k_gmm_cov_fb3 covers d = 128 (k_gmm_cov_bf3 takes d = 64)");
    static constexpr int RB = 16;                // samples per block (one k-step)
    static constexpr int CPW = 2;                // components per workgroup
    static constexpr int THREADS = 256;          // wavefront w: component w / 2, tiles part w % 2
    static constexpr int NF = D / 32;            // 32-feature fragments
    static constexpr int PLANE = D * RB * 2;     // bytes per part image (4 KB)
    static constexpr int IMG = 3 * PLANE;        // per component
    static constexpr int BUF = CPW * IMG;        // 24 KB
    static constexpr int LDS_BYTES = 2 * BUF;    // 48 KB
    static constexpr int NS = COME_COVF_NS;      // staging register sets (loads NS blocks ahead)
    // chunk ch (16 B, 8 features) of sample row r of part P: chunks XOR-swizzled by the row, so each
    // tr read's 32-lane half (4 rows x 4 chunks x two 8-B halves: 256 B) and each 8-lane
    // ds_write_b128 group (8 chunks of one row: 128 B) cover distinct banks
    __host__ __device__ static constexpr int at(int P, int r, int ch) {
        return P * PLANE + r * (D * 2) + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3)));
    }
};

template <int D, int P>
__device__ __forceinline__ void covfb3_body(const CovArgs &a, char *smb, int nb, int k0, int nk,
                                               int64_t c0, int64_t c1, int64_t chunk, int wid,
                                               int lane) {
    using C = CovFb3<D>;
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    using f32x16 = __attribute__((ext_vector_type(16))) float;
    typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
    typedef short s16x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    constexpr CovBf3Tiles<D> TT{};
    constexpr int NT = TT.cnt[P], NS = C::NS;
    const int tk = wid >> 1;
    const int i = lane & 31, h = lane >> 5;
    // staging role: sample s = 4 wid + lane / 16 of each block, features 8 ch .. 8 ch + 7
    const int s = 4 * wid + (lane >> 4), ch = lane & 15;
    float mu[2][8];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int e = 0; e < 8; ++e)
            mu[kk][e] = kk < nk ? a.means[(int64_t)(k0 + kk) * D + 8 * ch + e] : 0.0f;
    f32x4 xv[NS][2];
    float rv[NS][2];
    const int lastr = (int)(c1 - c0) - 1;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(a.x + c0 * D), 0, (int)((c1 - c0) * D * (int64_t)sizeof(float)),
        0x00020000);
    // the chunk's responsibilities rows, as a buffer too (32-bit lane offsets)
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(a.resp + c0 * a.K), 0, (int)((c1 - c0) * a.K * (int64_t)sizeof(float)),
        0x00020000);
    const int kc0 = 4 * k0, kc1 = 4 * min(k0 + 1, a.K - 1);
    auto load = [&](int u, int blk) {
        const int row = min(blk * C::RB + s, lastr);  // rows clamped to the chunk (zero weight)
        const int off = row * (D * 4) + 32 * ch;
        xv[u][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
        xv[u][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, off + 16, 0, 0));
        const int roff = row * a.K * 4;
        rv[u][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, roff, kc0, 0));
        rv[u][1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, roff, kc1, 0));
    };
    auto stage = [&](int u, int blk) {
        char *buf = smb + (blk & 1) * C::BUF;
        const bool live = blk * C::RB + s <= lastr;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            // sqrt(r) by v_sqrt_f32 (within 1 ulp; the correctly rounded sqrtf would add ~16 VALU
            // per block), 0 past the chunk or K: those E values are exact zeros
            float w = __builtin_amdgcn_sqrtf(rv[u][kk]);
            w = live && kk < nk ? w : 0.0f;
            uint32_t p1[4], p2[4], p3[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float v0 = w * (xv[u][e >> 1][2 * (e & 1)] - mu[kk][2 * e]);
                const float v1 = w * (xv[u][e >> 1][2 * (e & 1) + 1] - mu[kk][2 * e + 1]);
                bf16_split3(v0, v1, p1[e], p2[e], p3[e]);
            }
            char *im = buf + kk * C::IMG;
            *reinterpret_cast<uint4 *>(im + C::at(0, s, ch)) = uint4{p1[0], p1[1], p1[2], p1[3]};
            *reinterpret_cast<uint4 *>(im + C::at(1, s, ch)) = uint4{p2[0], p2[1], p2[2], p2[3]};
            *reinterpret_cast<uint4 *>(im + C::at(2, s, ch)) = uint4{p3[0], p3[1], p3[2], p3[3]};
        }
    };
    f32x16 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[n][e] = 0.0f;
    constexpr int NDG = COME_COVF_SYMU ? 2 : 1;
    f32x16 accu[NDG];
#pragma unroll
    for (int n = 0; n < NDG; ++n)
#pragma unroll
        for (int e = 0; e < 16; ++e) accu[n][e] = 0.0f;
    // fragment fr of block blk: lane (group g16 = lane / 16, i16 = lane % 16) receives feature
    // 32 fr + 16 (g16 & 1) + i16 of samples 8 (g16 / 2) + 4 t + 0..3 from read t; it supplies the
    // address of row 8 (g16 / 2) + 4 t + i16 / 4, features 32 fr + 16 (g16 & 1) + 4 (i16 % 4) .. + 3
    const int g16 = lane >> 4, i16 = lane & 15;
    auto read_frags = [&](bf16x8 (&F)[C::NF][3], int blk) {
        const char *im = smb + (blk & 1) * C::BUF + tk * C::IMG;
#pragma unroll
        for (int fr = 0; fr < C::NF; ++fr) {
            if (!TT.need[P][fr]) continue;
            const int cb = 4 * fr + 2 * (g16 & 1) + ((i16 & 3) >> 1);
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                s16x4 t2[2];
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const int r = 8 * (g16 >> 1) + 4 * t + (i16 >> 2);
                    const char *ad = im + C::at(p, r, cb) + 8 * (i16 & 1);
                    t2[t] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(ad));
                }
                const uint2 lo = __builtin_bit_cast(uint2, t2[0]), hi = __builtin_bit_cast(uint2, t2[1]);
                F[fr][p] = __builtin_bit_cast(bf16x8, uint4{lo.x, lo.y, hi.x, hi.y});
            }
        }
    };
    auto mfma_block = [&](const bf16x8 (&F)[C::NF][3]) {
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int ta = TT.ta[P][n], tb = TT.tb[P][n];
            if (COME_COVF_SYMU && ta == tb) {
                const int dg = TT.dslot(P, n);
                accu[dg] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][0], F[tb][2], accu[dg], 0, 0, 0);
                accu[dg] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][0], F[tb][1], accu[dg], 0, 0, 0);
                acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][1], F[tb][1], acc[n], 0, 0, 0);
                acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][0], F[tb][0], acc[n], 0, 0, 0);
                continue;
            }
            acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][2], F[tb][0], acc[n], 0, 0, 0);
            acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][1], F[tb][1], acc[n], 0, 0, 0);
            acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][0], F[tb][2], acc[n], 0, 0, 0);
            acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][1], F[tb][0], acc[n], 0, 0, 0);
            acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][0], F[tb][1], acc[n], 0, 0, 0);
            acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[ta][0], F[tb][0], acc[n], 0, 0, 0);
        }
    };
    if (nb > 0) {
#pragma unroll
        for (int u = 0; u < NS; ++u) load(u, u);
        stage(0, 0);
        load(0, NS);
        __syncthreads();
        for (int j0 = 0; j0 < nb; j0 += NS) {
#pragma unroll
            for (int u = 0; u < NS; ++u) {
                const int j = j0 + u;  // multiply block j, stage block j + 1 from set (u + 1) % NS
                bf16x8 F[C::NF][3];
                read_frags(F, j);
                stage((u + 1) % NS, j + 1);
                load((u + 1) % NS, j + 1 + NS);
                mfma_block(F);
                __syncthreads();  // block j + 1 staged; block j's buffer free
            }
        }
    }
    if (tk >= nk) return;  // wavefront-uniform: K not a multiple of CPW
#if COME_COVF_SYMU
    if (nb > 0) {
        float *ut = reinterpret_cast<float *>(smb) + wid * (NDG * 32 * 33);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            if (TT.ta[P][n] != TT.tb[P][n]) continue;
            const int dg = TT.dslot(P, n);
            float *u = ut + dg * 32 * 33;
#pragma unroll
            for (int r = 0; r < 16; ++r) u[((r & 3) + 8 * (r >> 2) + 4 * h) * 33 + i] = accu[dg][r];
#pragma unroll
            for (int r = 0; r < 16; ++r)
                acc[n][r] += accu[dg][r] + u[i * 33 + (r & 3) + 8 * (r >> 2) + 4 * h];
        }
    }
#endif
    float *out = a.out + (chunk * a.K + k0 + tk) * D * D;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int ta = TT.ta[P][n], tb = TT.tb[P][n];
        const int jj = 32 * tb + i;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int ii = 32 * ta + (r & 3) + 8 * (r >> 2) + 4 * h;
            out[(int64_t)ii * D + jj] = acc[n][r];
            if (ta != tb && !a.upper_only) out[(int64_t)jj * D + ii] = acc[n][r];
        }
    }
}

template <int D>
__global__ void __launch_bounds__(CovFb3<D>::THREADS) __attribute__((amdgpu_waves_per_eu(2)))
    k_gmm_cov_fb3(CovArgs a) {
    using C = CovFb3<D>;
    extern __shared__ __attribute__((aligned(16))) char smb[];
    const int64_t chunk = blockIdx.y;
    const int k0 = blockIdx.x * C::CPW;
    const int nk = a.K - k0 < C::CPW ? a.K - k0 : C::CPW;
    const int64_t c0 = chunk * a.rows_per_chunk;
    int64_t c1 = c0 + a.rows_per_chunk;
    if (c1 > a.V) c1 = a.V;
    const int nb = c1 > c0 ? (int)((c1 - c0 + C::RB - 1) / C::RB) : 0;
    const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    if (wid & 1) covfb3_body<D, 1>(a, smb, nb, k0, nk, c0, c1, chunk, wid, lane);
    else covfb3_body<D, 0>(a, smb, nb, k0, nk, c0, c1, chunk, wid, lane);
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

// out[i] = sum_c part[c][i] in chunk order (deterministic), i over K d^2 entries.  Four entries
// per thread (16-byte loads when n % 4 == 0) and eight chunks' loads issued ahead of their adds,
// which stay in chunk order: 534 MB of partials at C4 in 0.17 ms as one dword and one chunk at a
// time per thread.
template <bool VEC4>
__global__ void __launch_bounds__(256) k_gmm_cov_reduce(const float *part, float *out, int64_t n,
                                                        int chunks) {
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;  // entries 4 q .. 4 q + 3
    if (4 * q >= n) return;
    if (VEC4) {
        const f32x4 *p = reinterpret_cast<const f32x4 *>(part) + q;
        const int64_t stride = n / 4;
        f32x4 s = {0.0f, 0.0f, 0.0f, 0.0f};
        int c = 0;
        for (; c + 8 <= chunks; c += 8) {
            f32x4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(c + u) * stride];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; c < chunks; ++c) s += p[(int64_t)c * stride];
        reinterpret_cast<f32x4 *>(out)[q] = s;
    } else {
        for (int64_t i = 4 * q; i < 4 * q + 4 && i < n; ++i) {
            float s = 0.0f;
            for (int c = 0; c < chunks; ++c) s += part[(int64_t)c * n + i];
            out[i] = s;
        }
    }
}

// The 32-wide-tile kernels' partials hold only the upper tiles (CovArgs::upper_only): the threads
// cover the upper tiles only -- thread q of component k takes upper tile t = (q / 256) % NTU
// (row-major order of the upper triangle), row r = (q % 256) / 8 and columns 4 g .. 4 g + 3
// (g = q % 8) of it, eight lanes per 128-byte tile row -- sums them over the chunks (16-byte loads,
// eight chunks in flight, in chunk order) and writes them and their mirror images.
template <int D>
__global__ void __launch_bounds__(256) k_gmm_cov_reduce_upper(const float *part, float *out,
                                                                int64_t n, int chunks, int K) {
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    constexpr int NT = D / 32, NTU = NT * (NT + 1) / 2;
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= (int64_t)K * NTU * 256) return;
    const int k = (int)(q / (NTU * 256)), w = (int)(q % 256);
    int t = (int)((q / 256) % NTU), ti = 0;
    while (t >= NT - ti) {  // upper tile t -> (ti, tj), tj >= ti
        t -= NT - ti;
        ++ti;
    }
    const int tj = ti + t, i = 32 * ti + w / 8, j = 32 * tj + 4 * (w % 8);
    const int64_t e = (int64_t)k * D * D + (int64_t)i * D + j;
    const f32x4 *p = reinterpret_cast<const f32x4 *>(part + e);
    const int64_t stride = n / 4;
    f32x4 s = {0.0f, 0.0f, 0.0f, 0.0f};
    int c = 0;
    for (; c + 8 <= chunks; c += 8) {
        f32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(c + u) * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; c < chunks; ++c) s += p[(int64_t)c * stride];
    *reinterpret_cast<f32x4 *>(out + e) = s;
    if (tj > ti) {
        float *m = out + (int64_t)k * D * D + (int64_t)j * D + i;  // (j, i)
#pragma unroll
        for (int u = 0; u < 4; ++u) m[(int64_t)u * D] = s[u];
    }
}

static int launch_cov_reduce(const float *part, float *out, int64_t n, int chunks,
                             hipStream_t stream) {
    const unsigned grid = (unsigned)((n + 1023) / 1024);
    if (n % 4 == 0)
        hipLaunchKernelGGL(k_gmm_cov_reduce<true>, dim3(grid), dim3(256), 0, stream, part, out, n,
                           chunks);
    else
        hipLaunchKernelGGL(k_gmm_cov_reduce<false>, dim3(grid), dim3(256), 0, stream, part, out, n,
                           chunks);
    return hip_error(hipGetLastError(), "k_gmm_cov_reduce launch");
}

static int launch_cov_reduce_upper(const float *part, float *out, int64_t n, int chunks, int d,
                                   hipStream_t stream) {
    const int K = (int)(n / ((int64_t)d * d)), ntu = (d / 32) * (d / 32 + 1) / 2;
    const unsigned grid = (unsigned)(((int64_t)K * ntu * 256 + 255) / 256);
    if (d == 64)
        hipLaunchKernelGGL(k_gmm_cov_reduce_upper<64>, dim3(grid), dim3(256), 0, stream, part, out,
                           n, chunks, K);
    else
        hipLaunchKernelGGL(k_gmm_cov_reduce_upper<128>, dim3(grid), dim3(256), 0, stream, part,
                           out, n, chunks, K);
    return hip_error(hipGetLastError(), "k_gmm_cov_reduce_upper launch");
}

// ---- M-step parameters + E-step constants (come_gmm_params) ----------------------------------
//
// One workgroup per component, float64 in LDS (d <= 128: 128 x 129 doubles = 129 KB): cov =
// S / nk + reg I (sklearn _estimate_gaussian_covariances_full), the right-looking Cholesky
// factorisation in place (U = L^T in the upper triangle), then prec_chol = L^-T = U^-1 bottom-up by
// rows with two lanes of one wavefront per column (sklearn _compute_precision_cholesky:
// solve_triangular(L, I).T): a column's values are written and read by its own wavefront only, so
// the inverse needs no barrier.  Then the E-step's fp32 inputs.  Replaces ~30 small launches (torch
// cholesky_ex / solve_triangular / einsum) and a host sync per EM iteration.
struct ParamsArgs {
    const double *__restrict__ S, *__restrict__ nk, *__restrict__ means, *__restrict__ weights;
    int K, d;
    double reg;
    double *cov, *pc;
    float *e_pc, *e_mp, *e_ln;
    int *info;
};

// Right-looking Cholesky steps j .. j + NB - 1 in one phase (no barrier inside).  Step m turns
// A^(m) into A^(m+1)[i][c] = A^(m)[i][c] - t_m(i) A^(m)[c][j + m], t_m(i) = A^(m)[i][j + m] / pivot_m.
// Each thread recomputes, in registers and in exactly that order, the panel values A^(m)[i][j + m]
// it needs (the same expressions as one step per barrier, so the factor is bit-identical), writes
// rows j + m of U = L^T to the upper triangle and the NB steps' trailing update to the lower --
// disjoint from every read of the phase.
template <int NB>
__device__ __forceinline__ void chol_panel(double *A, int LD, int d, int j, int tid, double *ld,
                                           int *bad) {
    const int tx = tid & 15, ty = tid >> 4;
    double P[NB][NB], ra[NB], lk[NB];  // P[k][m] = A^(m)[j + k][j + m], m < k
    bool okv[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        double t[NB];
#pragma unroll
        for (int m = 0; m <= k; ++m) {
            double x = A[(j + k) * LD + j + m];
#pragma unroll
            for (int q = 0; q < m; ++q) x = x - t[q] * P[m][q];
            if (m < k) {
                P[k][m] = x;
                t[m] = x * ra[m];
            } else {
                okv[k] = x > 0.0;
                lk[k] = sqrt(okv[k] ? x : 1.0);
                ra[k] = 1.0 / (okv[k] ? x : 1.0);
            }
        }
    }
    if (tid == 0) {
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            ld[j + k] = lk[k];
            if (!okv[k] && *bad == 0) *bad = j + k + 1;
        }
    }
    // U rows j + m: U[j + m][i] = A^(m)[i][j + m] / L[j + m][j + m] for i > j + m
    for (int i = j + 1 + tid; i < d; i += 256) {
        double t[NB];
#pragma unroll
        for (int m = 0; m < NB; ++m) {
            if (j + m >= i) break;
            double x = A[i * LD + j + m];
#pragma unroll
            for (int q = 0; q < m; ++q) x = x - t[q] * P[m][q];
            t[m] = x * ra[m];
            A[(j + m) * LD + i] = x / lk[m];
        }
    }
    // trailing rows / columns from j + NB: the thread's columns cc = j + NB + tx + 16 n with their
    // panel values in registers, then each row's elements loaded, updated by the NB steps, stored
    double c[NB][8];
#pragma unroll
    for (int n = 0; n < 8; ++n) {
        const int cc = j + NB + tx + 16 * n;
        double t[NB];
#pragma unroll
        for (int m = 0; m < NB; ++m) {
            double x = cc < d ? A[cc * LD + j + m] : 0.0;
#pragma unroll
            for (int q = 0; q < m; ++q) x = x - t[q] * P[m][q];
            t[m] = x * ra[m];
            c[m][n] = x;
        }
    }
    for (int ii = j + NB + ty; ii < d; ii += 16) {
        double t[NB];
#pragma unroll
        for (int m = 0; m < NB; ++m) {
            double x = A[ii * LD + j + m];
#pragma unroll
            for (int q = 0; q < m; ++q) x = x - t[q] * P[m][q];
            t[m] = x * ra[m];
        }
        double v[8];
#pragma unroll
        for (int n = 0; n < 8; ++n) {
            const int cc = j + NB + tx + 16 * n;
            v[n] = cc <= ii ? A[ii * LD + cc] : 0.0;
        }
#pragma unroll
        for (int n = 0; n < 8; ++n) {
            const int cc = j + NB + tx + 16 * n;
            double y = v[n];
#pragma unroll
            for (int m = 0; m < NB; ++m) y = y - t[m] * c[m][n];
            if (cc <= ii) A[ii * LD + cc] = y;
        }
    }
}

// Rows r, r - 1, .., r - R + 1 of P = U^-1 for the lane pair of column c (h: the parity of q it
// sums): the R dots over q > r share the loads of P[q][c]; then row r - k adds U[r - k][q] P[q][c]
// for q = r, r - 1, .., r - k + 1 from registers before its dot.  P[q][c] (q < c) sits at A[c][q],
// the diagonal in pd.  Written by the h = 0 lane; read back only by this wavefront.
template <int R>
__device__ __forceinline__ void inv_rows(double *A, int LD, int d, int r, int c, int h,
                                         double pdc, const double *pd) {
    double S[R];
#pragma unroll
    for (int k = 0; k < R; ++k) S[k] = 0.0;
    if (c < d && c > r) {
        double s[R][4];
#pragma unroll
        for (int k = 0; k < R; ++k) s[k][0] = s[k][1] = s[k][2] = s[k][3] = 0.0;
        int q = r + 1 + h;
        for (; q + 6 < c; q += 8) {
            const double p0 = A[c * LD + q], p1 = A[c * LD + q + 2];
            const double p2 = A[c * LD + q + 4], p3 = A[c * LD + q + 6];
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const double *u = A + (r - k) * LD + q;
                s[k][0] += u[0] * p0;
                s[k][1] += u[2] * p1;
                s[k][2] += u[4] * p2;
                s[k][3] += u[6] * p3;
            }
        }
        for (; q <= c; q += 2) {
            const double pq = q == c ? pdc : A[c * LD + q];
#pragma unroll
            for (int k = 0; k < R; ++k) s[k][0] += A[(r - k) * LD + q] * pq;
        }
#pragma unroll
        for (int k = 0; k < R; ++k) S[k] = (s[k][0] + s[k][1]) + (s[k][2] + s[k][3]);
    }
    double O[R];
#pragma unroll
    for (int k = 0; k < R; ++k) O[k] = __shfl_xor(S[k], 1);
    if (h == 0 && c < d && c >= r - R + 1) {
        double Pv[R];  // P[r - k][c]
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int rk = r - k;
            if (c <= rk) {
                Pv[k] = c == rk ? pd[rk] : 0.0;
                continue;
            }
            double acc;
            if (k == 0) {
                acc = S[0] + O[0];
            } else {
                acc = A[rk * LD + r] * Pv[0];
#pragma unroll
                for (int m = 1; m < k; ++m) acc = acc + A[rk * LD + r - m] * Pv[m];
                acc = acc + (S[k] + O[k]);
            }
            Pv[k] = -acc * pd[rk];
            A[c * LD + rk] = Pv[k];
        }
    }
}

// Cholesky columns per barrier and inverse rows per round (scripts/params_ab.py at K = 50, d = 128:
// 8 / 4 -> 0.190 ms, 4 / 4 0.198, 8 / 2 0.215, 4 / 2 0.223; profiles/r07_ab_gmm_params6.txt)
constexpr int kParamsNB = 8, kParamsInvR = 4;

__global__ void __launch_bounds__(256) k_gmm_params(ParamsArgs p) {
    extern __shared__ __attribute__((aligned(16))) double A[];  // [d][d + 1]
    __shared__ double ld[128], pd[128], mus[128], red[256];
    __shared__ int bad;
    const int k = blockIdx.x, d = p.d, LD = d + 1, tid = threadIdx.x, dd = d * d;
    const int tx = tid & 15, ty = tid >> 4;
    const double *__restrict__ S = p.S + (int64_t)k * dd;
    double *__restrict__ cov = p.cov + (int64_t)k * dd;
    const double nkk = p.nk[k];
    // S / nk[:, None, None] + reg I (the torch path's order), 16 coalesced loads in flight per lane
    for (int base = tid; base < dd; base += 256 * 16) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = base + 256 * u < dd ? S[base + 256 * u] : 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = base + 256 * u;
            if (e >= dd) break;
            const int i = e / d, j = e - i * d;
            const double c = i == j ? v[u] / nkk + p.reg : v[u] / nkk;
            cov[e] = c;
            A[i * LD + j] = c;
        }
    }
    if (tid < d) mus[tid] = p.means[(int64_t)k * d + tid];
    if (tid == 0) bad = 0;
    __syncthreads();
    // Cholesky, right-looking, four columns per barrier (chol_panel)
    int j = 0;
    for (; j + kParamsNB <= d; j += kParamsNB) {
        chol_panel<kParamsNB>(A, LD, d, j, tid, ld, &bad);
        __syncthreads();
    }
    if (kParamsNB > 4 && j + 4 <= d) {
        chol_panel<4>(A, LD, d, j, tid, ld, &bad);
        __syncthreads();
        j += 4;
    }
    if (j + 2 <= d) {
        chol_panel<2>(A, LD, d, j, tid, ld, &bad);
        __syncthreads();
        j += 2;
    }
    if (j < d) {
        chol_panel<1>(A, LD, d, j, tid, ld, &bad);
        __syncthreads();
    }
    // P = U^-1 = L^-T (upper), bottom-up by rows: P[r][c] = -(sum_{r<q<=c} U[r][q] P[q][c]) /
    // U[r][r]; P[q][c] (q < c) kept in the lower triangle at A[c][q], its diagonal in pd.  Column
    // c = tid / 2 belongs to lanes 2c, 2c + 1 of one wavefront, which split the dot by the parity
    // of q (four partial sums each) and combine by a lane exchange: every P value a lane reads was
    // written by its own wavefront at an earlier row (LDS accesses of a wavefront are ordered), so
    // the rows need no barrier.
    for (int r = tid; r < d; r += 256) pd[r] = 1.0 / ld[r];
    __syncthreads();
    {
        const int c = tid >> 1, h = tid & 1;
        const double pdc = c < d ? pd[c] : 0.0;
        int r = d - 2;
        for (; r >= kParamsInvR - 1; r -= kParamsInvR)
            inv_rows<kParamsInvR>(A, LD, d, r, c, h, pdc, pd);
        if (kParamsInvR > 2 && r >= 1) {
            inv_rows<2>(A, LD, d, r, c, h, pdc, pd);
            r -= 2;
        }
        if (r == 0) inv_rows<1>(A, LD, d, r, c, h, pdc, pd);
    }
    __syncthreads();
    // prec_chol (upper): row r, column c > r at A[c][r], pd on the diagonal
    double *pc = p.pc + (int64_t)k * d * d;
    float *epc = p.e_pc + (int64_t)k * d * d;
    for (int r = ty; r < d; r += 16)
        for (int c = tx; c < d; c += 16) {
            const double v = c < r ? 0.0 : (c == r ? pd[r] : A[c * LD + r]);
            pc[r * d + c] = v;
            epc[r * d + c] = (float)v;
        }
    // mu_k prec_chol_k (column j: rows i <= j) and log det = sum log diag(prec_chol)
    if (tid < d) {
        const int j = tid;
        double s = mus[j] * pd[j];
        for (int i = 0; i < j; ++i) s += mus[i] * A[j * LD + i];
        p.e_mp[(int64_t)k * d + j] = (float)s;
    }
    red[tid] = tid < d ? log(pd[tid]) : 0.0;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (tid < w) red[tid] += red[tid + w];
        __syncthreads();
    }
    if (tid == 0) {
        p.e_ln[k] = (float)(log(p.weights[k]) + red[0] - 0.5 * d * log(2.0 * 3.14159265358979323846));
        p.info[k] = bad;
    }
}

}  // namespace come

using namespace come;

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
    CovArgs a{x, resp, means, used > 1 ? scratch : scatter_out, V, per, d, K, 0};
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
        return launch_cov_reduce((const float *)scratch, scatter_out, n, used, (hipStream_t)stream);
    }
    // gmm_cov_async: 4 (default) = k_gmm_cov_fb3 at d = 128 / k_gmm_cov_bf3 at d = 64 (bf16 parts),
    // 5 = k_gmm_cov_bf3 at both widths, 3 = k_gmm_cov16 (fp32 16x16x4)
    const int cv = current_opts().gmm_cov_async;
    if (cv < 3 || cv > 5)
        return set_error(COME_E_INVALID, "gmm_cov_async must be 3, 4 or 5 (got %d)", cv);
    // 4 at d = 128: k_gmm_cov_fb3 (its buffer descriptors span one chunk of x and of resp: each
    // under 2 GB, else k_gmm_cov_bf3); 4 at d = 64, and 5: k_gmm_cov_bf3
    const bool fb3_fits = per * std::max(d, K) * (int64_t)sizeof(float) < (int64_t(1) << 31);
    if (mfma && cv == 4 && d == 128 && fb3_fits) {
        static bool attr5 = false;
        if (!attr5) {
            (void)hipFuncSetAttribute((const void *)k_gmm_cov_fb3<128>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr5 = true;
        }
        a.upper_only = used > 1;
        hipLaunchKernelGGL(k_gmm_cov_fb3<128>, dim3((K + CovFb3<128>::CPW - 1) / CovFb3<128>::CPW, used),
                           dim3(CovFb3<128>::THREADS), CovFb3<128>::LDS_BYTES, (hipStream_t)stream, a);
        rc = hip_error(hipGetLastError(), "k_gmm_cov_fb3 launch");
        if (rc || used == 1) return rc;
        return launch_cov_reduce_upper((const float *)scratch, scatter_out, n, used, d,
                                       (hipStream_t)stream);
    }
    if (mfma && (cv == 4 || cv == 5)) {
        static bool attr4 = false;
        if (!attr4) {
            for (void (*f)(CovArgs) : {k_gmm_cov_bf3<64>, k_gmm_cov_bf3<128>})
                (void)hipFuncSetAttribute((const void *)f,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr4 = true;
        }
        const int cpw = d == 64 ? CovBf3<64>::CPW : CovBf3<128>::CPW;
        a.upper_only = used > 1;
        hipLaunchKernelGGL(d == 64 ? k_gmm_cov_bf3<64> : k_gmm_cov_bf3<128>,
                           dim3((K + cpw - 1) / cpw, used),
                           dim3(d == 64 ? CovBf3<64>::THREADS : CovBf3<128>::THREADS),
                           d == 64 ? CovBf3<64>::LDS_BYTES : CovBf3<128>::LDS_BYTES,
                           (hipStream_t)stream, a);
        rc = hip_error(hipGetLastError(), "k_gmm_cov_bf3 launch");
        if (rc || used == 1) return rc;
        return launch_cov_reduce_upper((const float *)scratch, scatter_out, n, used, d,
                                       (hipStream_t)stream);
    }
    void (*kern)(CovArgs) = !mfma ? k_gmm_cov_valu : (d == 64 ? k_gmm_cov16<64> : k_gmm_cov16<128>);
    const int threads = !mfma ? 256 : (d == 64 ? Cov16<64>::THREADS : Cov16<128>::THREADS);
    const int cpw = !mfma ? 1 : (d == 64 ? Cov16<64>::CPW : Cov16<128>::CPW);
    hipLaunchKernelGGL(kern, dim3((K + cpw - 1) / cpw, used), dim3(threads), 0,
                       (hipStream_t)stream, a);
    rc = hip_error(hipGetLastError(), "k_gmm_cov launch");
    if (rc || used == 1) return rc;
    return launch_cov_reduce((const float *)scratch, scatter_out, n, used, (hipStream_t)stream);
}

extern "C" int come_gmm_params(const double *scatter, const double *nk, const double *means,
                               const double *weights, int K, int d, double reg_covar,
                               double *cov_out, double *prec_chol_out, float *e_prec_chol,
                               float *e_mu_prec, float *e_log_norm, int *info, void *stream) {
    if (K < 1 || d < 1 || d > 128)
        return set_error(COME_E_INVALID, "gmm_params: need K >= 1 and 1 <= d <= 128");
    if (!scatter || !nk || !means || !weights || !cov_out || !prec_chol_out || !e_prec_chol ||
        !e_mu_prec || !e_log_norm || !info)
        return set_error(COME_E_INVALID, "null pointer");
    int dev;
    int rc = ensure_init(&dev);
    if (rc) return rc;
    static bool attr = false;
    if (!attr) {
        // (the kernel's static LDS, ~3 KB, counts against the 160 KB too: ask for what d = 128
        // needs, 129 KB, not the whole of it -- a refused attribute would also leave an error
        // for the launch check below to report)
        rc = hip_error(hipFuncSetAttribute((const void *)k_gmm_params,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)(sizeof(double) * 128 * 129)),
                       "k_gmm_params attribute");
        if (rc) return rc;
        attr = true;
    }
    ParamsArgs p{scatter, nk, means, weights, K, d, reg_covar, cov_out, prec_chol_out,
                 e_prec_chol, e_mu_prec, e_log_norm, info};
    hipLaunchKernelGGL(k_gmm_params, dim3(K), dim3(256), sizeof(double) * (size_t)d * (d + 1),
                       (hipStream_t)stream, p);
    return hip_error(hipGetLastError(), "k_gmm_params launch");
}
