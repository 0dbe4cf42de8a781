// come_cpu.cpp -- the CPU twins of the hot-path entry points ("a CPU twin of each
// entry point, come_cpu_*(..., int threads)"), plain host C++ in libcome.so.
//
// They are separate entry points on host memory, for callers without a GPU and as the product's
// own CPU path; no GPU entry point ever calls them (there is no fallback: a GPU call without a
// usable device fails with COME_E_HIP).  Semantics follow the reference's CPU path:
//   come_cpu_sgns_o2 / _o1   train_o2 / train_o1 (utils/training_sdg_inner.pyx:407-509) driven by
//                            `threads` worker threads that take jobs of kJobItems walks (edges)
//                            and update the shared tables without locks, as Context2Vec /
//                            Node2Vec's workers do (ADSCModel/context_embeddings.py:72-102,
//                            node_embeddings.py:58-95).  COME_MODE_SEQUENTIAL (= workers=1)
//                            runs the walks in order on the calling thread.  The dot product is
//                            in the GPU kernels' WAVE64 order (lane l sums elements l, l+64, ...
//                            by an fma chain, then an xor butterfly over the 64 lanes), so the
//                            sequential mode equals come_sgns_o2's sequential mode bit for bit.
//   come_cpu_community_grad  Community2Vec.train (community_embeddings.py:61-78) in the
//                            arithmetic order of the VALU kernel k_community_grad, rows split
//                            over the threads (each row's update reads only its own row).
//   come_cpu_gmm_resp/_estep GaussianMixture.predict_proba (community_embeddings.py:37) and the
//                            E-step's per-row log-sum-exp, rows split over the threads.
// Each compute body is built twice, for AVX2+FMA and for the baseline ISA (explicit fmaf either
// way, -ffp-contract=off: identical results), and the first call picks one from the CPU.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <immintrin.h>

#include <atomic>
#include <cmath>
#include <thread>
#include <vector>

#include "../../include/come.h"

namespace come {
int set_error(int code, const char *fmt, ...);
}
using come::set_error;

namespace {

constexpr int kExpTableSize = 1000;
constexpr int kMaxSentenceLen = 10000;  // pyx:18,480
constexpr int kMaxNegative = 20, kMaxDim = 512, kMaxThreads = 1024;
constexpr uint64_t kLcgMul = 25214903917ULL, kLcgAdd = 11ULL, kLcgMask = (1ULL << 48) - 1;
constexpr int64_t kJobItems = 150;  // the reference trainers' default chunksize

const float *exp_table() {
    static const struct T {
        float v[kExpTableSize];
        T() { come_exp_table(v); }  // pyx:531-533: the library's one definition
    } t;
    return t.v;
}

bool have_fma() {
    static const bool f = [] {
        __builtin_cpu_init();
        return __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
    }();
    return f;
}

#define COME_FMA_CLONE __attribute__((target("avx2,fma")))
#define HOT inline __attribute__((always_inline))

// The GPU kernels' dot-product order (come_wave.h; oracle/come_oracle.c COME_DOT_WAVE64).
HOT float dot_wave64(const float *a, const float *b, int d) {
    float lane[64];
    for (int l = 0; l < 64; ++l) lane[l] = 0.0f;
    for (int v = 0; v < d; v += 64) {
        const int n = d - v < 64 ? d - v : 64;
        for (int l = 0; l < n; ++l) lane[l] = fmaf(a[v + l], b[v + l], lane[l]);
    }
    for (int off = 1; off <= 32; off <<= 1) {
        float t[64];
        for (int l = 0; l < 64; ++l) t[l] = lane[l] + lane[l ^ off];
        memcpy(lane, t, sizeof(t));
    }
    return lane[0];
}

// The same value with AVX2: eight 8-lane accumulators hold the 64 lanes (fma chains over d in
// steps of 64, as above), then the butterfly's reduction tree.  The xor butterfly's lane 0 is the
// pairwise tree over lanes 0..63 in index order (stage `off` adds the neighbouring groups of size
// off) and float addition is commutative, so any evaluation of that tree is bit-identical:
// hadd(A, B) forms the off=1 pairs of two accumulators, a second hadd the off=2 pairs, adding the
// 128-bit halves the off=4 groups (one sum per accumulator), and the last three stages pair the
// eight sums (0,1) (2,3) (4,5) (6,7), then (01,23) (45,67), then the two halves.
// (Out of line: an always_inline target("avx2,fma") function cannot be inlined into the generic
// template chain; the call costs nothing beside d = 128 of work.)
__attribute__((target("avx2,fma"))) float dot_wave64_avx2(
    const float *a, const float *b, int d) {
    __m256 acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = _mm256_setzero_ps();
    for (int v = 0; v < d; v += 64)
        for (int j = 0; j < 8; ++j)
            acc[j] = _mm256_fmadd_ps(_mm256_loadu_ps(a + v + 8 * j),
                                     _mm256_loadu_ps(b + v + 8 * j), acc[j]);
    const __m256 h0 = _mm256_hadd_ps(_mm256_hadd_ps(acc[0], acc[1]),
                                     _mm256_hadd_ps(acc[2], acc[3]));
    const __m256 h1 = _mm256_hadd_ps(_mm256_hadd_ps(acc[4], acc[5]),
                                     _mm256_hadd_ps(acc[6], acc[7]));
    // s0 = [S0 S1 S2 S3], s1 = [S4 S5 S6 S7]: the per-accumulator sums (stage off=4)
    const __m128 s0 = _mm_add_ps(_mm256_castps256_ps128(h0), _mm256_extractf128_ps(h0, 1));
    const __m128 s1 = _mm_add_ps(_mm256_castps256_ps128(h1), _mm256_extractf128_ps(h1, 1));
    const __m128 p = _mm_hadd_ps(s0, s1);  // [S0+S1, S2+S3, S4+S5, S6+S7]   (off=8)
    const __m128 q = _mm_hadd_ps(p, p);    // [S0..3, S4..7, ...]             (off=16)
    return _mm_cvtss_f32(_mm_add_ss(q, _mm_movehdup_ps(q)));  //              (off=32)
}

struct Sgns {
    float *in_tab, *out_tab;  // O1: the same table (pyx:444)
    int64_t V;
    int d, negative, window, L;
    const int32_t *items;     // walks [P x L] or edges [E x 2]
    const uint64_t *seeds;
    const uint32_t *table;
    uint64_t T;
    float lr, alpha;
};

// Rows not yet in cache are the cost at the benchmarked sizes (a 1M x 128 table is 512 MB, a 1e8
// table 400 MB): every row a pair touches is prefetched before the first is read.
HOT void prefetch_row(const float *row, int d) {
    for (int i = 0; i < d; i += 16) __builtin_prefetch(row + i, 1, 3);
}

// One pair (pyx:105-151 for O2, pyx:205-249 for O1: no alpha, output rows not written).  The
// negative draws depend only on nr (pyx:133-134), so they are taken first -- the table reads and
// the target rows then overlap instead of queueing behind each dot product; the update sequence
// itself is unchanged.
template <bool O2, bool Simd>
HOT uint64_t pair_update(const Sgns &a, uint32_t word_index, uint32_t word2_index, uint64_t nr,
                         float *work, const float *expt) {
    float *in = a.in_tab + (int64_t)word2_index * a.d;
    uint32_t target[kMaxNegative + 1];
    target[0] = word_index;
    for (int k = 1; k <= a.negative; ++k) {
        target[k] = a.table[(nr >> 16) % a.T];
        nr = (nr * kLcgMul + kLcgAdd) & kLcgMask;  // pyx:134
    }
    prefetch_row(in, a.d);
    for (int k = 0; k <= a.negative; ++k)
        if ((int64_t)target[k] < a.V) prefetch_row(a.out_tab + (int64_t)target[k] * a.d, a.d);
    for (int i = 0; i < a.d; ++i) work[i] = 0.0f;
    for (int k = 0; k <= a.negative; ++k) {
        float label = 1.0f;
        if (k > 0) {
            if (target[k] == word_index) continue;     // pyx:135: the draw is consumed
            if ((int64_t)target[k] >= a.V) continue;   // a table value outside [0, V): skipped
            label = 0.0f;
        }
        float *out = a.out_tab + (int64_t)target[k] * a.d;
        float f;
        if constexpr (Simd)
            f = (a.d & 63) == 0 ? dot_wave64_avx2(in, out, a.d) : dot_wave64(in, out, a.d);
        else
            f = dot_wave64(in, out, a.d);
        if (f <= -6.0f || f >= 6.0f) continue;         // pyx:141: skip, not clamp
        const float s = expt[(int)(((double)f + 6.0) * 83.0)];
        const float g = O2 ? ((label - s) * a.lr) * a.alpha : (label - s) * a.lr;
        for (int i = 0; i < a.d; ++i) work[i] = fmaf(g, out[i], work[i]);    // pyx:146
        if (O2)
            for (int i = 0; i < a.d; ++i) out[i] = fmaf(g, in[i], out[i]);   // pyx:147
    }
    for (int i = 0; i < a.d; ++i) in[i] = in[i] + work[i];                  // pyx:149
    return nr;
}

// train_o2 on walk p (pyx:479-508): fixed window, j ascending, j != i; entries outside [0, V) are
// None (pyx:435-436).  Returns its pair updates.
template <bool Simd>
HOT int64_t walk_o2(const Sgns &a, int64_t p, float *work, const float *expt) {
    const int32_t *idx = a.items + p * (int64_t)a.L;
    const int n = a.L < kMaxSentenceLen ? a.L : kMaxSentenceLen;
    auto ok = [&](int j) { return idx[j] >= 0 && (int64_t)idx[j] < a.V; };
    uint64_t nr = a.seeds[p];
    int64_t pairs = 0;
    for (int i = 0; i < n; ++i) {
        if (!ok(i)) continue;
        const int j0 = i - a.window < 0 ? 0 : i - a.window;
        const int j1 = i + a.window + 1 > n ? n : i + a.window + 1;
        for (int j = j0; j < j1; ++j) {
            if (j == i || !ok(j)) continue;
            nr = pair_update<true, Simd>(a, (uint32_t)idx[i], (uint32_t)idx[j], nr, work, expt);
            ++pairs;
        }
    }
    return pairs;
}

// train_o1 on edge e (pyx:425-450): (input u, positive v) then (input v, positive u), the RNG
// state carried across both.  An edge with an endpoint outside [0, V) is skipped.
template <bool Simd>
HOT int64_t edge_o1(const Sgns &a, int64_t e, float *work, const float *expt) {
    const int32_t u = a.items[2 * e], v = a.items[2 * e + 1];
    if (u < 0 || v < 0 || (int64_t)u >= a.V || (int64_t)v >= a.V) return 0;
    uint64_t nr = a.seeds[e];
    nr = pair_update<false, Simd>(a, (uint32_t)v, (uint32_t)u, nr, work, expt);
    pair_update<false, Simd>(a, (uint32_t)u, (uint32_t)v, nr, work, expt);
    return 2;
}

template <bool O2, bool Simd>
HOT int64_t run_items(const Sgns &a, int64_t lo, int64_t hi, float *work) {
    const float *expt = exp_table();
    int64_t pairs = 0;
    for (int64_t i = lo; i < hi; ++i)
        pairs += O2 ? walk_o2<Simd>(a, i, work, expt) : edge_o1<Simd>(a, i, work, expt);
    return pairs;
}
template <bool O2>
COME_FMA_CLONE int64_t run_items_fma(const Sgns &a, int64_t lo, int64_t hi, float *work) {
    return run_items<O2, true>(a, lo, hi, work);
}
template <bool O2>
int64_t run_items_base(const Sgns &a, int64_t lo, int64_t hi, float *work) {
    return run_items<O2, false>(a, lo, hi, work);
}

// `threads` workers claim jobs of kJobItems consecutive items from a shared counter and race on
// the tables as the reference's Hogwild threads do; sequential = the calling thread, in order.
template <bool O2>
int64_t drive(const Sgns &a, int64_t n_items, bool sequential, int threads) {
    auto body = have_fma() ? run_items_fma<O2> : run_items_base<O2>;
    if (sequential || threads <= 1 || n_items <= kJobItems) {
        std::vector<float> work(a.d);
        return body(a, 0, n_items, work.data());
    }
    std::atomic<int64_t> next(0), total(0);
    auto worker = [&] {
        std::vector<float> work(a.d);
        int64_t mine = 0;
        for (;;) {
            const int64_t lo = next.fetch_add(kJobItems);
            if (lo >= n_items) break;
            mine += body(a, lo, lo + kJobItems < n_items ? lo + kJobItems : n_items, work.data());
        }
        total += mine;
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) pool.emplace_back(worker);
    for (auto &t : pool) t.join();
    return total.load();
}

// Rows [0, V) split into `threads` contiguous blocks, fn(lo, hi) on each.
template <class F>
void parallel_rows(int64_t V, int threads, F fn) {
    if (threads <= 1 || V < 64) {
        fn((int64_t)0, V);
        return;
    }
    std::vector<std::thread> pool;
    const int64_t per = (V + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        const int64_t lo = t * per, hi = lo + per < V ? lo + per : V;
        if (lo < hi) pool.emplace_back(fn, lo, hi);
    }
    for (auto &t : pool) t.join();
}

struct Comm {
    float *x;
    const float *pi, *mu, *inv_cov;
    int64_t V;
    int d, K, iters;
    float coef, lr;
};

// k_community_grad's arithmetic per row: G[c] = fma(pi_k, sum_j (x - mu_k)[j] M_k[c][j], G[c])
// over k (the inner sum an fma chain in j), g = clip(G * coef, -5, 5), x = x - g * lr.
HOT void community_rows(const Comm &a, int64_t lo, int64_t hi) {
    std::vector<float> dx(a.d), G(a.d);
    for (int64_t r = lo; r < hi; ++r) {
        float *x = a.x + r * a.d;
        for (int it = 0; it < a.iters; ++it) {
            for (int c = 0; c < a.d; ++c) G[c] = 0.0f;
            for (int k = 0; k < a.K; ++k) {
                const float *M = a.inv_cov + (int64_t)k * a.d * a.d;
                for (int j = 0; j < a.d; ++j) dx[j] = x[j] - a.mu[(int64_t)k * a.d + j];
                const float p = a.pi[r * a.K + k];
                for (int c = 0; c < a.d; ++c) {
                    float acc = 0.0f;
                    for (int j = 0; j < a.d; ++j) acc = fmaf(dx[j], M[(int64_t)c * a.d + j], acc);
                    G[c] = fmaf(p, acc, G[c]);
                }
            }
            for (int c = 0; c < a.d; ++c) {
                float g = G[c] * a.coef;
                g = g < -5.0f ? -5.0f : (g > 5.0f ? 5.0f : g);  // clip(min=-5, max=5), :79
                x[c] = x[c] - g * a.lr;
            }
        }
    }
}
COME_FMA_CLONE void community_rows_fma(const Comm &a, int64_t lo, int64_t hi) {
    community_rows(a, lo, hi);
}
void community_rows_base(const Comm &a, int64_t lo, int64_t hi) { community_rows(a, lo, hi); }

struct Resp {
    const float *x, *prec_chol, *mu_prec, *log_norm;
    float *resp, *lse;
    int64_t V;
    int d, K;
};

// Per row: y_c = sum_j x_j P_k[j][c] - (mu_k P_k)_c, lp_k = log_norm_k - 0.5 sum_c y_c^2, then
// resp = exp(lp - logsumexp(lp)) (sklearn _estimate_weighted_log_prob + _estimate_log_prob_resp).
HOT void resp_rows(const Resp &a, int64_t lo, int64_t hi) {
    std::vector<float> lp(a.K);
    for (int64_t r = lo; r < hi; ++r) {
        const float *x = a.x + r * a.d;
        float m = -INFINITY;
        for (int k = 0; k < a.K; ++k) {
            const float *P = a.prec_chol + (int64_t)k * a.d * a.d;
            float sq = 0.0f;
            for (int c = 0; c < a.d; ++c) {
                float y = 0.0f;
                for (int j = 0; j < a.d; ++j) y = fmaf(x[j], P[(int64_t)j * a.d + c], y);
                y = y - a.mu_prec[(int64_t)k * a.d + c];
                sq = fmaf(y, y, sq);
            }
            lp[k] = a.log_norm[k] - 0.5f * sq;
            m = fmaxf(m, lp[k]);
        }
        float s = 0.0f;
        for (int k = 0; k < a.K; ++k) s += expf(lp[k] - m);
        const float lse = m + logf(s);
        for (int k = 0; k < a.K; ++k) a.resp[r * a.K + k] = expf(lp[k] - lse);
        if (a.lse) a.lse[r] = lse;
    }
}
COME_FMA_CLONE void resp_rows_fma(const Resp &a, int64_t lo, int64_t hi) { resp_rows(a, lo, hi); }
void resp_rows_base(const Resp &a, int64_t lo, int64_t hi) { resp_rows(a, lo, hi); }

int check_threads(int threads) {
    if (threads < 1 || threads > kMaxThreads)
        return set_error(COME_E_INVALID, "threads must be in [1, %d]", kMaxThreads);
    return COME_OK;
}

int check_sgns(int64_t V, int d, int negative, const uint32_t *table, uint64_t T, int mode,
               int threads) {
    if (V < 0 || d < 1 || d > kMaxDim || negative < 0 || negative > kMaxNegative)
        return set_error(COME_E_INVALID, "need V>=0, 1<=d<=%d, 0<=negative<=%d", kMaxDim,
                         kMaxNegative);
    if (negative > 0 && (!table || T == 0))
        return set_error(COME_E_INVALID, "negative sampling needs a table with T >= 1");
    if (mode & COME_TABLE_PACKED)
        return set_error(COME_E_INVALID, "CPU twins take the uint32 table (not the packed form)");
    if ((mode & 0xFF) != COME_MODE_HOGWILD && (mode & 0xFF) != COME_MODE_SEQUENTIAL)
        return set_error(COME_E_INVALID, "mode must be COME_MODE_HOGWILD or COME_MODE_SEQUENTIAL");
    return check_threads(threads);
}

}  // namespace

extern "C" int come_cpu_sgns_o2(float *node, float *ctx, int64_t V, int d, const int32_t *walks,
                                int64_t P, int L, const uint64_t *seeds, int window, int negative,
                                const uint32_t *table, uint64_t T, float lr, float alpha, int mode,
                                int threads, int64_t *pairs_out) {
    int rc = check_sgns(V, d, negative, table, T, mode, threads);
    if (rc) return rc;
    if (P < 0 || L < 0 || window < 0) return set_error(COME_E_INVALID, "need P, L, window >= 0");
    if (pairs_out) *pairs_out = 0;
    if (P == 0 || L == 0 || V == 0) return COME_OK;
    if (!node || !ctx || !walks || !seeds) return set_error(COME_E_INVALID, "null pointer");
    const Sgns a{node, ctx, V, d, negative, window, L, walks, seeds, table, T, lr, alpha};
    const int64_t pairs =
        drive<true>(a, P, (mode & 0xFF) == COME_MODE_SEQUENTIAL, threads);
    if (pairs_out) *pairs_out = pairs;
    return COME_OK;
}

extern "C" int come_cpu_sgns_o1(float *node, int64_t V, int d, const int32_t *edges, int64_t E,
                                const uint64_t *seeds, int negative, const uint32_t *table,
                                uint64_t T, float lr, int mode, int threads, int64_t *pairs_out) {
    int rc = check_sgns(V, d, negative, table, T, mode, threads);
    if (rc) return rc;
    if (E < 0) return set_error(COME_E_INVALID, "need E >= 0");
    if (pairs_out) *pairs_out = 0;
    if (E == 0 || V == 0) return COME_OK;
    if (!node || !edges || !seeds) return set_error(COME_E_INVALID, "null pointer");
    const Sgns a{node, node, V, d, negative, 0, 2, edges, seeds, table, T, lr, 0.0f};
    const int64_t pairs =
        drive<false>(a, E, (mode & 0xFF) == COME_MODE_SEQUENTIAL, threads);
    if (pairs_out) *pairs_out = pairs;
    return COME_OK;
}

extern "C" int come_cpu_community_grad(float *x, int64_t V, int d, const float *pi,
                                       const float *mu, const float *inv_cov, int K, float beta,
                                       float lr, int iters, int threads) {
    if (V < 0 || d < 1 || d > kMaxDim || K < 1 || iters < 0)
        return set_error(COME_E_INVALID, "need V>=0, 1<=d<=%d, K>=1, iters>=0", kMaxDim);
    int rc = check_threads(threads);
    if (rc) return rc;
    if (V == 0 || iters == 0) return COME_OK;
    if (!x || !pi || !mu || !inv_cov) return set_error(COME_E_INVALID, "null pointer");
    // (float)(beta / K): community_embeddings.py:77 (numpy casts the Python float to fp32)
    const Comm a{x, pi, mu, inv_cov, V, d, K, iters, (float)((double)beta / K), lr};
    auto fn = have_fma() ? community_rows_fma : community_rows_base;
    parallel_rows(V, threads, [&](int64_t lo, int64_t hi) { fn(a, lo, hi); });
    return COME_OK;
}

extern "C" int come_cpu_gmm_estep(const float *x, int64_t V, int d, const float *prec_chol,
                                  const float *mu_prec, const float *log_norm, int K,
                                  float *resp_out, float *lse_out, int threads) {
    if (V < 0 || d < 1 || d > kMaxDim || K < 1)
        return set_error(COME_E_INVALID, "need V>=0, 1<=d<=%d, K>=1", kMaxDim);
    int rc = check_threads(threads);
    if (rc) return rc;
    if (V == 0) return COME_OK;
    if (!x || !prec_chol || !mu_prec || !log_norm || !resp_out)
        return set_error(COME_E_INVALID, "null pointer");
    const Resp a{x, prec_chol, mu_prec, log_norm, resp_out, lse_out, V, d, K};
    auto fn = have_fma() ? resp_rows_fma : resp_rows_base;
    parallel_rows(V, threads, [&](int64_t lo, int64_t hi) { fn(a, lo, hi); });
    return COME_OK;
}

extern "C" int come_cpu_gmm_resp(const float *x, int64_t V, int d, const float *prec_chol,
                                 const float *mu_prec, const float *log_norm, int K,
                                 float *resp_out, int threads) {
    return come_cpu_gmm_estep(x, V, d, prec_chol, mu_prec, log_norm, K, resp_out, nullptr,
                              threads);
}
