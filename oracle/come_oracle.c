/*
 * come_oracle.c -- CPU restatement of the reference SGNS hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library, and only as the checker.  The product path (libcome.so) never links it.
 *
 * It restates, sequentially and single-threaded, what the reference computes in
 *   /root/reference/utils/training_sdg_inner.pyx   (Cython; the generated C was inspected to pin
 *                                                   the exact float/double promotions noted below)
 *   /root/reference/ADSCModel/model.py:97-122      (make_table)
 * Parity of this file is pinned against golden vectors produced by the reference itself
 * (tests/golden/make_golden.py imports the Cython module built by oracle/build_ref.py).
 *
 * Two dot-product orders are offered (argument `dot_mode`):
 *   COME_DOT_REF    (0): double-accumulated sequential dot cast to float -- closest to what the
 *                        reference's BLAS sdot returns (pyx:140 casts the dsdot result to float).
 *                        Differs from OpenBLAS' own summation order by ~1 ulp, which is why the
 *                        reference comparison is tolerance-based (SURVEY.md §8c tiers A/B).
 *   COME_DOT_WAVE64 (1): the exact summation tree of the HIP kernel (lane l holds elements
 *                        l, l+64, ..., accumulated by an fmaf chain in that order, then an xor
 *                        butterfly over offsets 1,2,4,8,16,32).  With this order the GPU sequential mode must
 *                        agree with this oracle BIT FOR BIT.
 * Build: see oracle/Makefile (-O2 -ffp-contract=off, no fast-math: every fmaf below is explicit).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EXP_TABLE_SIZE 1000
#define MAX_EXP 6
#define MAX_SENTENCE_LEN 10000
#define LCG_MUL 25214903917ULL
#define LCG_ADD 11ULL
#define LCG_MASK 281474976710655ULL /* 2^48 - 1, pyx:121 */

enum { COME_DOT_REF = 0, COME_DOT_WAVE64 = 1 };

static float EXP_TABLE[EXP_TABLE_SIZE];
static int exp_table_ready = 0;

/* Smallest distance, over every dot product evaluated since the last reset, of (f+6)*83 to an
 * integer bucket edge or of |f| to the +-6 skip edge.  Fixture generators use it to flag cases
 * whose result could flip with a 1-ulp change of a dot product (SURVEY.md §8c tier A). */
static double g_min_margin = 1e30;
void oracle_reset_margin(void) { g_min_margin = 1e30; }
/* Target-row updates applied since the last reset (targets that passed the +-6 skip): the
 * quantity the GPU kernels count into come_launch_opts.o2_update_count. */
static int64_t g_updates = 0;
void oracle_reset_updates(void) { g_updates = 0; }
int64_t oracle_updates(void) { return g_updates; }
double oracle_min_margin(void) { return g_min_margin; }
static inline void note_margin(float f) {
    double x = ((double)f + 6.0) * 83.0;
    double m = fabs(x - floor(x + 0.5));
    double m6 = fabs(fabs((double)f) - 6.0) * 83.0;
    if (m6 < m) m = m6;
    if (m < g_min_margin) g_min_margin = m;
}

/* pyx:531-533 as generated: exp(((i/(float)1000)*2.0 - 1.0)*6.0) in double, stored as float, then
 * e/(e+1.0) in double stored as float. */
void oracle_exp_table(float *out) {
    for (int i = 0; i < EXP_TABLE_SIZE; ++i) {
        float q = (float)i / (float)EXP_TABLE_SIZE;
        float e = (float)exp(((double)q * 2.0 - 1.0) * 6.0);
        EXP_TABLE[i] = (float)((double)e / ((double)e + 1.0));
    }
    exp_table_ready = 1;
    if (out) memcpy(out, EXP_TABLE, sizeof(EXP_TABLE));
}

/* pyx:134: next_random = (next_random * 25214903917 + 11) & (2^48-1) */
uint64_t oracle_lcg_next(uint64_t s) { return (s * LCG_MUL + LCG_ADD) & LCG_MASK; }

#define HOT static inline __attribute__((always_inline))

HOT float dot_ref(const float *a, const float *b, int d) {
    double s = 0.0;
    for (int i = 0; i < d; ++i) s += (double)a[i] * (double)b[i];
    return (float)s;
}

HOT float dot_wave64(const float *a, const float *b, int d) {
    float lane[64];
    int vec = (d + 63) / 64;
    for (int l = 0; l < 64; ++l) {
        float p = 0.0f;
        for (int v = 0; v < vec; ++v) {
            int e = l + 64 * v;
            if (e < d) p = fmaf(a[e], b[e], p);
        }
        lane[l] = p;
    }
    for (int off = 1; off <= 32; off <<= 1) {
        float t[64];
        for (int l = 0; l < 64; ++l) t[l] = lane[l] + lane[l ^ off];
        memcpy(lane, t, sizeof(t));
    }
    return lane[0];
}

HOT float dotp(const float *a, const float *b, int d, int mode) {
    return mode == COME_DOT_WAVE64 ? dot_wave64(a, b, d) : dot_ref(a, b, d);
}

/* One pair, pyx:105-151 (o2=1, fast0_o2/fast1_o2) or pyx:205-296 (o2=0, fast0_o1/fast1_o1).
 * in_tab/out_tab are the input and output tables (the same pointer for O1, pyx:444). */
HOT uint64_t pair_update(int negative, const uint32_t *table, uint64_t table_len,
                            float *in_tab, float *out_tab, int size, uint32_t word_index,
                            uint32_t word2_index, float lr, float lam, int o2, float *work,
                            uint64_t next_random, int dot_mode) {
    float *in = in_tab + (int64_t)word2_index * size;
    memset(work, 0, sizeof(float) * size);
    for (int d = 0; d <= negative; ++d) {
        uint32_t target;
        float label;
        if (d == 0) {
            target = word_index;
            label = 1.0f;
        } else {
            target = table[(next_random >> 16) % table_len];
            next_random = oracle_lcg_next(next_random);
            if (target == word_index) continue; /* pyx:135: draw consumed, target skipped */
            label = 0.0f;
        }
        float *out = out_tab + (int64_t)target * size;
        float f = dotp(in, out, size, dot_mode);
        note_margin(f);
        if (f <= -MAX_EXP || f >= MAX_EXP) continue; /* pyx:141: skip, not clamp */
        /* pyx:143 as generated: EXP_TABLE[(int)((f + 6.0) * 83.0)] in double */
        float s = EXP_TABLE[(int)(((double)f + 6.0) * 83.0)];
        ++g_updates;
        float g = o2 ? ((label - s) * lr) * lam : (label - s) * lr; /* pyx:144 / :243 */
        for (int i = 0; i < size; ++i) work[i] = fmaf(g, out[i], work[i]);      /* :146 */
        if (o2)
            for (int i = 0; i < size; ++i) out[i] = fmaf(g, in[i], out[i]);    /* :147 */
    }
    for (int i = 0; i < size; ++i) in[i] = in[i] + work[i]; /* :149 saxpy(1.0) */
    return next_random;
}

/* train_o2 (pyx:454-509) over P walks in order.  walks: [P x L] int32 row indices, -1 = None
 * (codelens 0; trailing -1 padding is equivalent to a shorter path).  seeds: per-walk next_random
 * (pyx:477).  Returns the number of pair updates (fast_o2 calls). */
HOT int64_t sgns_o2_body(float *node, float *ctx, int d, const int32_t *walks, int64_t P, int L,
                         const uint64_t *seeds, int window, int negative, const uint32_t *table,
                         uint64_t table_len, float lr, float alpha, int dot_mode, float *work) {
    int64_t pairs = 0;
    int path_len = L < MAX_SENTENCE_LEN ? L : MAX_SENTENCE_LEN;
    for (int64_t p = 0; p < P; ++p) {
        const int32_t *idx = walks + p * (int64_t)L;
        uint64_t nr = seeds[p];
        for (int i = 0; i < path_len; ++i) {
            if (idx[i] < 0) continue;
            int j0 = i - window < 0 ? 0 : i - window;
            int k = i + window + 1 > path_len ? path_len : i + window + 1;
            for (int j = j0; j < k; ++j) {
                if (j == i || idx[j] < 0) continue;
                /* pyx:507: fast_o2(word_index=indexes[i], word2_index=indexes[j]) */
                nr = pair_update(negative, table, table_len, node, ctx, d, (uint32_t)idx[i],
                                 (uint32_t)idx[j], lr, alpha, 1, work, nr, dot_mode);
                ++pairs;
            }
        }
    }
    return pairs;
}

/* train_o1 (pyx:407-450) over E edges in order.  edges: [E x 2] int32 rows; seeds per edge
 * (pyx:427).  Pair 1: input edge[0], positive edge[1] (pyx:444); pair 2: input edge[1],
 * positive edge[0] (pyx:447), RNG state carried across both.  Edges with a negative endpoint are
 * skipped (the reference reads uninitialised indexes there: undefined behaviour).  Returns the
 * number of pair updates. */
HOT int64_t sgns_o1_body(float *node, int d, const int32_t *edges, int64_t E,
                         const uint64_t *seeds, int negative, const uint32_t *table,
                         uint64_t table_len, float lr, int dot_mode, float *work) {
    int64_t pairs = 0;
    for (int64_t e = 0; e < E; ++e) {
        int32_t u = edges[2 * e], v = edges[2 * e + 1];
        if (u < 0 || v < 0) continue;
        uint64_t nr = seeds[e];
        nr = pair_update(negative, table, table_len, node, node, d, (uint32_t)v, (uint32_t)u, lr,
                         0.0f, 0, work, nr, dot_mode);
        nr = pair_update(negative, table, table_len, node, node, d, (uint32_t)u, (uint32_t)v, lr,
                         0.0f, 0, work, nr, dot_mode);
        pairs += 2;
    }
    return pairs;
}

/* Each body is built twice: with AVX2 + FMA enabled (explicit fmaf() becomes one vfmadd instead
 * of a libm call -- the same correctly rounded result, only faster) and for the baseline ISA;
 * the first call picks one from the CPU.  No reassociation either way (-ffp-contract=off, no
 * fast-math), so results are identical across the two builds. */
#define O2_ARGS                                                                                   \
    float *node, float *ctx, int d, const int32_t *walks, int64_t P, int L, const uint64_t *seeds, \
        int window, int negative, const uint32_t *table, uint64_t table_len, float lr,           \
        float alpha, int dot_mode, float *work
#define O2_PASS \
    node, ctx, d, walks, P, L, seeds, window, negative, table, table_len, lr, alpha, dot_mode, work
#define O1_ARGS                                                                                   \
    float *node, int d, const int32_t *edges, int64_t E, const uint64_t *seeds, int negative,    \
        const uint32_t *table, uint64_t table_len, float lr, int dot_mode, float *work
#define O1_PASS node, d, edges, E, seeds, negative, table, table_len, lr, dot_mode, work
__attribute__((target("avx2,fma"))) static int64_t sgns_o2_fma(O2_ARGS) {
    return sgns_o2_body(O2_PASS);
}
static int64_t sgns_o2_base(O2_ARGS) { return sgns_o2_body(O2_PASS); }
__attribute__((target("avx2,fma"))) static int64_t sgns_o1_fma(O1_ARGS) {
    return sgns_o1_body(O1_PASS);
}
static int64_t sgns_o1_base(O1_ARGS) { return sgns_o1_body(O1_PASS); }
static int use_fma = -1;
static int have_fma(void) {
    if (use_fma < 0) {
        __builtin_cpu_init();
        use_fma = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
    }
    return use_fma;
}

int64_t oracle_sgns_o2(float *node, float *ctx, int d, const int32_t *walks, int64_t P, int L,
                       const uint64_t *seeds, int window, int negative, const uint32_t *table,
                       uint64_t table_len, float lr, float alpha, int dot_mode) {
    if (!exp_table_ready) oracle_exp_table(NULL);
    float *work = (float *)malloc(sizeof(float) * (size_t)d);
    int64_t pairs = (have_fma() ? sgns_o2_fma : sgns_o2_base)(O2_PASS);
    free(work);
    return pairs;
}

int64_t oracle_sgns_o1(float *node, int d, const int32_t *edges, int64_t E,
                       const uint64_t *seeds, int negative, const uint32_t *table,
                       uint64_t table_len, float lr, int dot_mode) {
    if (!exp_table_ready) oracle_exp_table(NULL);
    float *work = (float *)malloc(sizeof(float) * (size_t)d);
    int64_t pairs = (have_fma() ? sgns_o1_fma : sgns_o1_base)(O1_PASS);
    free(work);
    return pairs;
}

/* Model.make_table (model.py:97-122), literal slot-by-slot restatement.
 * counts: indexed by NODE ID, length V+1 (counts[0] unused; ids are 1..V, model.py:66).
 * Z is summed in ascending id order (dict order of build_vocab_, model.py:60-64). */
void oracle_make_table(const double *counts, int64_t V, uint32_t *table, uint64_t T,
                       double power) {
    double z = 0.0;
    for (int64_t id = 1; id <= V; ++id) z += pow(counts[id], power);
    int64_t widx = 1;
    double d1 = pow(counts[widx], power) / z;
    for (uint64_t t = 0; t < T; ++t) {
        table[t] = (uint32_t)widx;
        if (1.0 * (double)t / (double)T > d1) {
            widx += 1;
            d1 += pow(counts[widx], power) / z;
        }
        if (widx >= V) widx = V - 1;
    }
}
