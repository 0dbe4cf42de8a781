/*
 * come_oracle_mt.c -- multithreaded (Hogwild) CPU restatement of the reference SGNS hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library, and only as the checker / the timed CPU baseline.  The product path
 * (libcome.so) never links it.
 *
 * What it restates: the reference's Hogwild host drivers, which run `workers` threads that each
 * take a job of walks (edges), call train_o2 (train_o1) once per walk (edge), and release the GIL
 * inside it, so the threads race on the shared numpy tables with no locks:
 *   /root/reference/ADSCModel/context_embeddings.py:72-98  (worker threads, one train_o2 per walk)
 *   /root/reference/ADSCModel/node_embeddings.py:58-83      (worker threads, one train_o1 per edge)
 *   /root/reference/utils/training_sdg_inner.pyx:454-509    (train_o2, `with nogil` at :493)
 *   /root/reference/utils/training_sdg_inner.pyx:407-450    (train_o1, `with nogil` at :443)
 *   /root/reference/utils/training_sdg_inner.pyx:105-151, :205-249 (fast0_o2 / fast0_o1)
 * Same per-pair arithmetic as come_oracle.c (pair enumeration, LCG draws, skip of a draw equal to
 * the positive, +-6 skip, EXP_TABLE bucket, g formula, sequential negative updates, in += work).
 * Granularity: a thread claims a job of `chunk` consecutive walks (edges) from a shared counter --
 * the reference's job of `chunksize` items (context_embeddings.py:101-102, node_embeddings.py:
 * 94-95, default 150) -- and runs one train_o2 (train_o1) per item, so which thread runs which
 * walk, and the interleaving of their row updates, is as nondeterministic as the reference's
 * worker pool.  Plain loads and stores on the shared tables,
 * as the reference's BLAS saxpy does (races are the algorithm).
 *
 * Dot product: eight float partial sums over the row (element i goes to sum i % 8), then the
 * partials are added pairwise -- the shape of an 8-wide SIMD BLAS sdot (OpenBLAS' float kernels
 * accumulate in vector registers the same way).  The per-element fmaf updates (saxpy, pyx:146-149)
 * are vectorised.  The hot loops are compiled twice (target("avx2,fma") and the baseline ISA); the
 * first call picks one from the CPU the library runs on (oracle_mt_isa() reports which).
 *
 * Used as bench.py's cpu_baseline ("port"): timed on every CPU the process may use on the GPU box.
 * Its speed relative to the reference's own Cython train_o2 driven by Context2Vec's Python threads
 * is measured in this container by scripts/calibrate_cpu.py (profiles/r02_cpu_calibration.json).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define EXP_TABLE_SIZE 1000
#define MAX_EXP 6
#define MAX_SENTENCE_LEN 10000
#define LCG_MUL 25214903917ULL
#define LCG_ADD 11ULL
#define LCG_MASK 281474976710655ULL /* 2^48 - 1, pyx:121 */

static float MT_EXP_TABLE[EXP_TABLE_SIZE];
static pthread_once_t mt_exp_once = PTHREAD_ONCE_INIT;

/* pyx:531-533 as generated (same promotions as come_oracle.c's oracle_exp_table) */
static void mt_select(void);
static void mt_exp_init(void) {
    mt_select();
    for (int i = 0; i < EXP_TABLE_SIZE; ++i) {
        float q = (float)i / (float)EXP_TABLE_SIZE;
        float e = (float)exp(((double)q * 2.0 - 1.0) * 6.0);
        MT_EXP_TABLE[i] = (float)((double)e / ((double)e + 1.0));
    }
}

#define HOT static inline __attribute__((always_inline))

typedef float v8f __attribute__((vector_size(32)));

HOT float dot8(const float *a, const float *b, int d) {
    v8f acc = {0, 0, 0, 0, 0, 0, 0, 0};
    int i = 0;
    for (; i + 8 <= d; i += 8) {
        v8f x, y;
        memcpy(&x, a + i, sizeof(x));
        memcpy(&y, b + i, sizeof(y));
        acc = x * y + acc; /* contracted to one vfmadd231ps in the AVX2 build */
    }
    float s[8];
    memcpy(s, &acc, sizeof(s));
    for (; i < d; ++i) s[i & 7] = fmaf(a[i], b[i], s[i & 7]);
    return ((s[0] + s[4]) + (s[2] + s[6])) + ((s[1] + s[5]) + (s[3] + s[7]));
}

/* One pair (pyx:105-151 for o2 = 1, pyx:205-249 for o2 = 0). */
HOT uint64_t mt_pair(int negative, const uint32_t *table, uint64_t table_len, float *in_tab,
                     float *out_tab, int d, uint32_t word_index, uint32_t word2_index, float lr,
                     float lam, int o2, float *work, uint64_t nr, int64_t V) {
    float *in = in_tab + (int64_t)word2_index * d;
    for (int i = 0; i < d; ++i) work[i] = 0.0f;
    for (int k = 0; k <= negative; ++k) {
        uint32_t target;
        float label;
        if (k == 0) {
            target = word_index;
            label = 1.0f;
        } else {
            target = table[(nr >> 16) % table_len];
            nr = (nr * LCG_MUL + LCG_ADD) & LCG_MASK;
            if (target == word_index || (int64_t)target >= V) continue; /* pyx:135 */
            label = 0.0f;
        }
        float *out = out_tab + (int64_t)target * d;
        const float f = dot8(in, out, d);
        if (f <= -MAX_EXP || f >= MAX_EXP) continue; /* pyx:141 */
        const float s = MT_EXP_TABLE[(int)(((double)f + 6.0) * 83.0)];
        const float g = o2 ? ((label - s) * lr) * lam : (label - s) * lr;
        for (int i = 0; i < d; ++i) work[i] = fmaf(g, out[i], work[i]); /* :146 */
        if (o2)
            for (int i = 0; i < d; ++i) out[i] = fmaf(g, in[i], out[i]); /* :147 */
    }
    for (int i = 0; i < d; ++i) in[i] = in[i] + work[i]; /* :149 */
    return nr;
}

HOT int64_t walk_o2_body(
    float *node, float *ctx, int d, const int32_t *idx, int path_len, uint64_t nr, int window,
    int negative, const uint32_t *table, uint64_t T, float lr, float alpha, float *work,
    int64_t V) {
    int64_t pairs = 0;
    for (int i = 0; i < path_len; ++i) { /* pyx:494-508 */
        if (idx[i] < 0 || idx[i] >= V) continue;
        const int j0 = i - window < 0 ? 0 : i - window;
        const int j1 = i + window + 1 > path_len ? path_len : i + window + 1;
        for (int j = j0; j < j1; ++j) {
            if (j == i || idx[j] < 0 || idx[j] >= V) continue;
            nr = mt_pair(negative, table, T, node, ctx, d, (uint32_t)idx[i], (uint32_t)idx[j],
                         lr, alpha, 1, work, nr, V);
            ++pairs;
        }
    }
    return pairs;
}

HOT int64_t edge_o1_body(
    float *node, int d, int32_t u, int32_t v, uint64_t nr, int negative, const uint32_t *table,
    uint64_t T, float lr, float *work, int64_t V) {
    nr = mt_pair(negative, table, T, node, node, d, (uint32_t)v, (uint32_t)u, lr, 0.0f, 0, work,
                 nr, V); /* pyx:444 */
    nr = mt_pair(negative, table, T, node, node, d, (uint32_t)u, (uint32_t)v, lr, 0.0f, 0, work,
                 nr, V); /* pyx:447 */
    return 2;
}

/* Each body is compiled twice: an AVX2 + FMA build (fmaf becomes vfmadd, the row loops 8-wide)
 * and a baseline build; mt_select() picks one from the CPU the library runs on. */
#define WALK_ARGS                                                                                 \
    float *node, float *ctx, int d, const int32_t *idx, int path_len, uint64_t nr, int window,  \
        int negative, const uint32_t *table, uint64_t T, float lr, float alpha, float *work,    \
        int64_t V
#define WALK_PASS node, ctx, d, idx, path_len, nr, window, negative, table, T, lr, alpha, work, V
#define EDGE_ARGS                                                                                 \
    float *node, int d, int32_t u, int32_t v, uint64_t nr, int negative, const uint32_t *table, \
        uint64_t T, float lr, float *work, int64_t V
#define EDGE_PASS node, d, u, v, nr, negative, table, T, lr, work, V
__attribute__((target("avx2,fma"))) static int64_t mt_walk_o2_avx2(WALK_ARGS) {
    return walk_o2_body(WALK_PASS);
}
static int64_t mt_walk_o2_base(WALK_ARGS) { return walk_o2_body(WALK_PASS); }
__attribute__((target("avx2,fma"))) static int64_t mt_edge_o1_avx2(EDGE_ARGS) {
    return edge_o1_body(EDGE_PASS);
}
static int64_t mt_edge_o1_base(EDGE_ARGS) { return edge_o1_body(EDGE_PASS); }

static int64_t (*mt_walk_o2)(WALK_ARGS) = mt_walk_o2_base;
static int64_t (*mt_edge_o1)(EDGE_ARGS) = mt_edge_o1_base;

static void mt_select(void) {
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) {
        mt_walk_o2 = mt_walk_o2_avx2;
        mt_edge_o1 = mt_edge_o1_avx2;
    }
}

/* 1 when the AVX2 + FMA build is in use (reported with the baseline). */
int oracle_mt_isa(void);

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

typedef struct {
    int o2;
    float *node, *ctx;
    int64_t V;
    int d;
    const int32_t *items; /* walks [P x L] or edges [E x 2] */
    int64_t count;
    int L;
    const uint64_t *seeds;
    int window, negative;
    const uint32_t *table;
    uint64_t T;
    float lr, alpha;
    double deadline; /* 0 = none */
    int64_t chunk;   /* items per claim (the reference's chunksize) */
    int64_t next;    /* shared claim counter (the reference's job queue) */
    int64_t pairs, done;
} MtJob;

static void *mt_worker(void *arg) {
    MtJob *j = (MtJob *)arg;
    float *work = (float *)malloc(sizeof(float) * (size_t)j->d); /* per-worker py_work */
    int64_t pairs = 0, done = 0;
    const int path_len = j->L < MAX_SENTENCE_LEN ? j->L : MAX_SENTENCE_LEN; /* pyx:480 */
    for (;;) {
        if (j->deadline > 0.0 && now_s() > j->deadline) break;
        const int64_t p0 = __atomic_fetch_add(&j->next, j->chunk, __ATOMIC_RELAXED);
        if (p0 >= j->count) break;
        const int64_t p1 = p0 + j->chunk < j->count ? p0 + j->chunk : j->count;
        for (int64_t p = p0; p < p1; ++p) {
            if (j->o2) {
                pairs += mt_walk_o2(j->node, j->ctx, j->d, j->items + p * (int64_t)j->L,
                                    path_len, j->seeds[p], j->window, j->negative, j->table, j->T,
                                    j->lr, j->alpha, work, j->V);
            } else {
                const int32_t u = j->items[2 * p], v = j->items[2 * p + 1];
                if (u >= 0 && v >= 0 && u < j->V && v < j->V)
                    pairs += mt_edge_o1(j->node, j->d, u, v, j->seeds[p], j->negative, j->table,
                                        j->T, j->lr, work, j->V);
            }
            ++done;
        }
    }
    free(work);
    __atomic_fetch_add(&j->pairs, pairs, __ATOMIC_RELAXED);
    __atomic_fetch_add(&j->done, done, __ATOMIC_RELAXED);
    return NULL;
}

static int64_t mt_run(MtJob *j, int threads, int64_t *done_out) {
    pthread_once(&mt_exp_once, mt_exp_init);
    if (threads < 1) threads = 1;
    pthread_t *ts = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    int started = 0;
    for (int t = 0; t < threads; ++t)
        if (pthread_create(&ts[t], NULL, mt_worker, j) == 0) ++started;
    if (started == 0) mt_worker(j); /* could not start a thread: run on the caller */
    for (int t = 0; t < started; ++t) pthread_join(ts[t], NULL);
    free(ts);
    if (done_out) *done_out = j->done;
    return j->pairs;
}

/* Hogwild train_o2 over walks [P x L] (-1 = None) on `threads` threads, `chunk` walks per claim.
 * max_seconds > 0 stops claiming new jobs after that long (jobs already claimed finish).  Returns the pair updates
 * performed; *walks_done = walks processed. */
int64_t oracle_sgns_o2_hogwild(float *node, float *ctx, int64_t V, int d, const int32_t *walks,
                               int64_t P, int L, const uint64_t *seeds, int window, int negative,
                               const uint32_t *table, uint64_t T, float lr, float alpha,
                               int threads, double max_seconds, int64_t chunk,
                               int64_t *walks_done) {
    MtJob j = {1,  node,   ctx,      V,     d,           walks, P, L, seeds, window, negative, table,
               T,  lr,     alpha,    0.0,   chunk > 0 ? chunk : 1, 0, 0, 0};
    if (max_seconds > 0.0) j.deadline = now_s() + max_seconds;
    return mt_run(&j, threads, walks_done);
}

/* Hogwild train_o1 over edges [E x 2] on `threads` threads (same contract as above). */
int64_t oracle_sgns_o1_hogwild(float *node, int64_t V, int d, const int32_t *edges, int64_t E,
                               const uint64_t *seeds, int negative, const uint32_t *table,
                               uint64_t T, float lr, int threads, double max_seconds, int64_t chunk,
                               int64_t *edges_done) {
    MtJob j = {0, node, NULL, V, d,   edges, E, 2, seeds, 0, negative, table, T, lr, 1.0f, 0.0,
               chunk > 0 ? chunk : 1, 0,    0, 0};
    if (max_seconds > 0.0) j.deadline = now_s() + max_seconds;
    return mt_run(&j, threads, edges_done);
}

int oracle_mt_isa(void) {
    pthread_once(&mt_exp_once, mt_exp_init);
    return mt_walk_o2 == mt_walk_o2_avx2;
}
