/*
 * come.h -- C-ABI of the MI355X-native ComE hot path (libcome.so, gfx950).
 *
 * Drop-in boundary for the reference's Cython kernel module
 * (`from utils.training_sdg_inner import train_o1, train_o2, FAST_VERSION`,
 *  /root/reference/ADSCModel/node_embeddings.py:13, context_embeddings.py:14) and for the numpy /
 * sklearn hot loops of /root/reference/ADSCModel/community_embeddings.py.
 *
 * Conventions
 *  - Every pointer named "device" is a non-owning device pointer (the caller owns the buffer, e.g.
 *    a torch tensor); tables are C-contiguous row-major fp32 [rows x d], exactly the layout the
 *    reference's numpy arrays have (pyx:410-411,457-459).
 *  - `stream` is a hipStream_t passed as void* (NULL = the default stream).  Calls are
 *    asynchronous on that stream, capture-safe (no allocation / synchronisation inside) once
 *    come_init() has run for the device, and reentrant per stream.  Launch options: each call
 *    reads ONE consistent snapshot of the process-wide options (come_set_option, mutex-guarded:
 *    a change applies to calls that start after it returns, never half of one); the *_ex entry
 *    points take per-call options instead (come_launch_opts), so concurrent callers with
 *    different options do not interfere.
 *  - Return value: 0 = ok, < 0 = error (COME_E_*); come_last_error() returns a message
 *    (thread-local).  The reference checks nothing (bounds checks off, cython_utils.py:7); this
 *    library validates shapes/arguments on the host and never reads or writes out of bounds on
 *    the device: walk entries outside [0, V) are treated as None (pyx:435-436), table draws
 *    outside [0, V) are skipped.
 *  - Row index = the reference's Vocab.index (rank of the node id, model.py:60-64).
 */
#ifndef COME_H_
#define COME_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 5 (this header): "gmm_cov_async" accepts 3 / 4 / 5.  Its default 4 now runs k_gmm_cov_fb3 at
 * d = 128 (the staging inside the MFMA wavefronts; the diagonal 32x32 tiles' cross terms taken as
 * U + U^T, so their fp32 rounding differs from ABI 4's at the same fp32-level error; off-diagonal
 * tiles are bit-identical) and k_gmm_cov_bf3 at d = 64; 5 runs ABI 4's k_gmm_cov_bf3 at both widths.
 * ABI 4: the launch options "community_async" accept 2 / 3, "gmm_cov_async" 3 / 4
 * and "gmm_resp16" 2 / 3 only -- the 32x32 fp32 fallbacks that ABI 3's values 1 / 1 / 0 selected
 * were removed (COME_E_INVALID at the call now) -- and their defaults became the bf16-part MFMA
 * kernels (3 / 4 / 3: fp32 operands as three bf16 parts, fp32-level error).
 * ABI 3: the launch option "gmm_resp_db" (the double-buffered 32x32 E-step A/B kernels) was
 * removed, "community_async" accepts 1 / 2 / 3, "gmm_cov_async" 1 / 3 / 4 and "gmm_resp16"
 * 0 / 2 / 3 (other values: COME_E_INVALID at the call); come_source_sha256 was added.
 * ABI 2: come_*_ex hot_rows == NULL in COME_MODE_HOGWILD now means "derive the
 * contended-row bitmap from the table" (ABI 1: every row cold; now COME_HOT_NONE); the launch
 * options "o2_plain_writeback" and "o2_pair_atomics" (ABI 1, ring-kernel Hogwild) were removed and
 * come_set_option rejects them; o2_kernel = 2 with COME_MODE_HOGWILD returns COME_E_INVALID. */
#define COME_ABI_VERSION 5

enum {
    COME_OK = 0,
    COME_E_INVALID = -1, /* bad argument (message in come_last_error) */
    COME_E_HIP = -2,     /* HIP runtime error */
    COME_E_UNSUPPORTED = -3
};

enum {
    COME_MODE_HOGWILD = 0,    /* one wavefront per walk/edge, all walks/edges in flight (the
                                 reference's per-walk Hogwild threads, pyx:493) */
    COME_MODE_SEQUENTIAL = 1  /* one wavefront, walks/edges in order == workers=1: the parity
                                 anchor, bit-exact with oracle/ in its WAVE64 dot order */
};

/* Flag OR-ed into `mode` of come_sgns_o2 / come_sgns_o1: `table` points to come_pack_table's
 * packed words (T still the logical number of slots) instead of the uint32 table. */
#define COME_TABLE_PACKED 0x100

/* Flag OR-ed into `mode` (COME_MODE_HOGWILD): no contended rows -- every row is updated with plain
 * stores, hot_rows ignored.  Without it a NULL hot_rows makes the library derive the bitmap. */
#define COME_HOT_NONE 0x200

/* Share of the negative table from which a row counts as contended when the library derives the
 * bitmap itself: rows holding >= max(1, floor(share * T)) slots, share = COME_DEFAULT_HOT_SHARE
 * for rows of d <= 128 and COME_DEFAULT_HOT_SHARE_WIDE for wider rows
 * (come_amd.training_sdg_inner.default_hot_share; measured in DESIGN.md §3.1: with d = 256 and
 * 10 negatives, plain stores on rows between the two shares lose enough concurrent updates on a
 * 1M-node power-law graph to move the held-out loss 1.8% below the reference's). */
#define COME_DEFAULT_HOT_SHARE 5e-6
#define COME_DEFAULT_HOT_SHARE_WIDE 8e-7

int come_abi_version(void);

/* SHA-256 (hex) of the sources the library was built from (the csrc .hip / .cpp / .h files, the Makefile
 * and this header, concatenated in name order): the Python binding refuses a library whose stamp
 * differs from the sources beside it. */
const char *come_source_sha256(void);
const char *come_last_error(void);

/* Uploads the sigmoid table (pyx:531-533) to `device`'s constant memory.  Called implicitly by the
 * first launch on a device; call it explicitly before capturing a stream into a hipGraph. */
int come_init(int device);

/* Host: the reference's EXP_TABLE (pyx:92-95,531-533), 1000 floats. Replaces the module-global
 * table built by init() (pyx:512). */
void come_exp_table(float *out1000);

/* Host: value of the reference's FAST_VERSION (pyx:549).  Always 0: the dot product is consumed
 * as float after a double-width reduction, like fast0_* (pyx:140). */
int come_fast_version(void);

/* ---- SGNS, second order (context over walks): replaces train_o2 (pyx:454-509) over a batch ----
 * node, ctx   device fp32 [V x d] (node_embedding / context_embedding), updated in place.
 * walks       device int32 [P x L] row indices; -1 (or any value outside [0,V)) = None; trailing
 *             padding with -1 is equivalent to a shorter walk.  L <= 10000 (MAX_SENTENCE_LEN,
 *             pyx:18,480).
 * seeds       device uint64 [P], walk p's initial next_random (pyx:477: 2^24*randint+randint).
 * table       device uint32 [T] negative-sampling table (model.py:97-122), values are rows.
 * negative    0..20;  window >= 0;  1 <= d <= 512.
 * The number of pair updates a batch performs is come_count_o2_pairs() of its walks.
 * COME_MODE_HOGWILD: the contended rows are derived from `table` per call (as come_sgns_o2_ex with
 * hot_rows == NULL); OR COME_HOT_NONE into `mode` to treat every row as cold.
 */
int come_sgns_o2(float *node, float *ctx, int64_t V, int d, const int32_t *walks, int64_t P,
                 int L, const uint64_t *seeds, int window, int negative, const uint32_t *table,
                 uint64_t T, float lr, float alpha, int mode, void *stream);

/* ---- Packed negative table: an exact, 16x smaller equivalent of make_table's output ----
 * packed: device, 16 * ceil(T / 64) bytes, 16-byte aligned; word w = {uint32 base = table[64w],
 * uint32 0, uint64 bits} with bit i (1..63) set iff table[64w+i] == table[64w+i-1] + 1, so
 * table[64w+i] = base + popcount(bits & (2^(i+1) - 1)).  Exact when every step inside a word is
 * 0 or 1, which make_table guarantees (model.py:107-121 advances at most one id per slot).
 * status: device int32, set to 0 if the table packed exactly, 1 if some step was not 0/1 (then
 * the packed words must not be used).  Asynchronous on `stream`. */
int come_pack_table(const uint32_t *table, uint64_t T, void *packed, int32_t *status,
                    void *stream);

/* ---- SGNS, first order (edges): replaces train_o1 (pyx:407-450) over a batch ----
 * edges       device int32 [E x 2] rows (u, v): pair (input u, positive v) then (input v,
 *             positive u), RNG state carried across both (pyx:444-448).
 * seeds       device uint64 [E], edge e's initial next_random (pyx:427). */
int come_sgns_o1(float *node, int64_t V, int d, const int32_t *edges, int64_t E,
                 const uint64_t *seeds, int negative, const uint32_t *table, uint64_t T, float lr,
                 int mode, void *stream);

/* ---- Community gradient: replaces Community2Vec.train (community_embeddings.py:61-78) ----
 * x [V x d] updated in place, `iters` times:
 *   x_i -= lr * clip((beta/K) * sum_k pi[i,k] * inv_cov[k] @ (x_i - mu[k]), -5, 5)
 * pi [V x K], mu [K x d], inv_cov [K x d x d] (all device fp32).  1 <= d <= 512 (MFMA kernels at
 * d = 64, 128; VALU forms otherwise, the d x d matrices streamed in row chunks above d = 128). */
int come_community_grad(float *x, int64_t V, int d, const float *pi, const float *mu,
                        const float *inv_cov, int K, float beta, float lr, int iters,
                        void *stream);

/* ---- GMM responsibilities: replaces GaussianMixture.predict_proba (community_embeddings.py:37)
 * for covariance_type='full'.  prec_chol [K x d x d] (precision Cholesky factors, sklearn
 * layout), mu_prec [K x d] = mu_k @ prec_chol_k, log_norm [K] = log w_k + log det(prec_chol_k)
 * - d/2 log(2 pi) (all device fp32, precomputed on the host from the fitted parameters).
 * resp_out [V x K] device fp32.  1 <= d <= 512.  K <= 64 for d <= 128 other than 64 and 128;
 * K <= 4096 for d = 64, 128 and for d > 128 (those kernels keep the per-component
 * log-probabilities in resp_out itself). */
int come_gmm_resp(const float *x, int64_t V, int d, const float *prec_chol, const float *mu_prec,
                  const float *log_norm, int K, float *resp_out, void *stream);

/* ---- GMM EM fit (replaces GaussianMixture.fit, community_embeddings.py:27; sklearn
 * BaseMixture.fit_predict / _e_step / _m_step for covariance_type='full') ----
 * E-step: come_gmm_resp plus lse_out [V] = per-row log sum_k exp(log w_k + log N(x; mu_k, S_k))
 * (the mean of lse_out is sklearn's log_prob_norm / lower bound). */
int come_gmm_estep(const float *x, int64_t V, int d, const float *prec_chol, const float *mu_prec,
                   const float *log_norm, int K, float *resp_out, float *lse_out, void *stream);

/* M-step scatter matrices: scatter_out [K x d x d] = sum_i resp[i,k] (x_i - means_k)
 * (x_i - means_k)^T (device fp32; covariance_k = scatter_k / nk_k + reg_covar I, sklearn
 * _estimate_gaussian_covariances_full).  Rows are split into `chunks` partial sums reduced in a
 * fixed order (deterministic); scratch: device fp32 [chunks x K x d x d] (unused when
 * chunks == 1).  1 <= d <= 512. */
int come_gmm_scatter(const float *x, int64_t V, int d, const float *resp, const float *means,
                     int K, int chunks, float *scratch, float *scatter_out, void *stream);

/* The rest of one M-step and the E-step parameters it implies, one workgroup per component, in
 * float64 (sklearn _estimate_gaussian_covariances_full + _compute_precision_cholesky +
 * _estimate_log_gaussian_prob's constants): cov_out [K x d x d] = scatter_k / nk_k + reg_covar I,
 * its Cholesky factor L, prec_chol_out [K x d x d] = L^-T (upper), and the E-step's fp32 inputs:
 * e_prec_chol [K x d x d] = prec_chol, e_mu_prec [K x d] = means_k prec_chol_k, e_log_norm [K] =
 * log weights_k + sum log diag(prec_chol_k) - d/2 log(2 pi).  info [K] (device int32): 0, or j + 1
 * when the j-th pivot of component k's Cholesky factorisation is not positive (sklearn raises;
 * the caller checks).  All pointers are device memory; 1 <= d <= 128. */
int come_gmm_params(const double *scatter, const double *nk, const double *means,
                    const double *weights, int K, int d, double reg_covar, double *cov_out,
                    double *prec_chol_out, float *e_prec_chol, float *e_mu_prec,
                    float *e_log_norm, int *info, void *stream);

/* ---- Random walks: the producer of train_o2's input (utils/graph_utils.py) ----
 * Graphs are CSR over node POSITIONS 0..V-1 in networkx order (see come_graph_from_edges):
 * rowptr int64 [V+1], col int32 [rowptr[V]] (neighbours in adjacency order).  `emit` (optional,
 * int32 [V]) maps a position to the value written into a walk (e.g. the node's Vocab.index row);
 * NULL writes positions.  Walk rows are [P x path_length] int32, -1 after a walk ends. */

/* Device walker, same distribution as __random_walk__ (graph_utils.py:20-46): from the current
 * node jump back to the walk's start with probability alpha, else move to a uniform neighbour;
 * a node without neighbours ends the walk.  starts: device int32 [P] positions (one walk per
 * start; build_deepwalk_corpus_iter :187-192 starts one walk at every node per pass, in shuffled
 * order).  Random stream: Philox-4x32-10 keyed by `seed`, counter (walk_offset + walk, step) --
 * independent of launch shape, not the reference's CPython stream.  rowptr/col/emit/out are
 * device pointers. */
int come_random_walks(const int64_t *rowptr, const int32_t *col, int64_t V,
                      const int32_t *starts, int64_t P, int path_length, float alpha,
                      uint64_t seed, int64_t walk_offset, const int32_t *emit, int32_t *out,
                      void *stream);

/* Host, exact: build_deepwalk_corpus_iter (graph_utils.py:187-192) with the reference's own
 * random stream.  n_streams independent CPython random.Random streams (one per walk file of
 * write_walks_to_disk :122-146); stream s writes paths_per_stream[s] passes of V walks, streams
 * concatenated in order.  states: [n_streams x 625] uint32 = random.Random.getstate()[1] (624
 * MT19937 words + position), advanced in place (setstate() them back to continue the Python
 * streams).  Streams run on up to `threads` host threads.  All pointers are host pointers. */
int come_walks_reference(const int64_t *rowptr, const int32_t *col, int64_t V, int n_streams,
                         const int32_t *paths_per_stream, uint32_t *states, int path_length,
                         double alpha, const int32_t *emit, int threads, int32_t *out);

/* Host: random.Random(seed).getstate()[1] for 0 <= seed < 2^64 (CPython init_by_array). */
int come_pyrandom_seed(uint64_t seed, uint32_t *state625);

/* Host: `count` draws from a CPython random.Random state (advanced in place): kind 0 =
 * random(), kind 1 = _randbelow(arg) (arg <= 2^32).  Test hook for the restated stream. */
int come_pyrandom_draw(uint32_t *state625, int kind, uint64_t arg, int64_t count, double *out);

/* Host: the per-walk / per-edge seeds train_o2 / train_o1 draw from the GLOBAL numpy RNG
 * (pyx:477 / pyx:427: next_random = 2^24 * randint(0, 2^24) + randint(0, 2^24), two draws per
 * call, in call order), for n consecutive calls at once.  state625 = the 624 MT19937 words and
 * the position of numpy.random.get_state() (legacy RandomState: each bounded randint below 2^32
 * consumes one 32-bit output, masked to 24 bits -- the mask equals the range, so nothing is ever
 * rejected), advanced in place (set_state() it back).  out: uint64 [n]. */
int come_np_draw_seeds(uint32_t *state625, int64_t n, uint64_t *out);

/* Host: nx.Graph().add_edges_from(edges) (graph_utils.py:60-69) in networkx order.
 * edges int64 [E x 2] node ids in file order.  Outputs (capacities 2E, 2E+1 for rowptr):
 * node_ids[V] = list(G.nodes()) (first appearance), rowptr/col = adjacency in insertion order
 * (duplicates dropped, a self-loop listed once), degree[V] = G.degree() (self-loop counts 2),
 * edge_pos [E' x 2] = G.edges() as positions, in networkx order. */
int come_graph_from_edges(const int64_t *edges, int64_t E, int64_t *node_ids, int64_t *V_out,
                          int64_t *rowptr, int32_t *col, int64_t *degree, int32_t *edge_pos,
                          int64_t *E_out);

/* ---- Text formats (host) ----
 * Integer rows (edge lists graph_utils.py:49-109, walk files :112-120/:149-154): one row per
 * line of whitespace-separated integers; '#' lines and blank lines skipped.  With rows == NULL
 * only counts (nrows_out, max_tokens_out); else fills rows [cap_rows x width], -1 padded. */
int come_read_int_rows(const char *path, int64_t *rows, int64_t cap_rows, int width,
                       int64_t *nrows_out, int *max_tokens_out);
/* Writes rows [nrows x width] one per line, space separated, each ending at its first
 * negative entry (the walk-file format of _write_walks_to_disk :117-118). */
int come_write_int_rows(const char *path, const int64_t *rows, int64_t nrows, int width,
                        int append);
/* IO_utils.save_embedding (:49-62): "<first_id + i>\t<v1> <v2> ...\n", each value exactly as
 * numpy's str(np.float32) prints it.  emb: host fp32 [V x d]. */
int come_save_embedding(const char *path, const float *emb, int64_t V, int d, int64_t first_id);
/* str(np.float32(x)) into out32 (NUL-terminated); returns its length. */
int come_format_f32(float x, char *out32);

/* ---- Multi-GPU delta exchange (come_amd.distributed.DeltaAllReduce, overlapped) ----
 * Fused elementwise passes around the all-reduce of a replicated table of n floats (device,
 * 16-byte aligned, n % 4 == 0):
 *   come_delta_begin:  D = W - S;  Down = D           (D is then all-reduced in place)
 *   come_delta_end:    S += Dsum;  W += Dsum - Down   (Dsum = the all-reduced D) */
int come_delta_begin(const float *W, const float *S, float *D, float *Down, int64_t n,
                     void *stream);
int come_delta_end(float *W, float *S, const float *Dsum, const float *Down, int64_t n,
                   void *stream);

/* Row-sparse exchange (come_amd.distributed.SparseDeltaAllReduce): only rows some rank changed.
 * W, S: device fp32 [rows x d], d % 4 == 0, 16-byte aligned.
 *   come_delta_flags:   flags[r] = 1 iff row r of W differs bitwise from S, else 0 (uint8 [rows])
 *   come_delta_gather:  D[i] = W[idx[i]] - S[idx[i]]; Down = D    (D, Down: [n x d])
 *   come_delta_scatter: S[idx[i]] += Dsum[i]; W[idx[i]] += Dsum[i] - Down[i]
 * idx: device int64 [n] row indices.  A row no rank changed contributes exactly +0 to the dense
 * exchange, so the sparse one leaves the tables bit-identical to it. */
int come_delta_flags(const float *W, const float *S, int64_t rows, int d, uint8_t *flags,
                     void *stream);
int come_delta_gather(const float *W, const float *S, const int64_t *idx, int64_t n, int d,
                      float *D, float *Down, void *stream);
int come_delta_scatter(float *W, float *S, const int64_t *idx, int64_t n, int d,
                       const float *Dsum, const float *Down, void *stream);

/* ---- Launch options ----
 * Kernel-selection and grid knobs (0 = automatic unless stated):
 *   o2_kernel           1 = direct kernel, 2 = LDS-ring kernel (sequential mode only; Hogwild
 *                       returns COME_E_INVALID), 3 = streaming kernel.  Automatic: sequential ->
 *                       ring when it fits; Hogwild -> streaming when the vocabulary has >= 32 rows
 *                       per wavefront in flight (and window <= 31), else direct
 *   o2_blocks_per_cu    O2 grid cap in workgroups per CU
 *   o2_waves_per_block  1 or 2 (automatic 2)
 *   o2_static           1 = static grid-stride walk assignment instead of the device work queue
 *   rows_per_wave / o1_rows_per_wave  Hogwild launches keep at most V / rows_per_wave
 *                       wavefronts in flight so updates stay sparse on small vocabularies
 *                       (defaults 16 / 12; 0 = no cap)
 *   max_waves           absolute cap on wavefronts in flight (0 = none)
 *   o1_blocks_per_cu    O1 grid cap in 4-wave workgroups per CU (0 = 8 for the run kernel at
 *                       d <= 128, n <= 5 -- compiled for 8 waves per SIMD there -- else 6)
 *   resident_cap        1 = also clamp grids to the workgroups the occupancy API reports resident
 *   community_async     community gradient at d = 64, 128 (16-B aligned mu / inv_cov; else the
 *                       VALU kernel): default 3 = k_community_b16 (each fp32 operand as three
 *                       bf16 parts, six exact part products per multiply-add on 16x16x32 bf16
 *                       MFMAs -- fp32-level error, tests/test_gpu_c4.py; 6.75 vs 11.5 ms at C4);
 *                       2 = k_community16 (fp32 16x16x4 MFMAs, one 16-row tile per wavefront;
 *                       11.5 ms).  Other values: COME_E_INVALID
 *   gmm_cov_async       GMM M-step scatter at d = 64, 128: default 4 = k_gmm_cov_fb3 at d = 128
 *                       (E^T E with E = sqrt(r) (x - m) carried as three bf16 parts, six exact
 *                       part products per multiply-add on 32x32x16 bf16 MFMAs -- four on the
 *                       diagonal tiles, whose cross terms are U + U^T -- the staging inside the
 *                       MFMA wavefronts; 4.6 ms at C4) and k_gmm_cov_bf3 at d = 64 (specialised
 *                       staging wavefronts); 5 = k_gmm_cov_bf3 at both widths (5.5 ms at C4);
 *                       3 = k_gmm_cov16 (fp32 16x16x4 tiles: 36 of 64 upper tiles at d = 128;
 *                       7.22 ms).  Other values: COME_E_INVALID
 *   walk_staged         default 1: LDS-staged walker output (2 = 8-step, 3 = 32-step slices);
 *                       0 = one store per lane per step (identical walks)
 *   o2_fresh_loads      direct kernel: rows read with agent-scope loads (bypass the CU's L1)
 *   o2_atomic_writeback direct kernel: every row update written as a float-atomic delta
 *   gmm_resp16          GMM E-step at d = 64, 128: default 3 = k_gmm_resp_b16 (fp32 operands
 *                       as three bf16 parts, six exact part products per multiply-add on 16x16x32
 *                       bf16 MFMAs, the row's parts formed once, 4 waves per SIMD; 4.1 ms at
 *                       C4); 2 = k_gmm_resp16t on fp32 16x16x4 MFMAs (16-wide triangular skip,
 *                       in-lane row sums, the factors' non-zero 16x16 blocks packed, whole
 *                       components double-buffered, one barrier per component; 6.95 ms); a
 *                       launch holding a lower or dense factor runs every block, in
 *                       k_gmm_resp16_full, for both.  Other values: COME_E_INVALID
 *   o1_chunk            O1: > 0 = one wavefront per chunk of that many consecutive edges, the
 *                       input row held in registers over each run of edges sharing it
 *                       (k_sgns_o1_runs); default -1 = one contiguous chunk per wavefront of the
 *                       grid (the edges in flight spread over the whole list: tier C holds in
 *                       the reference's G.edges() order, +0.23% vs 1.6% for 0); 0 = one
 *                       wavefront per edge (k_sgns_o1).  Sequential mode: one chunk, in order
 *   o2_update_count     (per call, come_sgns_o2_ex only) device uint64: += the number of target
 *                       row updates the launch applied (positive + negatives that passed the
 *                       +-6 skip, pyx:141-147) -- what the data-dependent part of the O2 HBM
 *                       traffic is counted from.  NULL = not counted. */
typedef struct come_launch_opts {
    int o2_kernel;
    int o2_blocks_per_cu;
    int o2_waves_per_block;
    int o2_static;
    int rows_per_wave;
    int o1_rows_per_wave;
    int max_waves;
    int o1_blocks_per_cu;
    int resident_cap;
    int community_async;
    int gmm_cov_async;
    int walk_staged;
    int o2_fresh_loads;
    int o2_atomic_writeback;
    int gmm_resp16;
    int o1_chunk;
    uint64_t *o2_update_count;
} come_launch_opts;

/* Fills *out with the current process-wide options (o2_update_count = NULL). */
int come_get_options(come_launch_opts *out);

/* Sets one process-wide option by field name (thread-safe; calls already inside the library
 * keep the snapshot they took). */
int come_set_option(const char *name, int value);

/* come_sgns_o2 with the contended-row bitmap and per-call options.
 * hot_rows  device uint32 [ceil(V / 32)] (come_hot_rows), or NULL: in COME_MODE_HOGWILD every
 *           update of a row whose bit is set is a float-atomic delta at the memory side (no
 *           concurrent update lost); O2 also re-reads such a row before each pair (no stale
 *           cached copy), while O1's run kernel (o1_chunk != 0) holds its input row -- hot or
 *           not -- over a run of consecutive edges sharing it and flushes the run's delta once
 *           (atomically when hot: other wavefronts' updates of the row during the run are kept,
 *           the run computes on its own copy).  The other rows are written back with plain
 *           stores.  Ignored in COME_MODE_SEQUENTIAL.
 *           NULL: the library derives the bitmap from `table` on `stream` before EVERY launch
 *           (rows holding >= COME_DEFAULT_HOT_SHARE(_WIDE) of the table: a memset of V counters and a
 *           scan of the table, ~0.1 ms at T = 1e8, into library scratch that grows
 *           stream-ordered -- the first call at a larger V allocates, so warm up before capturing
 *           a stream).  Callers that launch many small batches should compute the bitmap once
 *           (come_hot_rows) and pass it; COME_HOT_NONE in `mode` makes every row cold (on graphs
 *           with hubs that trains measurably worse than the reference's Hogwild,
 *           tests/test_gpu_tierc.py).
 * opts      per-call launch options, or NULL = the process-wide ones. */
int come_sgns_o2_ex(float *node, float *ctx, int64_t V, int d, const int32_t *walks, int64_t P,
                    int L, const uint64_t *seeds, int window, int negative,
                    const uint32_t *table, uint64_t T, float lr, float alpha, int mode,
                    const uint32_t *hot_rows, const come_launch_opts *opts, void *stream);

/* Contended rows of a negative-sampling table: counts[v] = number of slots of table[0, T) holding
 * v (device uint32 [V] scratch, overwritten) and hot_bits (device uint32 [ceil(V / 32)]) bit v set
 * iff counts[v] >= min_count.  A row's share of the table is its draw probability as a negative
 * and grows with its count (degree), i.e. with how often walks visit it.  Asynchronous. */
int come_hot_rows(const uint32_t *table, uint64_t T, int64_t V, uint64_t min_count,
                  uint32_t *counts, uint32_t *hot_bits, void *stream);
/* come_sgns_o1 with the contended-row bitmap (Hogwild: an update of a hot endpoint row is a
 * float-atomic delta; NULL = derived from the table, COME_HOT_NONE = none, as come_sgns_o2_ex)
 * and per-call options (opts may be NULL = process-wide). */
int come_sgns_o1_ex(float *node, int64_t V, int d, const int32_t *edges, int64_t E,
                    const uint64_t *seeds, int negative, const uint32_t *table, uint64_t T,
                    float lr, int mode, const uint32_t *hot_rows, const come_launch_opts *opts,
                    void *stream);

/* ---- CPU twins: the same computations on HOST memory with `threads` worker
 * threads (1..1024), in come_cpu.cpp.  Separate entry points for callers without a GPU; no GPU
 * entry point calls them (no fallback).  Same argument meaning and validation as the GPU entry
 * points above; the uint32 table only (no COME_TABLE_PACKED); pairs_out (may be NULL) receives
 * the pair updates performed.
 *  come_cpu_sgns_o2 / _o1  COME_MODE_HOGWILD: `threads` workers take jobs of 150 walks (edges) and
 *                          update the shared tables without locks, as the reference's Context2Vec /
 *                          Node2Vec worker threads (context_embeddings.py:72-102,
 *                          node_embeddings.py:58-95); COME_MODE_SEQUENTIAL: the calling thread, in
 *                          order (= workers=1), bit-identical to come_sgns_o2 / _o1 sequential
 *                          mode (the same WAVE64 dot order).
 *  come_cpu_community_grad community_embeddings.py:61-78, k_community_grad's arithmetic order.
 *  come_cpu_gmm_resp / _estep  community_embeddings.py:37 predict_proba; _estep adds lse_out. */
int come_cpu_sgns_o2(float *node, float *ctx, int64_t V, int d, const int32_t *walks, int64_t P,
                     int L, const uint64_t *seeds, int window, int negative, const uint32_t *table,
                     uint64_t T, float lr, float alpha, int mode, int threads, int64_t *pairs_out);
int come_cpu_sgns_o1(float *node, int64_t V, int d, const int32_t *edges, int64_t E,
                     const uint64_t *seeds, int negative, const uint32_t *table, uint64_t T,
                     float lr, int mode, int threads, int64_t *pairs_out);
int come_cpu_community_grad(float *x, int64_t V, int d, const float *pi, const float *mu,
                            const float *inv_cov, int K, float beta, float lr, int iters,
                            int threads);
int come_cpu_gmm_resp(const float *x, int64_t V, int d, const float *prec_chol,
                      const float *mu_prec, const float *log_norm, int K, float *resp_out,
                      int threads);
int come_cpu_gmm_estep(const float *x, int64_t V, int d, const float *prec_chol,
                       const float *mu_prec, const float *log_norm, int K, float *resp_out,
                       float *lse_out, int threads);

/* ---- Host helpers ---- */

/* Model.make_table (model.py:97-122), exact: same double accumulation, same start at node id 1,
 * same clamp.  counts_by_id[0..V] (index 0 unused), table[T] (host memory).  O(V + T). */
int come_make_table(const double *counts_by_id, int64_t V, uint32_t *table, uint64_t T,
                    double power);

/* Host: the rows of `count` consecutive negative draws from next_random = seed (pyx:133-134:
 * table[(nr >> 16) % T], then the LCG step), i.e. every row the walk's (edge's) negatives can
 * touch: a train_o2 call on a walk with p pairs draws p * negative, train_o1 2 * negative. */
int come_lcg_table_draws(uint64_t seed, int64_t count, const uint32_t *table, uint64_t T,
                         uint32_t *out);

/* Number of pair updates train_o2 performs on host walks [P x L] (-1 = None). */
int64_t come_count_o2_pairs(const int32_t *walks, int64_t P, int L, int window);

#ifdef __cplusplus
}
#endif

#endif /* COME_H_ */
