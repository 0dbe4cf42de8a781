// come_sgns_impl.h -- skip-gram negative-sampling updates for gfx950 (MI355X, CDNA4).
//
// Replaces the reference's Cython hot loop, /root/reference/utils/training_sdg_inner.pyx:
//   fast0_o2/fast1_o2 (pyx:105-201) + train_o2 (pyx:454-509)   -> k_sgns_o2
//   fast0_o1/fast1_o1 (pyx:205-296) + train_o1 (pyx:407-450)   -> k_sgns_o1
//
// Execution model:
//  * One 64-lane wavefront owns one walk (O2) or one edge (O1) and processes its positive pairs in
//    the reference's order, one pair at a time -- exactly the work one reference thread does per
//    nogil call (pyx:493).  All walks/edges of a batch are in flight at once (Hogwild across
//    wavefronts, as the reference's worker threads are Hogwild across walks).
//  * A d-dim fp32 row is spread over the wave: lane l holds elements l, l+64, ... (VEC =
//    ceil(d/64) of them); every row access is VEC wave instructions of 256 contiguous bytes.
//  * The (1 + negative) target rows of a pair are gathered together, their dot products reduced
//    with interleaved xor butterflies, then resolved in reference order (a negative that repeats an
//    earlier target sees that target's updated row, pyx:147, via register forwarding).
//  * Negatives never touch the host: lane k of the wave computes LCG draw (base + k) by jump-ahead
//    (the LCG is affine mod 2^48, pyx:134) and gathers table[(s >> 16) % T] for 64 draws at once;
//    each pair then reads its n draws with v_readlane (wave-uniform, scalar registers).
//  * Dot product order is fixed: per-lane fmaf chain, then xor butterfly 1,2,4,8,16,32.  The CPU
//    oracle's WAVE64 mode restates this order, so COME_MODE_SEQUENTIAL is bit-exact with it.
//  * Compiled with -ffp-contract=off: every fused multiply-add is an explicit fmaf, matching the
//    reference's saxpy (pyx:146-149) element for element.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "come_internal.h"
#include "come_wave.h"

namespace come {

// One copy per translation unit (each .hip file is its own code object); come_init uploads the
// table into every copy (upload_exp_table_vec*).
static __constant__ float c_exp_table[kExpTableSize];

struct LcgLane {  // this lane's jump-ahead (A^k, C_k): s_{b+k} = A^k s_b + C_k  (mod 2^48)
    uint64_t a, c;
};

__device__ inline LcgLane lcg_lane_constants(int k) {
    uint64_t a = 1, c = 0;
    for (int i = 0; i < k; ++i) {
        a = (a * kLcgMul) & kLcgMask;
        c = (c * kLcgMul + kLcgAdd) & kLcgMask;
    }
    return {a, c};
}

__device__ inline uint64_t lcg_next(uint64_t s) { return (s * kLcgMul + kLcgAdd) & kLcgMask; }

// The 64 lanes' jump-ahead constants as a table in constant memory: a kernel short of registers
// reads its lane's pair when it refills a batch of draws (every 64 draws) instead of holding
// four VGPRs for the whole kernel.
struct LcgTable {
    uint64_t a[64], c[64];
};
constexpr LcgTable make_lcg_table() {
    LcgTable t{};
    uint64_t a = 1, c = 0;
    for (int k = 0; k < 64; ++k) {
        t.a[k] = a;
        t.c[k] = c;
        a = (a * kLcgMul) & kLcgMask;
        c = (c * kLcgMul + kLcgAdd) & kLcgMask;
    }
    return t;
}
static __constant__ LcgTable c_lcg = make_lcg_table();
constexpr LcgTable kLcgHost = make_lcg_table();
// state 64 draws after s, for any lane: A^64 s + C_64 (wave-uniform, scalar)
constexpr uint64_t kLcgA64 = (kLcgHost.a[63] * kLcgMul) & kLcgMask;
constexpr uint64_t kLcgC64 = (kLcgHost.c[63] * kLcgMul + kLcgAdd) & kLcgMask;

struct LcgFromTable {  // same interface as LcgLane, constants read at use
    int lane;
};
__device__ inline uint64_t lcg_state_of(uint64_t base, const LcgLane &lc) {
    return (lc.a * base + lc.c) & kLcgMask;
}
__device__ inline uint64_t lcg_state_of(uint64_t base, const LcgFromTable &lt) {
    return (c_lcg.a[lt.lane] * base + c_lcg.c[lt.lane]) & kLcgMask;
}

__device__ inline uint32_t table_slot(uint64_t s, uint64_t m, uint32_t d) {
    const uint32_t x = (uint32_t)(s >> 16);  // < 2^32 because s < 2^48 (pyx:133)
    if (d == 0) return x;                     // T >= 2^32: x % T == x
    return (uint32_t)__umul64hi(m * (uint64_t)x, (uint64_t)d);
}

// Packed negative table (come_pack_table): word w = {base, unused, bits} covers slots
// [64w, 64w + 64); table[64w + i] = base + popcount(bits & ((2 << i) - 1)), bit i (i >= 1) set iff
// slot i holds one more than slot i - 1.  Exact for every table whose values step by 0 or 1
// inside each 64-slot word -- make_table's are (model.py:107-121 advances widx by at most one per
// slot).  One 16-B load per draw from a T/4-byte structure (25 MB at T = 1e8, Infinity-Cache
// resident) instead of a 4-B load from the 400 MB table.
struct PackedWord {
    uint32_t base;
    uint32_t unused;
    uint64_t bits;
};

template <class Args>
__device__ inline uint32_t table_value(const Args &a, uint32_t slot) {
    if (a.packed) {
        const uint4 w = reinterpret_cast<const uint4 *>(a.table)[slot >> 6];
        const uint64_t bits = ((uint64_t)w.w << 32) | w.z;
        const uint64_t mask = (2ull << (slot & 63)) - 1ull;  // slot & 63 == 63: all ones
        return w.x + (uint32_t)__popcll(bits & mask);
    }
    return a.table[slot];
}

__device__ inline int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ inline float uniformf(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ inline uint64_t uniform64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ inline uint32_t readlane_u32(uint32_t v, int lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ inline uint64_t readlane_u64(uint64_t v, int lane) {
    const uint32_t lo = readlane_u32((uint32_t)v, lane);
    const uint32_t hi = readlane_u32((uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

// ---- row <-> registers -------------------------------------------------------------------------
template <int VEC, bool FULL>
struct Row {
    float v[VEC];  // lane l holds elements l, l + 64, ..., l + 64 (VEC - 1)

    // Every wave instruction touches 256 contiguous bytes (two 128-B lines): full-rate loads,
    // stores and -- what fixes this layout -- full-rate float atomics (MI355X_MICROARCH.md
    // "Global float atomics": 256 contiguous bytes per wave instruction).
    __device__ inline void load(const float *__restrict__ row, int lane, int d) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            const int e = lane + 64 * i;
            v[i] = (FULL || e < d) ? row[e] : 0.0f;
        }
    }

    // Non-temporal loads (global_load ... nt): rows with little reuse, so the L2 / Infinity Cache
    // keep the small structures every wavefront reads (hot bitmap, packed negative table)
    __device__ inline void load_nt(const float *__restrict__ row, int lane, int d) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            const int e = lane + 64 * i;
            v[i] = (FULL || e < d) ? __builtin_nontemporal_load(row + e) : 0.0f;
        }
    }

    // Agent-scope relaxed loads (global_load ... sc1): bypass this CU's L1, which other CUs'
    // stores never refresh (MI355X_MICROARCH.md: inter-workgroup visibility), so a row several
    // wavefronts update is read as last written to L2 / memory.
    __device__ inline void load_fresh(const float *__restrict__ row, int lane, int d) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            const int e = lane + 64 * i;
            v[i] = (FULL || e < d) ? __hip_atomic_load(row + e, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)
                                   : 0.0f;
        }
    }

    __device__ inline void load_as(const float *__restrict__ row, int lane, int d, bool fresh) {
        if (fresh) load_fresh(row, lane, d);
        else load(row, lane, d);
    }

    __device__ inline void store(float *__restrict__ row, int lane, int d) const {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            const int e = lane + 64 * i;
            if (FULL || e < d) row[e] = v[i];
        }
    }

    // row += v with no-return float atomics (Hogwild write-back: no update is lost)
    __device__ inline void atomic_add(float *__restrict__ row, int lane, int d) const {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            const int e = lane + 64 * i;
            if (FULL || e < d) atomicAdd(row + e, v[i]);
        }
    }
};

template <int VEC, bool FULL>
__device__ inline float lane_partial(const Row<VEC, FULL> &a, const Row<VEC, FULL> &b) {
    float p = 0.0f;
#pragma unroll
    for (int i = 0; i < VEC; ++i) p = __builtin_fmaf(a.v[i], b.v[i], p);
    return p;
}

__device__ inline float wave_sum(float p) {
    p = reduce_stage<0>(p);
    p = reduce_stage<1>(p);
    p = reduce_stage<2>(p);
    p = reduce_stage<3>(p);
    p = reduce_stage<4>(p);
    return reduce_stage<5>(p);
}

// Sum the first `count` of `part[]` across the wave, the six stages interleaved over the targets
// so their latencies overlap.
template <int N>
__device__ inline void wave_sum_n(float (&part)[N], int count) {
#define COME_STAGE(S)                                          \
    _Pragma("unroll") for (int k = 0; k < N; ++k) if (k < count) part[k] = reduce_stage<S>(part[k]);
    COME_STAGE(0) COME_STAGE(1) COME_STAGE(2) COME_STAGE(3) COME_STAGE(4) COME_STAGE(5)
#undef COME_STAGE
}

// sigma lookup exactly as generated from pyx:141-143: skip if f <= -6 or f >= 6, else
// EXP_TABLE[(int)(((double)f + 6.0) * 83.0)].  Returns false for a skipped target.
__device__ inline bool sigmoid_ref(float f, float *sig) {
    if (f <= -(float)kMaxExp || f >= (float)kMaxExp) return false;
    const int b = (int)(((double)f + 6.0) * 83.0);
    *sig = c_exp_table[b];
    return true;
}

// ---- batch of 64 negative draws held one per lane ------------------------------------------
struct DrawBatch {
    uint32_t target;  // this lane's table value for draw (base + lane)
    uint64_t base;    // LCG state of draw `base`'s index 0 (wave-uniform)
    int used;         // draws of the batch already consumed (wave-uniform)
};

// Lanes < count gather their draw's table value (the others hold 0 and must not be consumed).
template <class Args>
__device__ inline void draws_fill(DrawBatch &b, uint64_t state0, const LcgLane &lc,
                                  const Args &a, int count = 64) {
    b.base = state0;
    b.used = 0;
    b.target = 0;
    if ((int)(threadIdx.x & 63) < count) {
        const uint64_t s = (lc.a * state0 + lc.c) & kLcgMask;
        b.target = table_value(a, table_slot(s, a.fm.m, a.fm.d));
    }
}

// State of the draw `b.used` positions after the batch base (0 < used <= 64).
__device__ inline uint64_t draws_state_at_used(const DrawBatch &b, const LcgLane &lc) {
    const uint64_t s = (lc.a * b.base + lc.c) & kLcgMask;  // this lane's state
    if (b.used < 64) return uniform64(readlane_u64(s, b.used));
    return lcg_next(uniform64(readlane_u64(s, 63)));
}

// Double-buffered draws: lanes of t0 hold draws base0 + lane, lanes of t1 the next 64.  The next
// batch's table gather is issued as soon as the current one starts, so a pair never waits for
// the table.  take(k) = target of draw `used + k` (used + k < 128).
struct DrawPipe {
    uint32_t t0, t1;
    uint64_t base0, base1;
    int used;

    template <class Args, class Lcg>
    __device__ inline uint32_t gather(uint64_t base, const Lcg &lc, const Args &a) {
        const uint64_t s = lcg_state_of(base, lc);  // draw base + lane
        return table_value(a, table_slot(s, a.fm.m, a.fm.d));
    }

    // gather() plus the drawn row's hot bit (a.hot) in bit 31 (rows are < 2^31); a table value
    // outside [0, V) gets no bit and stays out of range.  The bitmap word is one more dependent
    // per-lane load, 64 draws ahead of use.
    template <class Args, class Lcg>
    __device__ inline uint32_t gather_hot(uint64_t base, const Lcg &lc, const Args &a) {
        const uint32_t v = gather(base, lc, a);
        if (a.hot == nullptr || (int64_t)v >= a.V) return v;
        return v | (((a.hot[v >> 5] >> (v & 31)) & 1u) << 31);
    }
};

// ---- O2: one wavefront per walk ------------------------------------------------------------

struct O2Args {
    float *node;
    float *ctx;
    const int32_t *walks;
    const uint64_t *seeds;
    const uint32_t *table;
    int64_t V;
    int64_t P;
    int L;
    int d;
    int window;
    int negative;
    float lr;
    float alpha;
    FastMod fm;
    int packed;        // table points to come_pack_table's words
    int64_t *counter;  // work queue: walks are claimed with atomicAdd (nullptr = grid-stride)
    unsigned long long *upd_count;  // optional: += target row updates applied (come.h
                                    // o2_update_count); one atomic per walk
    int fresh;       // direct kernel: rows read with agent-scope loads (bypass the CU's L1)
    int wb_atomic;   // direct kernel: row updates written as float-atomic deltas (none lost)
    const uint32_t *hot;  // HOG, optional: bitmap of contended rows (come_hot_rows); their
                          // updates are float-atomic deltas, their reads are per pair
};

// Row r is in the hot bitmap (wave-uniform r: one scalar load).
template <class Args>
__device__ inline bool is_hot(const Args &a, int r) {
    return a.hot != nullptr && ((a.hot[(uint32_t)r >> 5] >> (r & 31)) & 1u);
}

// Next unit of a wavefront: from the launch's work queue (one atomic per unit; a wavefront that
// starts late -- e.g. its CU was busy with a concurrent RCCL kernel -- simply claims fewer
// walks) or, without a queue, the static grid-stride sequence.
__device__ inline int64_t next_unit(int64_t *counter, int64_t cur, int64_t stride, int lane) {
    if (!counter) return cur + stride;
    int64_t v = 0;
    if (lane == 0) v = (int64_t)atomicAdd((unsigned long long *)counter, 1ull);
    return (int64_t)uniform64((uint64_t)v);  // lane 0 is the first active lane here
}

// State 64 draws after `base` (lane 63's state advanced once).
__device__ inline uint64_t advance64_uniform(uint64_t base) {
    return (kLcgA64 * base + kLcgC64) & kLcgMask;
}
__device__ inline uint64_t advance64(uint64_t base, const LcgLane &lc) {
    const uint64_t s = (lc.a * base + lc.c) & kLcgMask;
    return lcg_next(uniform64(readlane_u64(s, 63)));
}

template <int VEC, bool FULL>
__device__ inline void atomic_add_delta(float *__restrict__ row, const Row<VEC, FULL> &cur,
                                        const Row<VEC, FULL> &orig, int lane, int d) {
    Row<VEC, FULL> delta;
#pragma unroll
    for (int e = 0; e < VEC; ++e) delta.v[e] = cur.v[e] - orig.v[e];
    delta.atomic_add(row, lane, d);
}

// One O2 pair (pyx:105-151) with the input row `in` and the positive row `pos` already in
// registers.  Draws the pair's n negatives (pyx:133-135), gathers their rows, reduces every dot
// product, resolves the targets in reference order, stores the updated negative rows, updates
// `pos` in registers (pos_upd |= updated) and finally applies `in += work` (pyx:149).
template <int VEC, bool FULL, int MAXN>
__device__ inline void o2_pair(const O2Args &a, DrawBatch &db, const LcgLane &lc, int lane, int ci,
                               Row<VEC, FULL> &pos, bool &pos_upd, Row<VEC, FULL> &in,
                               Row<VEC, FULL> &work, int &nupd) {
    using R = Row<VEC, FULL>;
    const int n = a.negative;
    const int d = a.d;
    if (n > 0 && db.used + n > 64) draws_fill(db, draws_state_at_used(db, lc), lc, a);
    int t[MAXN + 1];
    bool valid[MAXN + 1];
    t[0] = ci;
    valid[0] = true;
#pragma unroll
    for (int k = 1; k <= MAXN; ++k) {
        if (k <= n) {
            const int tk = (int)readlane_u32(db.target, db.used + k - 1);
            t[k] = tk;
            // pyx:135 skip == positive; out-of-range table values skipped (no OOB)
            valid[k] = tk != ci && tk >= 0 && tk < a.V;
        } else {
            t[k] = -1;
            valid[k] = false;
        }
    }
    if (n > 0) db.used += n;

    R r[MAXN + 1], o[MAXN + 1];
#pragma unroll
    for (int k = 1; k <= MAXN; ++k)
        if (valid[k]) {
            r[k].load_as(a.ctx + (int64_t)t[k] * d, lane, d, a.fresh);
            o[k] = r[k];
        }

    // dots of every target against the (fixed) input row, butterflies interleaved
    float part[MAXN + 1];
    part[0] = lane_partial(in, pos);
#pragma unroll
    for (int k = 1; k <= MAXN; ++k) part[k] = valid[k] ? lane_partial(in, r[k]) : 0.0f;
    wave_sum_n(part, n + 1);

#pragma unroll
    for (int e = 0; e < VEC; ++e) work.v[e] = 0.0f;
    // positive (d == 0, label 1)
    {
        float sig;
        if (sigmoid_ref(uniformf(part[0]), &sig)) {
            const float g = ((1.0f - sig) * a.lr) * a.alpha;  // pyx:144
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                work.v[e] = __builtin_fmaf(g, pos.v[e], work.v[e]);  // pyx:146
                pos.v[e] = __builtin_fmaf(g, in.v[e], pos.v[e]);     // pyx:147
            }
            pos_upd = true;
            ++nupd;
        }
    }
    bool upd[MAXN + 1];
    upd[0] = false;
#pragma unroll
    for (int k = 1; k <= MAXN; ++k) {
        upd[k] = false;
        if (!valid[k]) continue;
        float f = part[k];
        // A repeated negative sees the row as left by its latest earlier occurrence.
        int prev = -1;
#pragma unroll
        for (int q = 1; q < k; ++q)
            if (valid[q] && t[q] == t[k]) prev = q;
        if (prev >= 0) {
#pragma unroll
            for (int q = 1; q < k; ++q) {
                if (q == prev) {
                    r[k] = r[q];
                    f = upd[q] ? wave_sum(lane_partial(in, r[k])) : part[q];
                }
            }
        }
        f = uniformf(f);
        part[k] = f;  // effective dot of this occurrence (a later repeat may reuse it)
        float sig;
        if (!sigmoid_ref(f, &sig)) continue;  // pyx:141-142
        const float g = ((0.0f - sig) * a.lr) * a.alpha;  // pyx:144, label 0
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
            work.v[e] = __builtin_fmaf(g, r[k].v[e], work.v[e]);  // pyx:146
            r[k].v[e] = __builtin_fmaf(g, in.v[e], r[k].v[e]);    // pyx:147
        }
        upd[k] = true;
        ++nupd;
    }
    // write back in order, so a repeated row ends with its last version; atomic mode adds the
    // row's change over the pair once (last updated occurrence minus the value loaded)
#pragma unroll
    for (int k = 1; k <= MAXN; ++k) {
        if (!upd[k]) continue;
        if (!a.wb_atomic && !is_hot(a, t[k])) {
            r[k].store(a.ctx + (int64_t)t[k] * d, lane, d);
            continue;
        }
        bool last = true;
#pragma unroll
        for (int q = k + 1; q <= MAXN; ++q)
            if (upd[q] && t[q] == t[k]) last = false;
        if (last) atomic_add_delta(a.ctx + (int64_t)t[k] * d, r[k], o[k], lane, d);
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) in.v[e] = in.v[e] + work.v[e];  // pyx:149
}

// Direct variant: every pair reads and writes its input and positive rows in HBM.  Used when the
// LDS ring of the cached variant would not fit (large window x d).
template <int VEC, bool FULL, int MAXN>
__global__ void __launch_bounds__(256) k_sgns_o2(O2Args a) {
    using R = Row<VEC, FULL>;
    const int lane = threadIdx.x & 63;
    const int64_t waves_per_block = blockDim.x >> 6;
    const int64_t gw = (int64_t)blockIdx.x * waves_per_block + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * waves_per_block;
    const LcgLane lc = lcg_lane_constants(lane);
    const int d = a.d;
    const int path_len = a.L < kMaxSentenceLen ? a.L : kMaxSentenceLen;  // pyx:480

    for (int64_t p = gw; p < a.P; p += nwaves) {
        const int32_t *__restrict__ idx = a.walks + p * (int64_t)a.L;
        DrawBatch db;
        db.used = 0;
        db.base = uniform64(a.seeds[p]);
        db.target = 0;
        if (a.negative > 0) draws_fill(db, db.base, lc, a);
        int nupd = 0;
        for (int i = 0; i < path_len; ++i) {
            const int ci = uniform(idx[i]);
            if (ci < 0 || ci >= a.V) continue;  // codelens[i] == 0 (pyx:495)
            const int j0 = i - a.window < 0 ? 0 : i - a.window;
            const int j1 = i + a.window + 1 > path_len ? path_len : i + a.window + 1;
            for (int j = j0; j < j1; ++j) {
                if (j == i) continue;
                const int cj = uniform(idx[j]);
                if (cj < 0 || cj >= a.V) continue;  // pyx:504
                R in, pos;
                in.load_as(a.node + (int64_t)cj * d, lane, d, a.fresh);
                pos.load_as(a.ctx + (int64_t)ci * d, lane, d, a.fresh);
                const R pos0 = pos;
                bool pos_upd = false;
                R work;
                o2_pair<VEC, FULL, MAXN>(a, db, lc, lane, ci, pos, pos_upd, in, work, nupd);
                // in += work and pos's change: at the memory side (float atomics) for contended
                // rows, plain stores otherwise
                if (pos_upd) {
                    if (a.wb_atomic || is_hot(a, ci))
                        atomic_add_delta(a.ctx + (int64_t)ci * d, pos, pos0, lane, d);
                    else
                        pos.store(a.ctx + (int64_t)ci * d, lane, d);
                }
                if (a.wb_atomic || is_hot(a, cj)) work.atomic_add(a.node + (int64_t)cj * d, lane, d);
                else in.store(a.node + (int64_t)cj * d, lane, d);
            }
        }
        if (a.upd_count && lane == 0 && nupd) atomicAdd(a.upd_count, (unsigned long long)nupd);
    }
}

// Cached, software-pipelined variant (the hot kernel).
//
// Traffic cuts, exact in sequential order:
//  * the center's positive row ctx[idx[i]] stays in registers across its 2w pairs (no negative of
//    those pairs can be that row: pyx:135 skips it) and is written back once per center;
//  * the input rows of the window [i-w, i+w] live in a per-wavefront LDS ring of 2w+1 rows: a
//    walk position's node row is read from HBM once, when it enters the window, instead of once
//    per pair.  Positions holding the same node id alias: entering copies the live LDS row, every
//    update is applied to all aliases.
// Latency hiding (one wavefront walks its pairs strictly in order, so memory-level parallelism
// has to come from running ahead):
//  * the walk's row indices sit in two VGPR chunks of 64 positions (v_readlane), refilled 64
//    positions ahead -- no dependent index loads;
//  * the next pair's negative rows are loaded while the current pair computes, the next center's
//    positive row and entering node row while the current center runs, the next 64 table draws
//    while the current 64 are consumed.  Every prefetched row that the current work writes before
//    it is used is replaced by the register copy (forwarding), so sequential order is preserved
//    bit for bit.  Prefetch loads are unconditional (out-of-range targets read row 0 and are
//    discarded) so the compiler's vmcnt waits stay counted, never vmcnt(0).
// Write-back: plain stores -- the positive once per center, a node row when its last alias leaves
// the window, negative rows per pair.
// This is the SEQUENTIAL-mode kernel (one wavefront, the parity anchor).  Its caching is exact
// only when no other wavefront touches the cached rows: for Hogwild, caching node rows for a
// window trains measurably worse on graphs with hubs (tests/test_gpu_tierc.py), so Hogwild runs
// k_sgns_o2_stream.
template <int VEC, bool FULL, int MAXN>
__global__ void __launch_bounds__(128) k_sgns_o2_ring(O2Args a) {
    using R = Row<VEC, FULL>;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x & 63;
    const int wib = threadIdx.x >> 6;
    const int64_t waves_per_block = blockDim.x >> 6;
    const int64_t gw = (int64_t)blockIdx.x * waves_per_block + wib;
    const int64_t nwaves = (int64_t)gridDim.x * waves_per_block;
    const LcgLane lc = lcg_lane_constants(lane);
    const int d = a.d;
    const int w = a.window;
    const int n = a.negative;
    const int RS = 2 * w + 1;  // ring slots (<= 64: ids live one per lane)
    const int path_len = a.L < kMaxSentenceLen ? a.L : kMaxSentenceLen;  // pyx:480
    const int wave_floats = (RS * d + 3) & ~3;
    float *ring = lds + wib * wave_floats;
    auto valid_row = [&](int r) { return r >= 0 && r < a.V; };
    auto slot_add = [&](int s, int delta) {  // (s + delta) mod RS for |delta| <= RS
        s += delta;
        if (s < 0) s += RS;
        if (s >= RS) s -= RS;
        return s;
    };

    for (int64_t p = a.counter ? next_unit(a.counter, 0, 0, lane) : gw; p < a.P;
         p = next_unit(a.counter, p, nwaves, lane)) {
        const int32_t *__restrict__ walk = a.walks + p * (int64_t)a.L;
        // ---- walk indices: positions [wbase, wbase + 128) in two VGPR chunks ----
        int wbase = 0;
        int c0 = lane < path_len ? walk[lane] : -1;
        int c1 = 64 + lane < path_len ? walk[64 + lane] : -1;
        auto idx_at = [&](int q) {  // validated row of walk position q (-1 = None / past the end)
            if (q >= path_len) return -1;
            const int off = q - wbase;
            const int r = off < 64 ? __builtin_amdgcn_readlane(c0, off)
                                   : __builtin_amdgcn_readlane(c1, off - 64);
            return valid_row(r) ? r : -1;
        };
        // ---- draws ----
        DrawPipe dp;
        dp.used = 0;
        dp.base0 = uniform64(a.seeds[p]);
        dp.t0 = dp.t1 = 0;
        if (n > 0) {
            dp.t0 = dp.gather(dp.base0, lc, a);
            dp.base1 = advance64(dp.base0, lc);
            dp.t1 = dp.gather(dp.base1, lc, a);
        }
        auto take = [&](int k) -> int {
            const int q = dp.used + k;
            return (int)(q < 64 ? readlane_u32(dp.t0, q) : readlane_u32(dp.t1, q - 64));
        };
        auto advance = [&]() {
            if (n == 0) return;
            dp.used += n;
            if (dp.used >= 64) {
                dp.used -= 64;
                dp.t0 = dp.t1;
                dp.base0 = dp.base1;
                dp.base1 = advance64(dp.base1, lc);
                dp.t1 = dp.gather(dp.base1, lc, a);
            }
        };
        // next pair's negatives: raw targets and their rows (row 0 stands in for bad targets)
        int tn[MAXN + 1];
        R rn[MAXN + 1];
        auto fetch_next = [&]() {
#pragma unroll
            for (int k = 1; k <= MAXN; ++k) {
                const int tk = k <= n ? take(k - 1) : -1;
                tn[k] = tk;
                rn[k].load(a.ctx + (int64_t)(valid_row(tk) ? tk : 0) * d, lane, d);
            }
        };
        fetch_next();

        int nupd = 0;  // target row updates of this walk (wave-uniform)
        // ---- ring (LDS rows) + ids (one per lane) ----
        int ids = -1;  // lane s: node row held by ring slot s
        auto id_of = [&](int s) { return __builtin_amdgcn_readlane(ids, s); };
        auto alias_mask = [&](int id, int except) -> uint64_t {
            return __ballot(lane < RS && lane != except && ids == id);
        };
        auto set_id = [&](int s, int id) { ids = lane == s ? id : ids; };
        auto write_back = [&](int s, int id) {  // the last holder of a node row stores it
            if (alias_mask(id, s) != 0) return;
            R row;
            row.load(ring + s * d, lane, d);
            row.store(a.node + (int64_t)id * d, lane, d);
        };
        auto enter_row = [&](int s, int id, const R &fetched) {  // fetched: node[id] loaded earlier
            const uint64_t m = alias_mask(id, s);
            if (m) {
                R row;
                row.load(ring + __builtin_ctzll(m) * d, lane, d);
                row.store(ring + s * d, lane, d);
            } else {
                fetched.store(ring + s * d, lane, d);
            }
            set_id(s, id);
        };
        for (int q = 0; q < w && q < path_len; ++q) {  // positions [0, w) before center 0
            const int id = idx_at(q);
            if (id >= 0) {
                R row;
                row.load(a.node + (int64_t)id * d, lane, d);
                enter_row(q, id, row);
            }
        }
        // center-level prefetch: the positive of the next center, the row entering with it
        R pos_n, ent_n;
        int pos_n_id = idx_at(0), ent_n_id = idx_at(w);
        pos_n.load(a.ctx + (int64_t)(pos_n_id >= 0 ? pos_n_id : 0) * d, lane, d);
        ent_n.load(a.node + (int64_t)(ent_n_id >= 0 ? ent_n_id : 0) * d, lane, d);

        int si = 0;  // slot of position i
        for (int i = 0; i < path_len; ++i) {
            // this center's prefetched rows, then prefetch for center i+1
            if (i + 1 + w >= wbase + 128) {  // keep [i, i + 1 + w] inside the two chunks
                wbase += 64;
                c0 = c1;
                c1 = wbase + 64 + lane < path_len ? walk[wbase + 64 + lane] : -1;
            }
            const int ci = pos_n_id;
            R pos = pos_n;
            // ring: position i-w-1 leaves, position i+w enters (same slot)
            const int se = slot_add(si, w);
            if (i + w < path_len || i - w - 1 >= 0) {
                const int old_id = i - w - 1 >= 0 ? id_of(se) : -1;
                if (old_id >= 0 && old_id == ent_n_id) {
                    // the same node leaves and enters: keep the live LDS row (no store, no load)
                } else {
                    if (old_id >= 0) write_back(se, old_id);
                    set_id(se, -1);
                    if (i + w < path_len && ent_n_id >= 0) enter_row(se, ent_n_id, ent_n);
                }
            }
            // prefetch for center i+1, after this boundary's write-back (a node that just left
            // may be the one entering next; its prefetched copy must not predate the store)
            pos_n_id = idx_at(i + 1);
            ent_n_id = idx_at(i + 1 + w);
            pos_n.load(a.ctx + (int64_t)(pos_n_id >= 0 ? pos_n_id : 0) * d, lane, d);
            ent_n.load(a.node + (int64_t)(ent_n_id >= 0 ? ent_n_id : 0) * d, lane, d);

            if (ci >= 0) {  // codelens[i] != 0 (pyx:495)
                bool pos_upd = false;
                const int j0 = i - w < 0 ? 0 : i - w;
                const int j1 = i + w + 1 > path_len ? path_len : i + w + 1;
                for (int j = j0; j < j1; ++j) {
                    if (j == i) continue;
                    const int sj = slot_add(si, j - i);
                    const int cj = id_of(sj);
                    if (cj < 0) continue;  // pyx:504
                    R in;
                    in.load(ring + sj * d, lane, d);
                    // this pair's negatives were prefetched; put the next pair's in flight
                    int t[MAXN + 1];
                    R r[MAXN + 1];
#pragma unroll
                    for (int k = 1; k <= MAXN; ++k) {
                        t[k] = tn[k];
                        r[k] = rn[k];
                    }
                    advance();
                    fetch_next();

                    // ---- the pair (pyx:128-149) ----
                    bool valid[MAXN + 1];
#pragma unroll
                    for (int k = 1; k <= MAXN; ++k)
                        valid[k] = k <= n && t[k] != ci && valid_row(t[k]);  // pyx:135
                    float part[MAXN + 1];
                    part[0] = lane_partial(in, pos);
#pragma unroll
                    for (int k = 1; k <= MAXN; ++k) part[k] = lane_partial(in, r[k]);
                    wave_sum_n(part, n + 1);
                    R work;
#pragma unroll
                    for (int e = 0; e < VEC; ++e) work.v[e] = 0.0f;
                    {
                        float sig;
                        if (sigmoid_ref(uniformf(part[0]), &sig)) {
                            const float g = ((1.0f - sig) * a.lr) * a.alpha;  // pyx:144
#pragma unroll
                            for (int e = 0; e < VEC; ++e) {
                                work.v[e] = __builtin_fmaf(g, pos.v[e], work.v[e]);  // pyx:146
                                pos.v[e] = __builtin_fmaf(g, in.v[e], pos.v[e]);     // pyx:147
                            }
                            pos_upd = true;
                            ++nupd;
                        }
                    }
                    bool upd[MAXN + 1];
#pragma unroll
                    for (int k = 1; k <= MAXN; ++k) {
                        upd[k] = false;
                        if (!valid[k]) continue;
                        float f = part[k];
                        int prev = -1;  // latest earlier occurrence of the same negative row
#pragma unroll
                        for (int q = 1; q < k; ++q)
                            if (valid[q] && t[q] == t[k]) prev = q;
                        if (prev >= 0) {
#pragma unroll
                            for (int q = 1; q < k; ++q) {
                                if (q == prev) {
                                    r[k] = r[q];
                                    f = upd[q] ? wave_sum(lane_partial(in, r[k])) : part[q];
                                }
                            }
                        }
                        f = uniformf(f);
                        part[k] = f;
                        float sig;
                        if (!sigmoid_ref(f, &sig)) continue;  // pyx:141-142
                        const float g = ((0.0f - sig) * a.lr) * a.alpha;  // pyx:144, label 0
#pragma unroll
                        for (int e = 0; e < VEC; ++e) {
                            work.v[e] = __builtin_fmaf(g, r[k].v[e], work.v[e]);  // pyx:146
                            r[k].v[e] = __builtin_fmaf(g, in.v[e], r[k].v[e]);    // pyx:147
                        }
                        upd[k] = true;
                        ++nupd;
                    }
#pragma unroll
                    for (int k = 1; k <= MAXN; ++k) {
                        if (!upd[k]) continue;
                        r[k].store(a.ctx + (int64_t)t[k] * d, lane, d);
                        // prefetched copies of this row are now stale: forward the new value
#pragma unroll
                        for (int q = 1; q <= MAXN; ++q)
                            if (tn[q] == t[k]) rn[q] = r[k];
                        if (pos_n_id == t[k]) pos_n = r[k];
                    }
#pragma unroll
                    for (int e = 0; e < VEC; ++e) in.v[e] = in.v[e] + work.v[e];  // pyx:149
                    uint64_t m = alias_mask(cj, -1);  // the slot and every alias of it
                    while (m) {
                        const int rr = __builtin_ctzll(m);
                        m &= m - 1;
                        in.store(ring + rr * d, lane, d);
                    }
                }
                if (pos_upd) {
                    pos.store(a.ctx + (int64_t)ci * d, lane, d);
#pragma unroll
                    for (int q = 1; q <= MAXN; ++q)
                        if (tn[q] == ci) rn[q] = pos;  // prefetched before this write-back
                    if (pos_n_id == ci) pos_n = pos;
                }
            }
            si = slot_add(si, 1);
        }
        // positions still in the ring leave in order
        const int first = path_len - w - 1 > 0 ? path_len - w - 1 : 0;
        for (int q = first; q < path_len; ++q) {
            const int s = q % RS;
            const int id = id_of(s);
            if (id >= 0) write_back(s, id);
            set_id(s, -1);
        }
        if (a.upd_count && lane == 0 && nupd) atomicAdd(a.upd_count, (unsigned long long)nupd);
    }
}

// Streaming Hogwild variant (COME_MODE_HOGWILD; the product's Hogwild mode).
//
// Semantics per pair are the reference thread's (pyx:128-149): the input row, the positive row and
// the negative rows are read from memory for the pair and written back after it -- nothing is
// cached across pairs except a cold center's positive row, held for that center's 2w pairs (no
// negative of those pairs can be that row, pyx:135).  Rows are split by contention (a.hot,
// come_hot_rows): cold rows are written back with plain stores (few other wavefronts touch them
// while the pair runs), hot rows (hubs) with float-atomic deltas at the memory side (none of the
// many concurrent updates lost).  Measured against the sequential oracle on a power-law graph
// (tests/test_gpu_tierc.py): caching node rows for a window (the ring kernel's traffic cut) and
// writing them back later trains 3.6-6% worse, plain stores for hubs 1.8% worse, this form within
// 1% (the 1% bar of SURVEY.md §8c tier C).
// Latency hiding as in the ring kernel, one pair ahead: the next pair's input row, its positive
// (when the center changes or is hot), its negative rows and the hot bits of its rows are in
// flight while the current pair computes; the next 64 table draws (with their hot bits) while the
// current 64 are consumed.  A prefetched copy of a row the current pair then updates is patched:
// a hot row's copy receives this wavefront's change additively (copy + delta: it keeps the other
// wavefronts' atomics it was loaded with), a cold row's copy is replaced by the stored value (what
// a read after the store returns; on walks that share no row the launch is bit-identical to the
// sequential order, tests/test_gpu_stream.py).
// Wavefronts per SIMD the stream kernel is compiled for: the kernel is latency-bound (one pair of
// loads in flight per wavefront), so at d <= 128, n <= 5 it is held to 64 VGPRs for 8 waves per
// SIMD (a 32-byte spill): 108 vs 119 ms per C3 launch at the 7 waves 70 VGPRs would give
// (profiles/r02_ab_stream_occupancy.txt).  Wider rows / more negatives keep their natural size:
// C5's <4, true, 10> held to 4 waves per SIMD ran 3.57 vs 2.10 s per 1M-walk launch
// (profiles/r05_ab_c5_waves.txt).
template <int VEC, int MAXN>
constexpr int stream_waves_per_eu() {
    return (VEC <= 2 && MAXN <= 5) ? 8 : 1;
}

template <int VEC, bool FULL, int MAXN>
__global__ void __launch_bounds__(256)
    __attribute__((amdgpu_waves_per_eu(stream_waves_per_eu<VEC, MAXN>())))
    k_sgns_o2_stream(O2Args a) {
    using R = Row<VEC, FULL>;
    const int lane = threadIdx.x & 63;
    const int64_t waves_per_block = blockDim.x >> 6;
    const int64_t gw = (int64_t)blockIdx.x * waves_per_block + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * waves_per_block;
    const LcgFromTable lc{lane};
    const int d = a.d;
    const int w = a.window;  // <= 31 (launcher): lookups never fall behind the index window
    const int n = a.negative;
    const int path_len = a.L < kMaxSentenceLen ? a.L : kMaxSentenceLen;  // pyx:480
    auto valid_row = [&](int r) { return r >= 0 && r < a.V; };
    constexpr uint32_t kHotBit = 0x80000000u;

    for (int64_t p = a.counter ? next_unit(a.counter, 0, 0, lane) : gw; p < a.P;
         p = next_unit(a.counter, p, nwaves, lane)) {
        const int32_t *__restrict__ walk = a.walks + p * (int64_t)a.L;
        // ---- walk indices: positions [wbase, wbase + 128) in two VGPR chunks, slid forward.
        // Each lane holds one position's row with its hot bit in bit 31 (gathered when the chunk
        // is loaded, 64 positions ahead of use); -1 = None / past the end.
        auto chunk = [&](int q0) {
            const int q = q0 + lane;
            int v = q < path_len ? walk[q] : -1;
            if (!valid_row(v)) return -1;
            if (a.hot != nullptr && ((a.hot[(uint32_t)v >> 5] >> (v & 31)) & 1u))
                v = (int)((uint32_t)v | kHotBit);
            return v;
        };
        int wbase = 0;
        int c0 = chunk(0);
        int c1 = chunk(64);
        auto raw_at = [&](int q) {  // encoded row of walk position q
            if (q >= path_len) return -1;
            while (q - wbase >= 128) {  // positions behind q - 2w are never asked for again
                wbase += 64;
                c0 = c1;
                c1 = chunk(wbase + 64);
            }
            const int off = q - wbase;
            return off < 64 ? __builtin_amdgcn_readlane(c0, off)
                            : __builtin_amdgcn_readlane(c1, off - 64);
        };
        // ---- pairs in the reference order (pyx:494-508): center i ascending, j ascending ----
        int it_i = 0, it_j = -1;
        auto next_pair = [&](int &ci, int &cj, int &pi, bool &hi, bool &hj) -> bool {
            for (;;) {
                if (it_i >= path_len) return false;
                const int i = it_i;
                const int j0 = i - w < 0 ? 0 : i - w;
                const int j1 = i + w + 1 > path_len ? path_len : i + w + 1;
                if (it_j < j0) it_j = j0;
                const int rci = raw_at(i);
                if (rci == -1 || it_j >= j1) {  // codelens[i] == 0, or the center is done
                    ++it_i;
                    it_j = -1;
                    continue;
                }
                const int j = it_j++;
                if (j == i) continue;
                const int rcj = raw_at(j);
                if (rcj == -1) continue;  // pyx:504
                ci = (int)((uint32_t)rci & ~kHotBit);
                cj = (int)((uint32_t)rcj & ~kHotBit);
                hi = ((uint32_t)rci & kHotBit) != 0;
                hj = ((uint32_t)rcj & kHotBit) != 0;
                pi = i;
                return true;
            }
        };
        // ---- draws (hot bit in bit 31) ----
        DrawPipe dp;
        dp.used = 0;
        dp.base0 = uniform64(a.seeds[p]);
        dp.t0 = dp.t1 = 0;
        if (n > 0) {
            dp.t0 = dp.gather_hot(dp.base0, lc, a);
            dp.base1 = advance64_uniform(dp.base0);
            dp.t1 = dp.gather_hot(dp.base1, lc, a);
        }
        auto take = [&](int k) -> uint32_t {
            const int q = dp.used + k;
            return q < 64 ? readlane_u32(dp.t0, q) : readlane_u32(dp.t1, q - 64);
        };
        auto advance = [&]() {
            if (n == 0) return;
            dp.used += n;
            if (dp.used >= 64) {
                dp.used -= 64;
                dp.t0 = dp.t1;
                dp.base0 = dp.base1;
                dp.base1 = advance64_uniform(dp.base1);
                dp.t1 = dp.gather_hot(dp.base1, lc, a);
            }
        };
        // ---- the next pair: ids, hot bits, rows in flight ----
        int nci = -1, ncj = -1, npi = -1;
        bool nhi = false, nhj = false;
        int tn[MAXN + 1];
        bool tnh[MAXN + 1];
        R in_n, pos_n, rn[MAXN + 1];
        int prev_i = -1;  // center of the pair just done
        // rows of the pair next_pair() just produced.  Negative rows are read non-temporally:
        // random rows with little reuse, so the caches keep the packed negative table's words
        // and the hot bitmap instead (with the packed table: 105.7-106.0 vs 108.1 ms per C3
        // launch; no gain with the plain table, profiles/r03_ab_nt_sites.txt)
        auto prefetch = [&](bool need_pos) {
            in_n.load(a.node + (int64_t)ncj * d, lane, d);
            if (need_pos) pos_n.load(a.ctx + (int64_t)nci * d, lane, d);
#pragma unroll
            for (int k = 1; k <= MAXN; ++k) {
                const uint32_t raw = k <= n ? take(k - 1) : 0xFFFFFFFFu;
                tn[k] = (int)(raw & ~kHotBit);
                tnh[k] = (raw & kHotBit) != 0;
                if (k > n) tn[k] = -1;
                rn[k].load_nt(a.ctx + (int64_t)(valid_row(tn[k]) ? tn[k] : 0) * d, lane, d);
            }
        };
        bool have = next_pair(nci, ncj, npi, nhi, nhj);
        if (have) prefetch(true);
        int nupd = 0;
        R pos;  // the current center's positive (carried across the center's pairs while cold)
        bool pos_upd = false;

        while (have) {
            // ---- the next pair becomes the current one ----
            const int ci = nci, cj = ncj, ic = npi;
            const bool hot_ci = nhi, hot_cj = nhj;
            R in = in_n;
            int t[MAXN + 1];
            bool th[MAXN + 1];
            R r[MAXN + 1];
#pragma unroll
            for (int k = 1; k <= MAXN; ++k) {
                t[k] = tn[k];
                th[k] = tnh[k];
                r[k] = rn[k];
            }
            const bool new_center = ic != prev_i;
            if (new_center || hot_ci) pos = pos_n;  // a hot positive is re-read for every pair
            if (new_center) pos_upd = false;
            prev_i = ic;
            // ---- put the pair after it in flight ----
            advance();
            have = next_pair(nci, ncj, npi, nhi, nhj);
            if (have) prefetch(npi != ic || nhi);

            // ---- the pair (pyx:128-149) ----
            bool valid[MAXN + 1];
#pragma unroll
            for (int k = 1; k <= MAXN; ++k)
                valid[k] = k <= n && t[k] != ci && valid_row(t[k]);  // pyx:135
            float part[MAXN + 1];
            part[0] = lane_partial(in, pos);
#pragma unroll
            for (int k = 1; k <= MAXN; ++k) part[k] = lane_partial(in, r[k]);
            wave_sum_n(part, n + 1);
            R work;
#pragma unroll
            for (int e = 0; e < VEC; ++e) work.v[e] = 0.0f;
            float gpos = 0.0f;  // this pair's g of the positive (0 = skipped)
            {
                float sig;
                if (sigmoid_ref(uniformf(part[0]), &sig)) {
                    const float g = ((1.0f - sig) * a.lr) * a.alpha;  // pyx:144
#pragma unroll
                    for (int e = 0; e < VEC; ++e) {
                        work.v[e] = __builtin_fmaf(g, pos.v[e], work.v[e]);  // pyx:146
                        pos.v[e] = __builtin_fmaf(g, in.v[e], pos.v[e]);     // pyx:147
                    }
                    pos_upd = true;
                    gpos = g;
                    ++nupd;
                }
            }
            bool upd[MAXN + 1];
            float gk[MAXN + 1];
#pragma unroll
            for (int k = 1; k <= MAXN; ++k) {
                upd[k] = false;
                gk[k] = 0.0f;
                if (!valid[k]) continue;
                float f = part[k];
                int prev = -1;  // latest earlier occurrence of the same negative row
#pragma unroll
                for (int q = 1; q < k; ++q)
                    if (valid[q] && t[q] == t[k]) prev = q;
                if (prev >= 0) {
#pragma unroll
                    for (int q = 1; q < k; ++q) {
                        if (q == prev) {
                            r[k] = r[q];
                            f = upd[q] ? wave_sum(lane_partial(in, r[k])) : part[q];
                        }
                    }
                }
                f = uniformf(f);
                part[k] = f;
                float sig;
                if (!sigmoid_ref(f, &sig)) continue;  // pyx:141-142
                const float g = ((0.0f - sig) * a.lr) * a.alpha;  // pyx:144, label 0
#pragma unroll
                for (int e = 0; e < VEC; ++e) {
                    work.v[e] = __builtin_fmaf(g, r[k].v[e], work.v[e]);  // pyx:146
                    r[k].v[e] = __builtin_fmaf(g, in.v[e], r[k].v[e]);    // pyx:147
                }
                upd[k] = true;
                gk[k] = g;
                ++nupd;
            }
            // ---- write-back: negatives (in order; a repeated row ends with its last version).
            // Prefetched copies of the row (the next pair's targets, read before this store):
            // hot -> + this occurrence's change (g * in; the memory-side atomics of other
            // wavefronts that the copy was loaded with are kept); cold -> replaced by the stored
            // value, exactly what a read after the store returns when no other wavefront wrote
            // the row meanwhile (the cold case; a concurrent plain update in that window is lost,
            // as in any plain read-modify-write of the reference's Hogwild) -- with walks that
            // share no row the launch is then bit-identical to the sequential order.  Written as
            // two branches: a select form of the same replacement let the compiler wait for the
            // prefetched copies' loads (826 vs 803 ms per C3 launch; round 2's additive patch for
            // every row 801 ms, not exact; re-reading the row after the store 803 ms;
            // profiles/r04_ab_stream_patch.txt) ----
#pragma unroll
            for (int k = 1; k <= MAXN; ++k) {
                if (!upd[k]) continue;
                if (th[k]) {
                    R dlt;  // this occurrence's change, g * in
#pragma unroll
                    for (int e = 0; e < VEC; ++e) dlt.v[e] = gk[k] * in.v[e];
                    dlt.atomic_add(a.ctx + (int64_t)t[k] * d, lane, d);
                    if constexpr (VEC <= 2) {
#pragma unroll
                        for (int q = 1; q <= MAXN; ++q)
                            if (tn[q] == t[k])
#pragma unroll
                                for (int e = 0; e < VEC; ++e) rn[q].v[e] += dlt.v[e];
                        if (have && nci == t[k] && (npi != ic || nhi))
#pragma unroll
                            for (int e = 0; e < VEC; ++e) pos_n.v[e] += dlt.v[e];
                    }
                } else {
                    r[k].store(a.ctx + (int64_t)t[k] * d, lane, d);
                    if constexpr (VEC <= 2) {
#pragma unroll
                        for (int q = 1; q <= MAXN; ++q)
                            if (tn[q] == t[k]) rn[q] = r[k];
                        if (have && nci == t[k] && (npi != ic || nhi)) pos_n = r[k];
                    }
                }
                if constexpr (VEC > 2) {
                    // wide rows: one patch for hot and cold copies, the row update's own fma
                    // (pyx:147) -- exact for a cold copy read after the previous store (it holds
                    // the row this pair updated), and without r[k] live past its store: 149
                    // instead of 181 VGPRs at d = 256, n = 10 (3 waves per SIMD instead of 2:
                    // 2137 vs 2741 ms per C5 launch; at C3 the branch form above is 1.4% faster,
                    // profiles/r04_ab_stream_patch.txt)
#pragma unroll
                    for (int q = 1; q <= MAXN; ++q)
                        if (tn[q] == t[k])
#pragma unroll
                            for (int e = 0; e < VEC; ++e)
                                rn[q].v[e] = __builtin_fmaf(gk[k], in.v[e], rn[q].v[e]);
                    if (have && nci == t[k] && (npi != ic || nhi))
#pragma unroll
                        for (int e = 0; e < VEC; ++e)
                            pos_n.v[e] = __builtin_fmaf(gk[k], in.v[e], pos_n.v[e]);
                }
            }
            // ---- the positive: hot -> this pair's change, g * in, now (memory side) and into the
            // prefetched copies; cold -> stored once when the center ends, and its final value
            // replaces prefetched copies (no other wavefront updates a cold row meanwhile)
            if (hot_ci && gpos != 0.0f) {
                R pdl;
#pragma unroll
                for (int e = 0; e < VEC; ++e) pdl.v[e] = gpos * in.v[e];
                pdl.atomic_add(a.ctx + (int64_t)ci * d, lane, d);
#pragma unroll
                for (int q = 1; q <= MAXN; ++q)
                    if (tn[q] == ci)
#pragma unroll
                        for (int e = 0; e < VEC; ++e) rn[q].v[e] += pdl.v[e];
                if (have && nci == ci)
#pragma unroll
                    for (int e = 0; e < VEC; ++e) pos_n.v[e] += pdl.v[e];
            } else if (!hot_ci && pos_upd && (!have || npi != ic)) {
                pos.store(a.ctx + (int64_t)ci * d, lane, d);
#pragma unroll
                for (int q = 1; q <= MAXN; ++q)
                    if (tn[q] == ci) rn[q] = pos;
                if (have && nci == ci) pos_n = pos;
            }
            // ---- the input row: in += work (pyx:149) ----
            if (hot_cj) {
                work.atomic_add(a.node + (int64_t)cj * d, lane, d);
            } else {
#pragma unroll
                for (int e = 0; e < VEC; ++e) in.v[e] = in.v[e] + work.v[e];
                in.store(a.node + (int64_t)cj * d, lane, d);
            }
            if (have && ncj == cj)
#pragma unroll
                for (int e = 0; e < VEC; ++e) in_n.v[e] += work.v[e];
        }
        if (a.upd_count && lane == 0 && nupd) atomicAdd(a.upd_count, (unsigned long long)nupd);
    }
}

// ---- O1: one wavefront per edge ------------------------------------------------------------
struct O1Args {
    float *node;
    const int32_t *edges;
    const uint64_t *seeds;
    const uint32_t *table;
    int64_t V;
    int64_t E;
    int d;
    int negative;
    float lr;
    FastMod fm;
    int packed;
    const uint32_t *hot;  // HOG, optional: contended rows (come_hot_rows), updated atomically
    int64_t chunk;        // k_sgns_o1_runs: consecutive edges per wavefront unit
};

template <int VEC, bool FULL, int MAXN>
__global__ void __launch_bounds__(256) k_sgns_o1(O1Args a) {
    using R = Row<VEC, FULL>;
    const int lane = threadIdx.x & 63;
    const int64_t waves_per_block = blockDim.x >> 6;
    const int64_t gw = (int64_t)blockIdx.x * waves_per_block + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * waves_per_block;
    const LcgLane lc = lcg_lane_constants(lane);
    const int n = a.negative;
    const int d = a.d;

    for (int64_t e = gw; e < a.E; e += nwaves) {
        const int u = uniform(a.edges[2 * e]);
        const int v = uniform(a.edges[2 * e + 1]);
        if (u < 0 || u >= a.V || v < 0 || v >= a.V) continue;  // reference: undefined behaviour
        // 2n draws: pair 1 uses draws 0..n-1, pair 2 draws n..2n-1 (state carried, pyx:444-448)
        DrawBatch db;
        db.used = 0;
        db.base = uniform64(a.seeds[e]);
        db.target = 0;
        if (n > 0) draws_fill(db, db.base, lc, a, 2 * n);  // only the 2n draws the edge uses

        int t1[MAXN + 1], t2[MAXN + 1];
        bool v1[MAXN + 1], v2[MAXN + 1];
        t1[0] = v;  // pair 1: input u, positive v (pyx:444)
        t2[0] = u;  // pair 2: input v, positive u (pyx:447)
        v1[0] = v2[0] = true;
#pragma unroll
        for (int k = 1; k <= MAXN; ++k) {
            if (k <= n) {
                t1[k] = (int)readlane_u32(db.target, k - 1);
                t2[k] = (int)readlane_u32(db.target, n + k - 1);
                v1[k] = t1[k] != v && t1[k] >= 0 && t1[k] < a.V;
                v2[k] = t2[k] != u && t2[k] >= 0 && t2[k] < a.V;
            } else {
                t1[k] = t2[k] = -1;
                v1[k] = v2[k] = false;
            }
        }
        // Every row both pairs read can be gathered up front: pair 1 writes only node[u]; pair 2
        // never reads node[u] through a negative (skipped, == its positive) and gets its positive
        // (and, for a self-loop, its input) forwarded from pair 1's registers.
        R in1, in2;
        in1.load(a.node + (int64_t)u * d, lane, d);
        if (v != u) in2.load(a.node + (int64_t)v * d, lane, d);
        const bool hot_u = is_hot(a, u), hot_v = is_hot(a, v);
        R r1[MAXN + 1], r2[MAXN + 1];
#pragma unroll
        for (int k = 1; k <= MAXN; ++k) {
            if (v1[k]) r1[k].load(a.node + (int64_t)t1[k] * d, lane, d);
            if (v2[k]) r2[k].load(a.node + (int64_t)t2[k] * d, lane, d);
        }
        if (v != u) r1[0] = in2; else r1[0] = in1;  // positive of pair 1 = node[v] (pre-update)

        // pair 1
        {
            float part[MAXN + 1];
#pragma unroll
            for (int k = 0; k <= MAXN; ++k) part[k] = v1[k] ? lane_partial(in1, r1[k]) : 0.0f;
            wave_sum_n(part, n + 1);
            R work;
#pragma unroll
            for (int q = 0; q < VEC; ++q) work.v[q] = 0.0f;
#pragma unroll
            for (int k = 0; k <= MAXN; ++k) {
                if (!v1[k]) continue;
                float sig;
                if (!sigmoid_ref(uniformf(part[k]), &sig)) continue;
                const float g = ((k == 0 ? 1.0f : 0.0f) - sig) * a.lr;  // pyx:243
#pragma unroll
                for (int q = 0; q < VEC; ++q) work.v[q] = __builtin_fmaf(g, r1[k].v[q], work.v[q]);
            }
#pragma unroll
            for (int q = 0; q < VEC; ++q) in1.v[q] = in1.v[q] + work.v[q];  // pyx:247
            if (hot_u) work.atomic_add(a.node + (int64_t)u * d, lane, d);
            else in1.store(a.node + (int64_t)u * d, lane, d);
        }
        // pair 2: positive = node[u] as pair 1 left it; self-loop: the input is that row too.
        r2[0] = in1;
        if (v == u) in2 = in1;
        {
            float part[MAXN + 1];
#pragma unroll
            for (int k = 0; k <= MAXN; ++k) part[k] = v2[k] ? lane_partial(in2, r2[k]) : 0.0f;
            wave_sum_n(part, n + 1);
            R work;
#pragma unroll
            for (int q = 0; q < VEC; ++q) work.v[q] = 0.0f;
#pragma unroll
            for (int k = 0; k <= MAXN; ++k) {
                if (!v2[k]) continue;
                float sig;
                if (!sigmoid_ref(uniformf(part[k]), &sig)) continue;
                const float g = ((k == 0 ? 1.0f : 0.0f) - sig) * a.lr;
#pragma unroll
                for (int q = 0; q < VEC; ++q) work.v[q] = __builtin_fmaf(g, r2[k].v[q], work.v[q]);
            }
#pragma unroll
            for (int q = 0; q < VEC; ++q) in2.v[q] = in2.v[q] + work.v[q];
            if (hot_v) work.atomic_add(a.node + (int64_t)v * d, lane, d);
            else in2.store(a.node + (int64_t)v * d, lane, d);
        }
    }
}

// Kernel entry addresses per instantiation (defined in come_sgns_vec{1,2,4,8}.hip so the
// instantiations compile in parallel).
// O1 with the input row held over runs of edges (a.chunk > 0; option o1_chunk): a wavefront takes
// `chunk` consecutive edges and processes them in order, as one of the reference's worker
// threads does with its job of consecutive edges (node_embeddings.py:58-95).  Edge lists come
// grouped by their first endpoint (G.edges() order: all (u, *) of a node together), so the
// wavefront keeps node[u] in registers for the run of edges sharing u -- read once, updated by
// every pair-1 of the run (pyx:444: input u) and read as pair 2's positive (pyx:447) -- and writes
// it back once when u changes or the chunk ends: a float-atomic delta of the run's updates if u is
// contended, else a plain store.  Any target row equal to the held u is taken from the registers.
// One wavefront in sequential mode: bit-identical to k_sgns_o1 (the held row is what memory holds).
// Wavefronts per SIMD the run kernel is compiled for: latency-bound like the stream kernel (one
// edge's rows in flight per wavefront), so at d <= 128, n <= 5 it is held to 64 VGPRs (a 12-byte
// prologue spill) for 8 waves per SIMD and launched 8 four-wave workgroups per CU: C2 at lr 0.1
// 1.161 vs 1.277 ms per pass at its natural 79 VGPRs / 6 waves (7 waves: 1.186 ms;
// profiles/r05_ab_o1_waves.txt).
template <int VEC, int MAXN>
constexpr int o1_runs_waves_per_eu() {
    return (VEC <= 2 && MAXN <= 5) ? 8 : 1;
}

template <int VEC, bool FULL, int MAXN>
__global__ void __launch_bounds__(256)
    __attribute__((amdgpu_waves_per_eu(o1_runs_waves_per_eu<VEC, MAXN>())))
    k_sgns_o1_runs(O1Args a) {
    using R = Row<VEC, FULL>;
    const int lane = threadIdx.x & 63;
    const int64_t waves_per_block = blockDim.x >> 6;
    const int64_t gw = (int64_t)blockIdx.x * waves_per_block + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * waves_per_block;
    const LcgLane lc = lcg_lane_constants(lane);
    const int n = a.negative;
    const int d = a.d;
    const int64_t nchunks = (a.E + a.chunk - 1) / a.chunk;

    for (int64_t c = gw; c < nchunks; c += nwaves) {
        const int64_t e0 = c * a.chunk;
        const int64_t e1 = e0 + a.chunk < a.E ? e0 + a.chunk : a.E;
        int cu = -1;        // the held row (wave-uniform), -1 = none
        bool hot_cu = false;
        R hu, du;           // its value and this run's change
        auto flush = [&]() {
            if (cu < 0) return;
            if (hot_cu) du.atomic_add(a.node + (int64_t)cu * d, lane, d);
            else hu.store(a.node + (int64_t)cu * d, lane, d);
        };
        for (int64_t e = e0; e < e1; ++e) {
            const int u = uniform(a.edges[2 * e]);
            const int v = uniform(a.edges[2 * e + 1]);
            if (u < 0 || u >= a.V || v < 0 || v >= a.V) continue;  // reference: undefined
            if (u != cu) {
                flush();
                cu = u;
                hot_cu = is_hot(a, u);
                hu.load(a.node + (int64_t)u * d, lane, d);
#pragma unroll
                for (int q = 0; q < VEC; ++q) du.v[q] = 0.0f;
            }
            DrawBatch db;
            db.used = 0;
            db.base = uniform64(a.seeds[e]);
            db.target = 0;
            if (n > 0) draws_fill(db, db.base, lc, a, 2 * n);
            int t1[MAXN + 1], t2[MAXN + 1];
            bool v1[MAXN + 1], v2[MAXN + 1];
            t1[0] = v;
            t2[0] = u;
            v1[0] = v2[0] = true;
#pragma unroll
            for (int k = 1; k <= MAXN; ++k) {
                if (k <= n) {
                    t1[k] = (int)readlane_u32(db.target, k - 1);
                    t2[k] = (int)readlane_u32(db.target, n + k - 1);
                    v1[k] = t1[k] != v && t1[k] >= 0 && t1[k] < a.V;
                    v2[k] = t2[k] != u && t2[k] >= 0 && t2[k] < a.V;
                } else {
                    t1[k] = t2[k] = -1;
                    v1[k] = v2[k] = false;
                }
            }
            R in2;
            if (v != u) in2.load(a.node + (int64_t)v * d, lane, d);
            const bool hot_v = is_hot(a, v);
            R r1[MAXN + 1], r2[MAXN + 1];
#pragma unroll
            for (int k = 1; k <= MAXN; ++k) {
                if (v1[k]) {
                    if (t1[k] == u) r1[k] = hu;  // the held row (pair 1's input, pre-update)
                    else r1[k].load(a.node + (int64_t)t1[k] * d, lane, d);
                }
                if (v2[k] && t2[k] != v) r2[k].load(a.node + (int64_t)t2[k] * d, lane, d);
            }
            r1[0] = v != u ? in2 : hu;  // pair 1's positive node[v] (pre-update)
            // pair 1: input = the held u
            {
                float part[MAXN + 1];
#pragma unroll
                for (int k = 0; k <= MAXN; ++k) part[k] = v1[k] ? lane_partial(hu, r1[k]) : 0.0f;
                wave_sum_n(part, n + 1);
                R work;
#pragma unroll
                for (int q = 0; q < VEC; ++q) work.v[q] = 0.0f;
#pragma unroll
                for (int k = 0; k <= MAXN; ++k) {
                    if (!v1[k]) continue;
                    float sig;
                    if (!sigmoid_ref(uniformf(part[k]), &sig)) continue;
                    const float g = ((k == 0 ? 1.0f : 0.0f) - sig) * a.lr;  // pyx:243
#pragma unroll
                    for (int q = 0; q < VEC; ++q) work.v[q] = __builtin_fmaf(g, r1[k].v[q], work.v[q]);
                }
#pragma unroll
                for (int q = 0; q < VEC; ++q) {
                    hu.v[q] = hu.v[q] + work.v[q];  // pyx:247
                    du.v[q] = du.v[q] + work.v[q];
                }
            }
            // pair 2: input v, positive = the held u as pair 1 left it; a self-loop's input is
            // that row too; a negative equal to v reads v before pair 2's update
            r2[0] = hu;
            if (v == u) in2 = hu;
#pragma unroll
            for (int k = 1; k <= MAXN; ++k)
                if (v2[k] && t2[k] == v) r2[k] = in2;
            {
                float part[MAXN + 1];
#pragma unroll
                for (int k = 0; k <= MAXN; ++k) part[k] = v2[k] ? lane_partial(in2, r2[k]) : 0.0f;
                wave_sum_n(part, n + 1);
                R work;
#pragma unroll
                for (int q = 0; q < VEC; ++q) work.v[q] = 0.0f;
#pragma unroll
                for (int k = 0; k <= MAXN; ++k) {
                    if (!v2[k]) continue;
                    float sig;
                    if (!sigmoid_ref(uniformf(part[k]), &sig)) continue;
                    const float g = ((k == 0 ? 1.0f : 0.0f) - sig) * a.lr;
#pragma unroll
                    for (int q = 0; q < VEC; ++q) work.v[q] = __builtin_fmaf(g, r2[k].v[q], work.v[q]);
                }
                if (v == u) {  // self-loop: pair 2 updates the held row itself
#pragma unroll
                    for (int q = 0; q < VEC; ++q) {
                        hu.v[q] = hu.v[q] + work.v[q];
                        du.v[q] = du.v[q] + work.v[q];
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < VEC; ++q) in2.v[q] = in2.v[q] + work.v[q];
                    if (hot_v) work.atomic_add(a.node + (int64_t)v * d, lane, d);
                    else in2.store(a.node + (int64_t)v * d, lane, d);
                }
            }
        }
        flush();
    }
}

struct KernelSet {
    void *o2_direct[2][3];  // [FULL][maxn idx]
    void *o2_ring[2][3];    // sequential mode
    void *o2_stream[2][3];  // Hogwild mode
    void *o1[2][3];
    void *o1_runs[2][3];
};
#define COME_DECLARE_VEC(V) \
    const KernelSet &kernels_vec##V(); \
    hipError_t upload_exp_table_vec##V(const float *host1000);
COME_DECLARE_VEC(1)
COME_DECLARE_VEC(2)
COME_DECLARE_VEC(4)
COME_DECLARE_VEC(8)
#undef COME_DECLARE_VEC

}  // namespace come
