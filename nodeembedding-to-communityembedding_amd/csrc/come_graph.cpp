// come_graph.cpp -- host side of the walk producer (the reference's utils/graph_utils.py) and of
// the on-disk text formats around the hot path (graph_utils.py, IO_utils.py).  Plain C++17, no
// HIP: the exact-stream walker is inherently sequential per random stream (CPython's MT19937 with
// data-dependent rejection sampling), so it runs on host threads, one stream per thread -- the
// same granularity as the reference's one-process-per-walk-file pool (graph_utils.py:144-146).
//
//  * graph build in networkx order: nx.Graph().add_edges_from(rows) (graph_utils.py:60-69) keeps
//    nodes in first-appearance order and every adjacency in insertion order; G.edges() walks
//    nodes in that order and skips already-visited endpoints; G.degree() counts a self-loop twice.
//  * CPython's random.Random: MT19937 (init_by_array seeding), random(), getrandbits(k) for
//    k <= 32, _randbelow (rejection on k = n.bit_length() bits), shuffle, choice (CPython 3.10,
//    Modules/_randommodule.c and Lib/random.py) -- restated, bit-exact.
//  * build_deepwalk_corpus_iter (graph_utils.py:187-192) + __random_walk__ (:20-46).
//  * text formats: edge lists (:49-69, 72-109), walk files (:112-120, 149-154), embeddings
//    (IO_utils.py:49-62, numpy float32 str() = shortest round-trip digits).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <charconv>
#include <cmath>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/come.h"

namespace come {
int set_error(int code, const char *fmt, ...);
}
using come::set_error;

namespace {

// ---- CPython random.Random ----------------------------------------------------------------
struct PyRandom {
    static constexpr int N = 624, M = 397;
    uint32_t mt[N];
    int mti;

    void init_genrand(uint32_t s) {
        mt[0] = s;
        for (mti = 1; mti < N; mti++)
            mt[mti] = 1812433253U * (mt[mti - 1] ^ (mt[mti - 1] >> 30)) + (uint32_t)mti;
    }
    void init_by_array(const uint32_t *key, int len) {
        init_genrand(19650218U);
        int i = 1, j = 0;
        for (int k = N > len ? N : len; k; k--) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525U)) + key[j] + (uint32_t)j;
            i++;
            j++;
            if (i >= N) {
                mt[0] = mt[N - 1];
                i = 1;
            }
            if (j >= len) j = 0;
        }
        for (int k = N - 1; k; k--) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941U)) - (uint32_t)i;
            i++;
            if (i >= N) {
                mt[0] = mt[N - 1];
                i = 1;
            }
        }
        mt[0] = 0x80000000U;
        mti = N;
    }
    // random.seed(int): key = 32-bit words of abs(seed), least significant first, at least one
    void seed(uint64_t s) {
        uint32_t key[2] = {(uint32_t)s, (uint32_t)(s >> 32)};
        init_by_array(key, key[1] ? 2 : 1);
    }
    uint32_t genrand() {
        static const uint32_t mag01[2] = {0x0U, 0x9908b0dfU};
        uint32_t y;
        if (mti >= N) {
            int kk;
            for (kk = 0; kk < N - M; kk++) {
                y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
                mt[kk] = mt[kk + M] ^ (y >> 1) ^ mag01[y & 0x1U];
            }
            for (; kk < N - 1; kk++) {
                y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
                mt[kk] = mt[kk + (M - N)] ^ (y >> 1) ^ mag01[y & 0x1U];
            }
            y = (mt[N - 1] & 0x80000000U) | (mt[0] & 0x7fffffffU);
            mt[N - 1] = mt[M - 1] ^ (y >> 1) ^ mag01[y & 0x1U];
            mti = 0;
        }
        y = mt[mti++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680U;
        y ^= (y << 15) & 0xefc60000U;
        y ^= (y >> 18);
        return y;
    }
    double random() {  // random_random: 53-bit float from two draws
        const uint32_t a = genrand() >> 5, b = genrand() >> 6;
        return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
    }
    uint64_t randbelow(uint64_t n) {  // _randbelow_with_getrandbits, n < 2^32 + 1
        if (n == 0) return 0;
        int k = 64 - __builtin_clzll(n);  // n.bit_length()
        if (k <= 32) {
            uint32_t r = genrand() >> (32 - k);
            while (r >= n) r = genrand() >> (32 - k);
            return r;
        }
        // 33..64 bits: getrandbits concatenates 32-bit words, least significant first
        for (;;) {
            uint64_t lo = genrand();
            uint64_t hi = genrand() >> (64 - k);
            uint64_t r = (hi << 32) | lo;
            if (r < n) return r;
        }
    }
    // Whole blocks at once (come_np_draw_seeds): regenerate the 624 words in place and temper
    // all of them -- branch-free loops the compiler vectorises (genrand() above costs ~1.4 ns
    // per output with its per-call branch; this ~0.4 ns).  Same recurrence, same outputs.
    void regenerate() {
        int kk;
        for (kk = 0; kk < N - M; kk++) {  // reads mt[kk + 1], mt[kk + M]: not yet rewritten
            const uint32_t y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
            mt[kk] = mt[kk + M] ^ (y >> 1) ^ ((0U - (y & 1U)) & 0x9908b0dfU);
        }
        for (; kk < N - 1; kk++) {  // reads mt[kk + M - N]: rewritten 227 words earlier
            const uint32_t y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
            mt[kk] = mt[kk + (M - N)] ^ (y >> 1) ^ ((0U - (y & 1U)) & 0x9908b0dfU);
        }
        const uint32_t y = (mt[N - 1] & 0x80000000U) | (mt[0] & 0x7fffffffU);
        mt[N - 1] = mt[M - 1] ^ (y >> 1) ^ ((0U - (y & 1U)) & 0x9908b0dfU);
        mti = 0;
    }
    static uint32_t temper(uint32_t y) {
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680U;
        y ^= (y << 15) & 0xefc60000U;
        y ^= (y >> 18);
        return y;
    }
    void get(uint32_t *st) const {
        memcpy(st, mt, sizeof(mt));
        st[N] = (uint32_t)mti;
    }
    bool set(const uint32_t *st) {
        if (st[N] > (uint32_t)N) return false;
        memcpy(mt, st, sizeof(mt));
        mti = (int)st[N];
        return true;
    }
};

// One stream of build_deepwalk_corpus_iter (graph_utils.py:187-192): per pass shuffle the node
// list in place (the list persists across passes) and start one walk at every node.
void corpus_stream(const int64_t *rowptr, const int32_t *col, int64_t V, int num_paths, int L,
                   double alpha, PyRandom &rng, const int32_t *emit, int32_t *out) {
    std::vector<int32_t> nodes(V);
    for (int64_t i = 0; i < V; ++i) nodes[i] = (int32_t)i;  // list(G.nodes())
    int64_t w = 0;
    for (int p = 0; p < num_paths; ++p) {
        for (int64_t i = V - 1; i >= 1; --i) {  // random.shuffle
            const int64_t j = (int64_t)rng.randbelow((uint64_t)i + 1);
            std::swap(nodes[i], nodes[j]);
        }
        for (int64_t s = 0; s < V; ++s, ++w) {
            int32_t *row = out + w * (int64_t)L;
            const int32_t start = nodes[s];
            int len = 0;
            if (L > 0) row[len++] = start;  // path = [start]
            int32_t cur = start;
            while (len < L) {  // __random_walk__ (:34-45)
                const int64_t b = rowptr[cur], deg = rowptr[cur + 1] - b;
                if (deg <= 0) break;
                if (rng.random() >= alpha)
                    cur = col[b + (int64_t)rng.randbelow((uint64_t)deg)];
                else
                    cur = start;
                row[len++] = cur;
            }
            if (emit)
                for (int t = 0; t < len; ++t) row[t] = emit[row[t]];
            for (int t = len; t < L; ++t) row[t] = -1;
        }
    }
}

// ---- numbers <-> text ------------------------------------------------------------------------
struct Reader {
    FILE *f = nullptr;
    std::vector<char> buf;
    explicit Reader(const char *path) : f(fopen(path, "rb")), buf(1 << 20) {}
    ~Reader() {
        if (f) fclose(f);
    }
    // Calls fn(tokens) for every line (tokens = the line's integers); returns false on a
    // malformed token.  Lines starting with '#' and blank lines are skipped.
    template <class Fn>
    bool lines(Fn fn) {
        std::string carry;
        std::vector<int64_t> toks;
        size_t n;
        auto line = [&](const char *s, const char *e) {
            if (s == e || *s == '#') return true;
            toks.clear();
            while (s < e) {
                while (s < e && (*s == ' ' || *s == '\t' || *s == '\r')) ++s;
                if (s >= e) break;
                int64_t v;
                auto r = std::from_chars(s, e, v);
                if (r.ec != std::errc()) return false;
                s = r.ptr;
                if (s < e && !(*s == ' ' || *s == '\t' || *s == '\r')) return false;
                toks.push_back(v);
            }
            if (!toks.empty()) fn(toks);
            return true;
        };
        while ((n = fread(buf.data(), 1, buf.size(), f)) > 0) {
            const char *p = buf.data(), *end = p + n;
            for (;;) {
                const char *nl = (const char *)memchr(p, '\n', end - p);
                if (!nl) {
                    carry.append(p, end);
                    break;
                }
                bool ok;
                if (!carry.empty()) {
                    carry.append(p, nl);
                    ok = line(carry.data(), carry.data() + carry.size());
                    carry.clear();
                } else {
                    ok = line(p, nl);
                }
                if (!ok) return false;
                p = nl + 1;
            }
        }
        return carry.empty() || line(carry.data(), carry.data() + carry.size());
    }
};

// numpy float32 str(): shortest round-trip digits, positional for 1e-4 <= |x| < 1e16 (with a
// trailing ".0" on integral values), scientific otherwise ("1.5e-05", exponent >= 2 digits).
int format_f32(float x, char *o) {
    if (std::isnan(x)) return (int)(stpcpy(o, "nan") - o);
    if (std::isinf(x)) return (int)(stpcpy(o, x < 0 ? "-inf" : "inf") - o);
    const float ax = std::fabs(x);
    if (x == 0.0f) return (int)(stpcpy(o, std::signbit(x) ? "-0.0" : "0.0") - o);
    if ((double)ax >= 1e-4 && (double)ax < 1e16) {  // numpy compares in double
        // shortest digits from the scientific form, then laid out positionally (numpy pads
        // with zeros beyond the shortest digits instead of printing the exact integer)
        char sci[64];
        auto r = std::to_chars(sci, sci + sizeof(sci), ax, std::chars_format::scientific);
        char *ep = (char *)memchr(sci, 'e', r.ptr - sci);
        int exp10 = 0;  // sci is not NUL-terminated: parse [ep + 1, r.ptr) only
        const char *xs = ep + 1;
        if (*xs == '+') ++xs;
        std::from_chars(xs, r.ptr, exp10);
        char dig[32];
        int nd = 0;
        for (char *c = sci; c < ep; ++c)
            if (*c != '.') dig[nd++] = *c;
        char *e = o;
        if (x < 0) *e++ = '-';
        if (exp10 >= nd - 1) {  // integral: digits, zeros, ".0"
            memcpy(e, dig, nd);
            e += nd;
            for (int i = 0; i < exp10 - (nd - 1); ++i) *e++ = '0';
            *e++ = '.';
            *e++ = '0';
        } else if (exp10 >= 0) {
            memcpy(e, dig, exp10 + 1);
            e += exp10 + 1;
            *e++ = '.';
            memcpy(e, dig + exp10 + 1, nd - exp10 - 1);
            e += nd - exp10 - 1;
        } else {
            *e++ = '0';
            *e++ = '.';
            for (int i = 0; i < -exp10 - 1; ++i) *e++ = '0';
            memcpy(e, dig, nd);
            e += nd;
        }
        return (int)(e - o);
    }
    auto r = std::to_chars(o, o + 64, x, std::chars_format::scientific);
    return (int)(r.ptr - o);
}

}  // namespace

// =============================================================================================
extern "C" int come_pyrandom_seed(uint64_t seed, uint32_t *state625) {
    if (!state625) return set_error(COME_E_INVALID, "null state");
    PyRandom r;
    r.seed(seed);
    r.get(state625);
    return COME_OK;
}

extern "C" int come_pyrandom_draw(uint32_t *state625, int kind, uint64_t arg, int64_t count,
                                  double *out) {
    if (!state625 || (!out && count > 0)) return set_error(COME_E_INVALID, "null pointer");
    PyRandom r;
    if (!r.set(state625)) return set_error(COME_E_INVALID, "bad MT19937 state position");
    for (int64_t i = 0; i < count; ++i) {
        if (kind == 0) out[i] = r.random();
        else if (kind == 1) out[i] = (double)r.randbelow(arg);
        else return set_error(COME_E_INVALID, "kind must be 0 (random) or 1 (randbelow)");
    }
    r.get(state625);
    return COME_OK;
}

extern "C" int come_np_draw_seeds(uint32_t *state625, int64_t n, uint64_t *out) {
    if (!state625 || (!out && n > 0)) return set_error(COME_E_INVALID, "null pointer");
    if (n < 0) return set_error(COME_E_INVALID, "n must be >= 0");
    PyRandom r;  // CPython's MT19937 core is numpy's legacy one (genrand_int32, same state)
    if (!r.set(state625)) return set_error(COME_E_INVALID, "bad MT19937 state position");
    // 2n consecutive outputs (randint(0, 2^24) each: one output masked, never rejected), block
    // by block: out[i] = 2^24 * t[2i] + t[2i + 1]
    uint32_t t[PyRandom::N + 1];
    int64_t need = 2 * n, done = 0;
    uint64_t hi = 0;
    bool have_hi = false;
    while (need > 0) {
        if (r.mti >= PyRandom::N) r.regenerate();
        const int take = (int)std::min<int64_t>(need, PyRandom::N - r.mti);
        for (int k = 0; k < take; ++k) t[k] = PyRandom::temper(r.mt[r.mti + k]) & 0xFFFFFFu;
        r.mti += take;
        need -= take;
        int k = 0;
        if (have_hi) {  // the high half drawn at the end of the previous block
            out[done++] = (hi << 24) + t[0];
            have_hi = false;
            k = 1;
        }
        for (; k + 1 < take; k += 2) out[done++] = ((uint64_t)t[k] << 24) + t[k + 1];
        if (k < take) {
            hi = t[k];
            have_hi = true;
        }
    }
    r.get(state625);
    return COME_OK;
}

extern "C" int come_graph_from_edges(const int64_t *edges, int64_t E, int64_t *node_ids,
                                     int64_t *V_out, int64_t *rowptr, int32_t *col,
                                     int64_t *degree, int32_t *edge_pos, int64_t *E_out) {
    if (E < 0 || (E > 0 && !edges)) return set_error(COME_E_INVALID, "bad edge array");
    if (!node_ids || !V_out || !rowptr || !col || !degree || !edge_pos || !E_out)
        return set_error(COME_E_INVALID, "null output pointer");
    if (2 * E > INT32_MAX) return set_error(COME_E_INVALID, "too many edges for int32 positions");
    std::unordered_map<int64_t, int32_t> pos;
    pos.reserve((size_t)(2 * E + 1));
    std::vector<std::vector<int32_t>> adj;
    std::unordered_set<uint64_t> seen_pair;
    seen_pair.reserve((size_t)(2 * E + 1));
    int64_t V = 0;
    auto node = [&](int64_t id) {
        auto it = pos.find(id);
        if (it != pos.end()) return it->second;
        pos.emplace(id, (int32_t)V);
        node_ids[V] = id;
        adj.emplace_back();
        return (int32_t)V++;
    };
    std::vector<uint8_t> selfloop;
    for (int64_t e = 0; e < E; ++e) {  // add_edges_from: u, then v, then adj[u][v], adj[v][u]
        const int32_t u = node(edges[2 * e]);
        const int32_t v = node(edges[2 * e + 1]);
        const uint64_t key = ((uint64_t)(uint32_t)u << 32) | (uint32_t)v;
        if (!seen_pair.insert(key).second) continue;  // existing key keeps its position
        adj[u].push_back(v);
        if (u != v) {
            seen_pair.insert(((uint64_t)(uint32_t)v << 32) | (uint32_t)u);
            adj[v].push_back(u);
        }
    }
    rowptr[0] = 0;
    int64_t nnz = 0, ne = 0;
    std::vector<uint8_t> done(V, 0);
    for (int64_t n = 0; n < V; ++n) {
        bool loop = false;
        for (int32_t m : adj[n]) {
            col[nnz++] = m;
            loop |= (m == n);
            if (!done[m]) {  // Graph.edges(): skip neighbours already visited
                edge_pos[2 * ne] = (int32_t)n;
                edge_pos[2 * ne + 1] = m;
                ++ne;
            }
        }
        done[n] = 1;
        rowptr[n + 1] = nnz;
        degree[n] = (int64_t)adj[n].size() + (loop ? 1 : 0);  // a self-loop counts twice
    }
    *V_out = V;
    *E_out = ne;
    return COME_OK;
}

extern "C" int come_walks_reference(const int64_t *rowptr, const int32_t *col, int64_t V,
                                    int n_streams, const int32_t *paths_per_stream,
                                    uint32_t *states, int path_length, double alpha,
                                    const int32_t *emit, int threads, int32_t *out) {
    if (V < 0 || n_streams < 0 || path_length < 0)
        return set_error(COME_E_INVALID, "V, n_streams and path_length must be >= 0");
    if (V > INT32_MAX) return set_error(COME_E_INVALID, "V must fit int32");
    if (n_streams == 0 || V == 0) return COME_OK;
    if (!rowptr || !col || !paths_per_stream || !states || !out)
        return set_error(COME_E_INVALID, "null pointer");
    std::vector<int64_t> first(n_streams + 1, 0);
    for (int s = 0; s < n_streams; ++s) {
        if (paths_per_stream[s] < 0) return set_error(COME_E_INVALID, "negative path count");
        if (states[s * 625 + 624] > 624) return set_error(COME_E_INVALID, "bad MT19937 state");
        first[s + 1] = first[s] + (int64_t)paths_per_stream[s] * V;
    }
    for (int64_t n = 0; n < V; ++n)
        if (rowptr[n + 1] < rowptr[n]) return set_error(COME_E_INVALID, "rowptr not monotone");
    auto run = [&](int s) {
        PyRandom r;
        r.set(states + s * 625);
        corpus_stream(rowptr, col, V, paths_per_stream[s], path_length, alpha, r, emit,
                      out + first[s] * (int64_t)path_length);
        r.get(states + s * 625);
    };
    int nt = threads < 1 ? 1 : threads;
    if (nt > n_streams) nt = n_streams;
    if (nt == 1) {
        for (int s = 0; s < n_streams; ++s) run(s);
        return COME_OK;
    }
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t)
        pool.emplace_back([&, t] {
            for (int s = t; s < n_streams; s += nt) run(s);
        });
    for (auto &th : pool) th.join();
    return COME_OK;
}

extern "C" int come_read_int_rows(const char *path, int64_t *rows, int64_t cap_rows, int width,
                                  int64_t *nrows_out, int *max_tokens_out) {
    if (!path || !nrows_out || !max_tokens_out)
        return set_error(COME_E_INVALID, "null pointer");
    if (rows && width <= 0) return set_error(COME_E_INVALID, "width must be > 0");
    Reader rd(path);
    if (!rd.f) return set_error(COME_E_INVALID, "cannot open %s", path);
    int64_t n = 0;
    int mx = 0;
    bool overflow = false;
    const bool ok = rd.lines([&](const std::vector<int64_t> &t) {
        if ((int)t.size() > mx) mx = (int)t.size();
        if (rows) {
            if (n >= cap_rows) {
                overflow = true;
                return;
            }
            int64_t *r = rows + n * (int64_t)width;
            const int k = (int)t.size() < width ? (int)t.size() : width;
            for (int i = 0; i < k; ++i) r[i] = t[i];
            for (int i = k; i < width; ++i) r[i] = -1;
        }
        ++n;
    });
    if (!ok) return set_error(COME_E_INVALID, "%s: malformed integer token", path);
    if (overflow) return set_error(COME_E_INVALID, "%s: more than %lld rows", path,
                                   (long long)cap_rows);
    *nrows_out = n;
    *max_tokens_out = mx;
    return COME_OK;
}

extern "C" int come_write_int_rows(const char *path, const int64_t *rows, int64_t nrows,
                                   int width, int append) {
    if (!path || (nrows > 0 && !rows) || width < 0)
        return set_error(COME_E_INVALID, "bad arguments");
    FILE *f = fopen(path, append ? "ab" : "wb");
    if (!f) return set_error(COME_E_INVALID, "cannot open %s", path);
    std::string buf;
    buf.reserve(1 << 20);
    char num[24];
    for (int64_t r = 0; r < nrows; ++r) {
        const int64_t *row = rows + r * (int64_t)width;
        for (int i = 0; i < width && row[i] >= 0; ++i) {  // a walk ends at its first -1
            if (i) buf.push_back(' ');
            auto res = std::to_chars(num, num + sizeof(num), row[i]);
            buf.append(num, res.ptr);
        }
        buf.push_back('\n');
        if (buf.size() > (1 << 20) - 4096) {
            fwrite(buf.data(), 1, buf.size(), f);
            buf.clear();
        }
    }
    fwrite(buf.data(), 1, buf.size(), f);
    const bool bad = ferror(f);
    fclose(f);
    return bad ? set_error(COME_E_INVALID, "write error on %s", path) : COME_OK;
}

extern "C" int come_format_f32(float x, char *out32) {
    if (!out32) return set_error(COME_E_INVALID, "null pointer");
    const int n = format_f32(x, out32);
    out32[n] = 0;
    return n;
}

extern "C" int come_save_embedding(const char *path, const float *emb, int64_t V, int d,
                                   int64_t first_id) {
    if (!path || (V > 0 && !emb) || d < 0) return set_error(COME_E_INVALID, "bad arguments");
    FILE *f = fopen(path, "wb");
    if (!f) return set_error(COME_E_INVALID, "cannot open %s", path);
    std::string buf;
    buf.reserve(1 << 20);
    char num[64];
    for (int64_t i = 0; i < V; ++i) {
        auto res = std::to_chars(num, num + sizeof(num), first_id + i);
        buf.append(num, res.ptr);
        buf.push_back('\t');
        for (int k = 0; k < d; ++k) {
            if (k) buf.push_back(' ');
            buf.append(num, format_f32(emb[i * (int64_t)d + k], num));
        }
        buf.push_back('\n');
        if (buf.size() > (1 << 20) - 65536) {
            fwrite(buf.data(), 1, buf.size(), f);
            buf.clear();
        }
    }
    fwrite(buf.data(), 1, buf.size(), f);
    const bool bad = ferror(f);
    fclose(f);
    return bad ? set_error(COME_E_INVALID, "write error on %s", path) : COME_OK;
}
