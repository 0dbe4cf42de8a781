/*
 * come_oracle_walks.c -- CPU restatement of libcome's device random-walk generator
 * (nodeembedding-to-communityembedding_amd/csrc/come_walk.hip, k_random_walks /
 * k_random_walks_staged), itself the distribution of the reference's __random_walk__
 * (/root/reference/utils/graph_utils.py:20-46): from the current node jump back to the walk's
 * start with probability alpha, else move to a uniformly chosen neighbour; a node without
 * neighbours ends the walk.
 *
 * TEST INFRASTRUCTURE ONLY (see come_oracle.c).  Used to pin the device walker bit for bit
 * (tests/test_gpu_walks.py) and to build tier-C inputs on a host without a GPU
 * (tests/tierc_inputs.py), so a sequential-oracle fixture and the GPU test see the same walks.
 *
 * Random stream: Philox-4x32-10 keyed by `seed` (k0 = low, k1 = high 32 bits), counter
 * (step t, walk_offset + walk low, high, 0); restart iff (r1 >> 8) < ceil(alpha * 2^24);
 * neighbour index = (r0 * degree) >> 32.
 */
#include <math.h>
#include <stdint.h>

static void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = lo1;
        c[2] = n2;
        c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

/* out [P x L] int32: walk w starts at starts[w] (position; outside [0, V) = an empty walk). */
int oracle_philox_walks(const int64_t *rowptr, const int32_t *col, int64_t V,
                        const int32_t *starts, int64_t P, int L, float alpha, uint64_t seed,
                        int64_t walk_offset, const int32_t *emit, int32_t *out) {
    const uint32_t thr = (uint32_t)ceil((double)alpha * 16777216.0);
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (int64_t w = 0; w < P; ++w) {
        int32_t *row = out + w * (int64_t)L;
        const int32_t start = starts[w];
        const uint64_t gw = (uint64_t)(walk_offset + w);
        int t = 0;
        if (start >= 0 && start < V) {
            int32_t cur = start;
            row[t++] = emit ? emit[cur] : cur;
            for (; t < L; ++t) {
                const int64_t b = rowptr[cur];
                const int64_t deg = rowptr[cur + 1] - b;
                if (deg <= 0) break;
                uint32_t c[4] = {(uint32_t)t, (uint32_t)gw, (uint32_t)(gw >> 32), 0u};
                philox4x32_10(c, k0, k1);
                if ((c[1] >> 8) >= thr)
                    cur = col[b + (int64_t)(((uint64_t)c[0] * (uint64_t)deg) >> 32)];
                else
                    cur = start;
                row[t] = emit ? emit[cur] : cur;
            }
        }
        for (; t < L; ++t) row[t] = -1;
    }
    return 0;
}
