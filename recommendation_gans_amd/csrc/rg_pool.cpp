// Negative-pool builder on the host (spotlight/sampling.py:46-70, get_negative_samples),
// continuing NumPy's legacy global generator exactly: the caller passes
// np.random.get_state()'s MT19937 key and position and stores the advanced state back.
//
//   users = np.random.choice(num_users, n); items = np.random.choice(num_items, n)
//     (legacy RandomState.choice -> randint(0, size) -> masked rejection on 32-bit draws)
//   for k in index order with rating(users[k], items[k]) == 1 (has_key, the summed CSR value):
//     pos = the user's nonzero columns, sorted; raw = randint(0, num_items - len(pos))
//     items[k] = raw + #{j : pos[j] - j <= raw}        (sampling.py:37-44, searchsorted 'right')
//
// The reference runs this as an n-iteration Python loop (8.1 M at ML-20M); here the
// draws are a tight loop and the has_key test a binary search in the user's CSR row.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "rg_common.h"

namespace {

struct LegacyMt {
    uint32_t *key;
    int pos;

    uint32_t next() {
        if (pos >= 624) {
            for (int i = 0; i < 624; ++i) {
                const uint32_t y = (key[i] & 0x80000000u) | (key[(i + 1) % 624] & 0x7fffffffu);
                key[i] = key[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            pos = 0;
        }
        uint32_t y = key[pos++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }

    // legacy randint(0, high) for high - 1 <= 0xFFFFFFFF: the smallest all-ones mask
    // covering high - 1, 32-bit draws rejected above it (no draw when high == 1)
    int64_t bounded(int64_t high) {
        const uint64_t rng = (uint64_t)(high - 1);
        if (rng == 0) return 0;
        if (rng == 0xFFFFFFFFull) return (int64_t)next();
        uint64_t mask = rng;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        uint64_t v;
        while ((v = (uint64_t)(next() & (uint32_t)mask)) > rng) {
        }
        return (int64_t)v;
    }
};

}  // namespace

using namespace rg;

extern "C" int rg_pool_build(uint32_t *mt_key, int32_t *mt_pos, int64_t n, int64_t num_users, int64_t num_items,
                             const int64_t *indptr, const int32_t *indices, const float *ratings, int64_t *out_users,
                             int64_t *out_items) {
    if (!mt_key || !mt_pos || !out_users || !out_items) return fail_arg("rg_pool_build: null argument");
    if (n < 0 || num_users < 1 || num_items < 1) return fail_arg("rg_pool_build: bad sizes");
    if (num_users - 1 > 0xFFFFFFFFll || num_items - 1 > 0xFFFFFFFFll) return fail_arg("rg_pool_build: range > 2^32");
    if (*mt_pos < 0 || *mt_pos > 624) return fail_arg("rg_pool_build: MT position must be in [0, 624]");
    if ((indptr == nullptr) != (indices == nullptr) || (indptr && !ratings))
        return fail_arg("rg_pool_build: give indptr, indices and ratings together");
    LegacyMt mt{mt_key, *mt_pos};
    for (int64_t k = 0; k < n; ++k) out_users[k] = mt.bounded(num_users);
    for (int64_t k = 0; k < n; ++k) out_items[k] = mt.bounded(num_items);
    if (indptr) {
        std::vector<int64_t> adj;
        for (int64_t k = 0; k < n; ++k) {
            const int64_t u = out_users[k], i = out_items[k];
            const int32_t *b = indices + indptr[u], *e = indices + indptr[u + 1];
            const int32_t *f = std::lower_bound(b, e, (int32_t)i);
            if (f == e || *f != i || ratings[indptr[u] + (f - b)] != 1.0f) continue;   // has_key
            adj.clear();
            for (const int32_t *c = b; c != e; ++c)                   // nonzero columns, sorted
                if (ratings[indptr[u] + (c - b)] != 0.0f) adj.push_back((int64_t)*c);
            const int64_t span = num_items - (int64_t)adj.size();
            if (span < 1) {
                *mt_pos = mt.pos;
                return fail_arg("rg_pool_build: a user with every item positive has no negative");
            }
            const int64_t raw = mt.bounded(span);
            for (size_t j = 0; j < adj.size(); ++j) adj[j] -= (int64_t)j;
            out_items[k] = raw + (int64_t)(std::upper_bound(adj.begin(), adj.end(), raw) - adj.begin());
        }
    }
    *mt_pos = mt.pos;
    return RG_OK;
}
