/*
 * oracle/rng.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C restatement of the two MT19937-based generators the reference's hot
 * path draws from.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library.
 *
 *  1. CPython `random` (3.10, Modules/_randommodule.c algorithm):
 *       - random.seed(int s)      -> init_by_array(key = 32-bit LE words of |s|)
 *       - random.random()         -> ((a>>5)*67108864.0 + (b>>6)) / 2^53
 *       - random.choices(pop, k)  -> pop[floor(random() * float(len(pop)))]
 *     Call sites: implicit.py:352 (train draw), implicit.py:370 (valid draw).
 *
 *  2. NumPy legacy RandomState (numpy/random/_mt19937 + distributions.c):
 *       - RandomState(s) / np.random.seed(s)  -> init_genrand(s)
 *       - randint(lo, hi) / choice(n, size)   -> masked rejection on 32-bit words
 *       - shuffle(x)                          -> Fisher-Yates with random_interval
 *     Call sites: mf_spotlight.py:36, implicit.py:146 (set_seed draw),
 *     implicit.py:262 (shuffle), spotlight/sampling.py:55-56 (pool builder).
 *
 * The state layout shared with the product and with Python's getstate() is
 * 624 uint32 words + one position word (625 total).
 */
#include <stdint.h>
#include <string.h>
#include <math.h>

#define MT_N 624
#define MT_M 397
#define MATRIX_A 0x9908b0dfU
#define UPPER_MASK 0x80000000U
#define LOWER_MASK 0x7fffffffU

/* state[0..623] = words, state[624] = position (index of the next word). */

static void mt_twist(uint32_t *mt) {
    static const uint32_t mag01[2] = {0x0U, MATRIX_A};
    uint32_t y;
    int kk;
    for (kk = 0; kk < MT_N - MT_M; kk++) {
        y = (mt[kk] & UPPER_MASK) | (mt[kk + 1] & LOWER_MASK);
        mt[kk] = mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 0x1U];
    }
    for (; kk < MT_N - 1; kk++) {
        y = (mt[kk] & UPPER_MASK) | (mt[kk + 1] & LOWER_MASK);
        mt[kk] = mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 0x1U];
    }
    y = (mt[MT_N - 1] & UPPER_MASK) | (mt[0] & LOWER_MASK);
    mt[MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 0x1U];
}

uint32_t orc_mt_next(uint32_t *state) {
    uint32_t y;
    if (state[MT_N] >= MT_N) {
        mt_twist(state);
        state[MT_N] = 0;
    }
    y = state[state[MT_N]++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}

/* init_genrand(s): NumPy legacy seeding, also the first half of init_by_array. */
void orc_mt_init_genrand(uint32_t *state, uint32_t s) {
    int i;
    state[0] = s;
    for (i = 1; i < MT_N; i++)
        state[i] = (1812433253U * (state[i - 1] ^ (state[i - 1] >> 30)) + (uint32_t)i);
    state[MT_N] = MT_N;
}

/* init_by_array: CPython random.seed(int) with key = |s| split in 32-bit words. */
void orc_mt_init_by_array(uint32_t *state, const uint32_t *key, int64_t key_length) {
    int64_t i, j, k;
    uint32_t *mt = state;
    orc_mt_init_genrand(state, 19650218U);
    i = 1; j = 0;
    k = (MT_N > key_length ? MT_N : key_length);
    for (; k; k--) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525U)) + key[j] + (uint32_t)j;
        i++; j++;
        if (i >= MT_N) { mt[0] = mt[MT_N - 1]; i = 1; }
        if (j >= key_length) j = 0;
    }
    for (k = MT_N - 1; k; k--) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941U)) - (uint32_t)i;
        i++;
        if (i >= MT_N) { mt[0] = mt[MT_N - 1]; i = 1; }
    }
    mt[0] = 0x80000000U;
    state[MT_N] = MT_N;
}

/* CPython random.random() */
double orc_py_random(uint32_t *state) {
    uint32_t a = orc_mt_next(state) >> 5, b = orc_mt_next(state) >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}

/* CPython random.choices(range(n), k=k) -> indices (implicit.py:352). */
void orc_py_choices(uint32_t *state, int64_t n, int64_t k, int64_t *out) {
    double fn = (double)n;
    for (int64_t t = 0; t < k; t++)
        out[t] = (int64_t)floor(orc_py_random(state) * fn);
}

/* NumPy: smallest all-ones mask >= max. */
static uint64_t gen_mask(uint64_t max) {
    uint64_t mask = max;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
    mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
    return mask;
}

/* NumPy legacy randint(low, high, size=cnt, dtype=int64) for high-low-1 < 2^32-1
 * (random_bounded_uint64_fill, masked branch). */
int orc_np_randint(uint32_t *state, int64_t low, int64_t high, int64_t cnt, int64_t *out) {
    uint64_t rng = (uint64_t)(high - low - 1);
    if (high <= low) return -1;
    if (rng >= 0xFFFFFFFFULL) return -2; /* not needed on the hot path */
    if (rng == 0) { for (int64_t t = 0; t < cnt; t++) out[t] = low; return 0; }
    uint64_t mask = gen_mask(rng);
    for (int64_t t = 0; t < cnt; t++) {
        uint64_t v;
        while ((v = (orc_mt_next(state) & mask)) > rng) {}
        out[t] = low + (int64_t)v;
    }
    return 0;
}

/* NumPy legacy random_interval(max) (32-bit branch). */
static uint64_t np_interval(uint32_t *state, uint64_t max) {
    uint64_t v, mask;
    if (max == 0) return 0;
    mask = gen_mask(max);
    while ((v = (orc_mt_next(state) & mask)) > max) {}
    return v;
}

/* NumPy legacy RandomState.shuffle on a 1-d int64 array (spotlight/torch_utils.py:38-55). */
void orc_np_shuffle_i64(uint32_t *state, int64_t *x, int64_t n) {
    for (int64_t i = n - 1; i >= 1; i--) {
        int64_t j = (int64_t)np_interval(state, (uint64_t)i);
        int64_t t = x[i]; x[i] = x[j]; x[j] = t;
    }
}
