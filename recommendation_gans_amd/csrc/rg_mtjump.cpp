// MT19937 jump-ahead (host code): lets the device generate one step's words as
// several independent segments instead of one sequential 81,920-word walk.
//
// MT19937 is linear over GF(2).  With S_n = (top bit of x[n], x[n+1], ..., x[n+623])
// the 19,937-bit state whose next word is x[n+624], S_{n+1} = A S_n, and for any
// e >= 0
//     S_e = p_e(A) S_0 = XOR_{i : c_i = 1} S_i,   p_e(t) = t^e mod chi(t) = sum c_i t^i,
// chi the characteristic polynomial of A (degree 19,937).  S_i are just windows of
// the word stream x[] generated from S_0, so the state e words ahead is an XOR
// of windows of the first 19,937 + 624 words.  chi is obtained once by
// Berlekamp-Massey on one bit of the stream; p_e by square-and-multiply-by-t.
//
// Window form of a state: mt = x[D .. D+624), position 624 (the next word is
// x[D+624]).  From the XOR of windows with exponent D - 1 we get top(x[D-1]) and
// x[D .. D+622]; x[D+623] = x[D+396] ^ mix(x[D-1], x[D]) completes it.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "rg_common.h"

namespace rg {
namespace mtj {

constexpr int kN = 624, kM = 397;
constexpr int kDeg = 19937;
constexpr uint32_t kMatrixA = 0x9908b0dfU;

inline uint32_t mix(uint32_t hi_src, uint32_t lo_src) {
    const uint32_t y = (hi_src & 0x80000000U) | (lo_src & 0x7fffffffU);
    return (y >> 1) ^ ((y & 1U) ? kMatrixA : 0U);
}

// x[0 .. n) of the raw word stream whose next word is state[state[624]] (CPython layout)
void stream(const uint32_t *state, int64_t n, uint32_t *out) {
    const int64_t pos = state[kN];
    std::vector<uint32_t> x(kN + (size_t)(pos + n));
    std::memcpy(x.data(), state, kN * sizeof(uint32_t));
    for (size_t k = kN; k < x.size(); ++k) x[k] = x[k - (kN - kM)] ^ mix(x[k - kN], x[k - kN + 1]);
    std::memcpy(out, x.data() + pos, (size_t)n * sizeof(uint32_t));
}

using Poly = std::vector<uint64_t>;   // bit i = coefficient of t^i

inline int bit(const Poly &p, int64_t i) { return (int)((p[(size_t)(i >> 6)] >> (i & 63)) & 1U); }

// characteristic polynomial chi (degree kDeg, bit kDeg set) by Berlekamp-Massey
const Poly &charpoly() {
    static Poly chi;
    static std::once_flag once;
    std::call_once(once, [] {
        const int64_t n = 2 * (int64_t)kDeg + 64;
        std::vector<uint32_t> st(kN + 1);
        for (int i = 0; i < kN; ++i) st[i] = 0x9e3779b9U * (uint32_t)(i + 1) ^ (uint32_t)(i * 7919);
        st[kN] = kN;
        std::vector<uint32_t> w((size_t)n);
        stream(st.data(), n, w.data());
        // rev bit j = s[n-1-j]: the window s[k], s[k-1], ... is rev from bit n-1-k up
        const size_t nw = (size_t)(n / 64 + 2);
        Poly rev(nw + 1, 0);
        for (int64_t k = 0; k < n; ++k)
            if (w[(size_t)k] & 1U) rev[(size_t)((n - 1 - k) >> 6)] |= 1ULL << ((n - 1 - k) & 63);
        auto rev_word = [&](int64_t off, size_t j) {      // 64 bits of rev starting at bit off + 64 j
            const int64_t b = off + 64 * (int64_t)j;
            const size_t q = (size_t)(b >> 6);
            const int r = (int)(b & 63);
            return r ? (rev[q] >> r) | (rev[q + 1] << (64 - r)) : rev[q];
        };
        Poly C(nw, 0), B(nw, 0), T;
        C[0] = B[0] = 1;
        int64_t L = 0, m = 1;
        for (int64_t k = 0; k < n; ++k) {
            // d = parity(sum_{i=0..L} c_i s[k-i]), c_0 = 1
            uint64_t acc = 0;
            const size_t words = (size_t)(L / 64 + 1);
            for (size_t j = 0; j < words; ++j) {
                uint64_t c = C[j];
                if (j == words - 1 && ((L + 1) & 63)) c &= (1ULL << ((L + 1) & 63)) - 1;
                acc ^= c & rev_word(n - 1 - k, j);
            }
            if (!__builtin_parityll(acc)) { ++m; continue; }
            T = C;
            const size_t ws = (size_t)(m >> 6);
            const int bs = (int)(m & 63);
            for (size_t j = 0; j + ws < nw; ++j) {       // C += t^m B
                const uint64_t v = B[j];
                if (!v) continue;
                C[j + ws] ^= v << bs;
                if (bs && j + ws + 1 < nw) C[j + ws + 1] ^= v >> (64 - bs);
            }
            if (2 * L <= k) { L = k + 1 - L; B = T; m = 1; } else { ++m; }
        }
        if (L != kDeg) { chi.clear(); return; }
        // chi(t) = t^L C(1/t): coefficient of t^(L-i) is c_i
        chi.assign((size_t)(kDeg / 64 + 1), 0);
        for (int64_t i = 0; i <= L; ++i)
            if (bit(C, i)) chi[(size_t)((L - i) >> 6)] ^= 1ULL << ((L - i) & 63);
    });
    return chi;
}

// r <- r mod chi for r of degree < 2*kDeg
void reduce(Poly &r, const Poly &chi) {
    for (int64_t i = 2 * (int64_t)kDeg; i >= kDeg; --i) {
        if (!bit(r, i)) continue;
        const int64_t sh = i - kDeg;             // r ^= chi << sh
        const int64_t ws = sh >> 6, bs = sh & 63;
        for (size_t j = 0; j < chi.size(); ++j) {
            const uint64_t v = chi[j];
            if (!v) continue;
            r[(size_t)(j + ws)] ^= v << bs;
            if (bs && j + ws + 1 < r.size()) r[(size_t)(j + ws + 1)] ^= v >> (64 - bs);
        }
    }
}

// set bits of t^e mod chi, ascending
std::vector<int32_t> jump_terms(int64_t e) {
    static std::mutex mu;
    static std::map<int64_t, std::vector<int32_t>> cache;
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache.find(e);
        if (it != cache.end()) return it->second;
    }
    const Poly &chi = charpoly();
    std::vector<int32_t> terms;
    if (chi.empty()) return terms;
    const size_t nw = (size_t)(2 * kDeg / 64 + 2);
    Poly r(nw, 0);
    r[0] = 1;
    int top = 62;
    while (top > 0 && !((e >> top) & 1)) --top;
    for (int b = top; b >= 0; --b) {
        Poly sq(nw, 0);                          // squaring spreads bit i to 2i
        for (int64_t i = 0; i < kDeg; ++i)
            if (bit(r, i)) sq[(size_t)((2 * i) >> 6)] |= 1ULL << ((2 * i) & 63);
        reduce(sq, chi);
        r.swap(sq);
        if ((e >> b) & 1) {                      // r <- r * t
            for (size_t j = nw - 1; j > 0; --j) r[j] = (r[j] << 1) | (r[j - 1] >> 63);
            r[0] <<= 1;
            reduce(r, chi);
        }
    }
    for (int64_t i = 0; i < kDeg; ++i)
        if (bit(r, i)) terms.push_back((int32_t)i);
    std::lock_guard<std::mutex> g(mu);
    cache[e] = terms;
    return terms;
}

// window-form state at x-index D >= 1 from the stream x[0 .. kDeg + kN - 1) (host reference)
void window_from_stream(const uint32_t *x, int64_t D, uint32_t *mt) {
    const std::vector<int32_t> terms = jump_terms(D - 1);
    std::vector<uint32_t> acc(kN, 0);
    for (int32_t i : terms)
        for (int k = 0; k < kN; ++k) acc[k] ^= x[i + k];
    for (int j = 0; j < kN - 1; ++j) mt[j] = acc[j + 1];
    mt[kN - 1] = acc[kM] ^ mix(acc[0], acc[1]);
}

}  // namespace mtj

// a plan from explicit tail segments (start, length) past the head, and the state `words` ahead
static MtJumpPlan *plan_from(int64_t words, const std::vector<std::pair<int64_t, int64_t>> &segs) {
    using namespace mtj;
    if ((int)segs.size() > kMtMaxTail || mtj::charpoly().empty()) return nullptr;
    MtJumpPlan *p = new MtJumpPlan();
    p->words = words;
    p->head = kDeg + kN - 1;
    p->segs.n = (int)segs.size();
    std::vector<int32_t> terms, off{0};
    for (size_t j = 0; j <= segs.size(); ++j) {
        const int64_t start = j < segs.size() ? segs[j].first : words;
        if (j < segs.size()) {
            p->segs.start[j] = start;
            p->segs.len[j] = segs[j].second;
        }
        const std::vector<int32_t> t = jump_terms(start - kN - 1);   // window at D = start - 624
        terms.insert(terms.end(), t.begin(), t.end());
        off.push_back((int32_t)terms.size());
    }
    size_t longest = 0;
    for (size_t j = 0; j + 1 < off.size(); ++j) longest = std::max<size_t>(longest, (size_t)(off[j + 1] - off[j]));
    p->chunks = (int)((longest + 1000 - 1) / 1000);       // <= 1000 terms per block (LDS staging)
    if (p->chunks < 16) p->chunks = 16;
    hipError_t e = hipMalloc(&p->terms, terms.size() * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&p->term_off, off.size() * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&p->raw, (size_t)(p->segs.n + 1) * kN * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemcpy(p->terms, terms.data(), terms.size() * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->term_off, off.data(), off.size() * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        set_error(std::string("mt_jump_plan_create: ") + hipGetErrorString(e));
        mt_jump_plan_destroy(p);
        return nullptr;
    }
    return p;
}

MtJumpPlan *mt_jump_plan_create(int64_t words, int tail) {
    using namespace mtj;
    const int64_t head = kDeg + kN - 1;          // windows S_i, i < 19937, need x[0 .. 20560)
    // a jump alone (tail 0) needs only its window stream; tail segments at least one head apart
    if (words < (tail == 0 ? (int64_t)kN + 1 : 2 * head)) return nullptr;
    // tail segments of ~20k words: each walks about as long as the head does
#if RG_AB
    const char *env = getenv("RG_MT_TAIL");
#else
    const char *env = nullptr;
#endif
    int n = env ? atoi(env) : (int)((words - head + 19999) / 20000);
    n = n < 1 ? 1 : (n > kMtMaxTail ? kMtMaxTail : n);
    if (tail >= 0) n = tail > kMtMaxTail ? kMtMaxTail : tail;   // 0: the jump alone
    const int64_t rest = words - head, len = n > 0 ? (rest + n - 1) / n : 0;
    std::vector<std::pair<int64_t, int64_t>> segs;
    for (int j = 0; j < n; ++j) {
        const int64_t start = head + j * len;
        segs.emplace_back(start, std::min<int64_t>(len, words - start));
    }
    return plan_from(words, segs);
}

MtJumpPlan *mt_slice_plan_create(int64_t W, int64_t L, int64_t units) {
    using namespace mtj;
    const int64_t head = kDeg + kN - 1;
    if (L < head || W < L || units < 1) return nullptr;
    // the head walks the first slice's first `head` words; segment 0 the rest of it; segment k
    // unit k's slice; the state ends units * W ahead (this rank's slice of the next slot's first unit)
    std::vector<std::pair<int64_t, int64_t>> segs;
    if (L > head) segs.emplace_back(head, L - head);
    for (int64_t k = 1; k < units; ++k) segs.emplace_back(k * W, L);
    return plan_from(units * W, segs);
}

void mt_jump_plan_destroy(MtJumpPlan *p) {
    if (!p) return;
    if (p->terms) hipFree(p->terms);
    if (p->term_off) hipFree(p->term_off);
    if (p->raw) hipFree(p->raw);
    delete p;
}

}  // namespace rg

extern "C" int rg_mt_window_host(const uint32_t *state, int64_t D, uint32_t *window_out) {
    using namespace rg::mtj;
    if (!state || !window_out || D < 1) return rg::fail_arg("rg_mt_window_host: bad argument");
    if (charpoly().empty()) { rg::set_error("rg_mt_window_host: Berlekamp-Massey failed"); return RG_E_ARG; }
    std::vector<uint32_t> x((size_t)(kDeg + kN));
    stream(state, (int64_t)x.size(), x.data());
    window_from_stream(x.data(), D, window_out);
    return RG_OK;
}

extern "C" int rg_mt_window_to_cpython(const uint32_t *window, int32_t pos, uint32_t *state_out) {
    using namespace rg::mtj;
    if (!window || !state_out || pos < 1 || pos > kN) return rg::fail_arg("rg_mt_window_to_cpython: bad argument");
    // window = x[P-624 .. P); CPython block = x[P-pos .. P-pos+624), next word index pos
    std::vector<uint32_t> st(kN + 1);
    std::memcpy(st.data(), window, kN * sizeof(uint32_t));
    st[kN] = kN;
    std::vector<uint32_t> ahead((size_t)(kN - pos));
    if (!ahead.empty()) stream(st.data(), (int64_t)ahead.size(), ahead.data());
    std::memcpy(state_out, window + (kN - pos), (size_t)pos * sizeof(uint32_t));
    std::memcpy(state_out + pos, ahead.data(), ahead.size() * sizeof(uint32_t));
    state_out[kN] = (uint32_t)pos;
    return RG_OK;
}

extern "C" int rg_mt_advance_host(uint32_t *state, int64_t k) {
    using namespace rg::mtj;
    if (!state || k < 0 || state[kN] > (uint32_t)kN)
        return rg::fail_arg("rg_mt_advance_host: bad argument");
    const int64_t P = (int64_t)state[kN] + k;        // stream index of the next word, block 0 = state
    if (P <= kN) { state[kN] = (uint32_t)P; return RG_OK; }
    const int64_t fb = (P - 1) / kN;                 // block holding the last consumed word
    std::vector<uint32_t> x((size_t)(kN * (fb + 1)));
    std::memcpy(x.data(), state, kN * sizeof(uint32_t));
    for (size_t n = kN; n < x.size(); ++n) x[n] = x[n - (kN - kM)] ^ mix(x[n - kN], x[n - kN + 1]);
    std::memcpy(state, x.data() + kN * fb, kN * sizeof(uint32_t));
    state[kN] = (uint32_t)(P - kN * fb);
    return RG_OK;
}
