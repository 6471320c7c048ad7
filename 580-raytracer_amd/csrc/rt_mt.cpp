// rt_mt.cpp — block jump-ahead of std::mt19937 (see rt_mt.h).
#include "rt_mt.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <thread>

namespace rt580 {
namespace {

constexpr uint32_t kUpper = 0x80000000u, kLower = 0x7fffffffu, kMatrixA = 0x9908b0dfu;
constexpr int kDeg = 19937;  // degree of phi (the engine's period is 2^19937 - 1)

// y_{n+624} from y_n, y_{n+1}, y_{n+397} (the twist, libstdc++ random.tcc / MSVC <random>)
inline uint32_t twist(uint32_t yn, uint32_t yn1, uint32_t yn397) {
    const uint32_t y = (yn & kUpper) | (yn1 & kLower);
    return yn397 ^ (y >> 1) ^ ((y & 1u) ? kMatrixA : 0u);
}

inline uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// GF(2) polynomials: bit i of the word array = coefficient of x^i.
using Poly = std::vector<uint64_t>;
inline bool bit(const Poly& p, int i) { return (p[(size_t)i >> 6] >> (i & 63)) & 1u; }
inline void flip(Poly& p, int i) { p[(size_t)i >> 6] ^= 1ull << (i & 63); }

int degree(const Poly& p) {
    for (int w = (int)p.size() - 1; w >= 0; w--)
        if (p[(size_t)w]) return w * 64 + 63 - __builtin_clzll(p[(size_t)w]);
    return -1;
}

// p ^= q << s (p must hold the result)
void xor_shifted(Poly& p, const Poly& q, int s) {
    const int ws = s >> 6, bs = s & 63;
    for (size_t k = 0; k < q.size(); k++) {
        if (!q[k]) continue;
        p[k + (size_t)ws] ^= q[k] << bs;
        if (bs && k + (size_t)ws + 1 < p.size()) p[k + (size_t)ws + 1] ^= q[k] >> (64 - bs);
    }
}

// phi by Berlekamp-Massey on bit 0 of the first 2 * 19937 + 64 draws of the engine
// (a linear functional of the state: its minimal polynomial is phi).
Poly char_poly() {
    const int n = 2 * kDeg + 64;
    std::mt19937 g(5489u);  // any seed: phi is the engine's, not the stream's
    // the sequence reversed, as words: bit t of R = s[n - 1 - t], so that
    // s[i - j] for j = 0..L is bits (n - 1 - i) + j of R
    Poly R((size_t)n / 64 + 3, 0);
    for (int i = 0; i < n; i++)
        if (g() & 1u) flip(R, n - 1 - i);
    const size_t words = (size_t)(kDeg + 2 + 64) / 64 + 2;
    Poly C(words, 0), B(words, 0), T;
    C[0] = B[0] = 1;
    int L = 0, m = 1;
    for (int i = 0; i < n; i++) {
        // discrepancy: s[i] + sum_j C_j s[i - j] = parity of C & (R >> (n - 1 - i))
        const int off = n - 1 - i, ow = off >> 6, ob = off & 63;
        uint64_t acc = 0;
        for (int w = 0; w <= (L >> 6); w++) {
            uint64_t r = R[(size_t)(ow + w)] >> ob;
            if (ob) r |= R[(size_t)(ow + w + 1)] << (64 - ob);
            if (w == (L >> 6)) r &= (L & 63) == 63 ? ~0ull : ((2ull << (L & 63)) - 1);  // bits 0..L only
            acc ^= C[(size_t)w] & r;
        }
        const int d = __builtin_popcountll(acc) & 1;
        if (!d) {
            m++;
        } else if (2 * L <= i) {
            T = C;
            xor_shifted(C, B, m);
            L = i + 1 - L;
            B = T;
            m = 1;
        } else {
            xor_shifted(C, B, m);
            m++;
        }
    }
    // phi(x) = x^L C(1/x)
    Poly phi((size_t)(L + 64) / 64 + 1, 0);
    for (int j = 0; j <= L; j++)
        if (bit(C, j)) flip(phi, L - j);
    return L == kDeg ? phi : Poly();
}

const Poly& phi() {
    static const Poly p = char_poly();
    return p;
}

// p mod phi for deg p < 2 * kDeg (in place; p keeps its size)
void reduce(Poly& p) {
    const Poly& f = phi();
    for (int k = degree(p); k >= kDeg; k = degree(p)) xor_shifted(p, f, k - kDeg);
}

// (p * p) mod phi
Poly square_mod(const Poly& p) {
    Poly r(2 * p.size() + 1, 0);
    for (size_t k = 0; k < p.size(); k++) {
        uint64_t w = p[k];
        for (int half = 0; half < 2; half++) {
            uint64_t v = (uint32_t)(w >> (32 * half));
            // spread the 32 bits of v to the even bits of a 64-bit word
            v = (v | (v << 16)) & 0x0000ffff0000ffffull;
            v = (v | (v << 8)) & 0x00ff00ff00ff00ffull;
            v = (v | (v << 4)) & 0x0f0f0f0f0f0f0f0full;
            v = (v | (v << 2)) & 0x3333333333333333ull;
            v = (v | (v << 1)) & 0x5555555555555555ull;
            r[2 * k + (size_t)half] = v;
        }
    }
    reduce(r);
    r.resize(p.size());
    return r;
}

// (p * x) mod phi
void times_x_mod(Poly& p) {
    uint64_t carry = 0;
    for (uint64_t& w : p) {
        const uint64_t nc = w >> 63;
        w = (w << 1) | carry;
        carry = nc;
    }
    if (bit(p, kDeg)) xor_shifted(p, phi(), 0);
}

// x^e mod phi
Poly x_pow_mod(uint64_t e) {
    Poly r((size_t)kDeg / 64 + 2, 0);
    r[0] = 1;
    for (int b = 63; b >= 0; b--) {
        if (degree(r) > 0 || r[0] != 1) r = square_mod(r);
        if ((e >> b) & 1u) times_x_mod(r);
    }
    return r;
}

// A h(A) W by Horner's rule (A: one twist step of the window).
MtWindow horner_apply(const Poly& h, const MtWindow& w) {
    uint32_t acc[kMtN];
    std::memset(acc, 0, sizeof acc);
    int head = 0;  // acc[head] holds the window's first word
    auto step = [&]() {
        const uint32_t y = twist(acc[head], acc[(head + 1) % kMtN], acc[(head + 397) % kMtN]);
        acc[head] = y;
        head = head + 1 == kMtN ? 0 : head + 1;
    };
    for (int i = degree(h); i >= 0; i--) {
        step();
        if (bit(h, i)) {
            const int a = kMtN - head;  // acc[head + k] ^= w[k], in two runs
            for (int k = 0; k < a; k++) acc[head + k] ^= w.y[k];
            for (int k = a; k < kMtN; k++) acc[k - a] ^= w.y[k];
        }
    }
    step();
    MtWindow out;
    for (int k = 0; k < kMtN; k++) out.y[k] = acc[(head + k) % kMtN];
    return out;
}

struct Cache {
    uint64_t k0 = 0;          // block index of w[0]
    std::vector<MtWindow> w;  // W_{(k0 + i) kMtBlock}, i = 0, 1, ...
};

}  // namespace

MtWindow mt_seed_window(uint32_t seed) {
    MtWindow w;
    w.y[0] = seed;
    for (int i = 1; i < kMtN; i++) w.y[i] = 1812433253u * (w.y[i - 1] ^ (w.y[i - 1] >> 30)) + (uint32_t)i;
    return w;
}

MtWindow mt_jump(const MtWindow& w, uint64_t J) {
    if (J == 0) return w;
    return horner_apply(x_pow_mod(J - 1), w);
}

void mt_draws(const MtWindow& w, uint64_t count, uint32_t* out) {
    uint32_t r[kMtN];
    std::memcpy(r, w.y, sizeof r);
    int head = 0;
    for (uint64_t k = 0; k < count; k++) {
        const uint32_t y = twist(r[head], r[(head + 1) % kMtN], r[(head + 397) % kMtN]);
        r[head] = y;
        head = head + 1 == kMtN ? 0 : head + 1;
        out[k] = temper(y);
    }
}

bool mt_checkpoints(uint32_t seed, uint64_t k0, uint64_t k1, std::vector<MtWindow>& out) {
    out.clear();
    if (k1 < k0) return false;
    // Berlekamp-Massey found no degree-19937 polynomial (cannot happen for the
    // engine; a wrong phi would make reduce() loop forever): report, not hang
    if (phi().empty()) return false;
    static std::mutex mu;
    static std::map<uint32_t, Cache> caches;
    std::lock_guard<std::mutex> lock(mu);
    Cache& c = caches[seed];
    // a request that does not start inside (or right after) the cached run
    // starts a new run with ONE jump to k0 (not every window from 0)
    if (c.w.empty() || k0 < c.k0 || k0 > c.k0 + c.w.size()) {
        c.k0 = k0;
        c.w.assign(1, mt_jump(mt_seed_window(seed), k0 * kMtBlock));
    }
    const uint64_t have = c.k0 + c.w.size();  // absolute block index one past the run
    if (k1 > have) {
        static const Poly hb = x_pow_mod(kMtBlock - 1);  // one block: W -> A hb(A) W
        c.w.resize((size_t)(k1 - c.k0));
        const uint64_t todo = k1 - have;
        // threads: the host's share ($OMP_NUM_THREADS on the GPU pool), at most 16
        unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        if (const char* e = std::getenv("OMP_NUM_THREADS")) hw = std::max(1, std::atoi(e));
        const unsigned nt = (unsigned)std::min<uint64_t>(std::min(hw, 16u), todo);
        const MtWindow last = c.w[(size_t)(have - 1 - c.k0)];
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; t++)
            th.emplace_back([&, t] {
                const uint64_t a = have + todo * t / nt, b = have + todo * (t + 1) / nt;
                if (a >= b) return;
                // a thread's first window by one long jump from the run's last
                // window, then block by block
                MtWindow cur = mt_jump(last, (a - (have - 1)) * kMtBlock);
                c.w[(size_t)(a - c.k0)] = cur;
                for (uint64_t k = a + 1; k < b; k++) {
                    cur = horner_apply(hb, cur);
                    c.w[(size_t)(k - c.k0)] = cur;
                }
            });
        for (auto& x : th) x.join();
    }
    out.assign(c.w.begin() + (ptrdiff_t)(k0 - c.k0), c.w.begin() + (ptrdiff_t)(k1 - c.k0));
    return true;
}

}  // namespace rt580
