// Host side of phase_mt.hip's jump-ahead: the GF(2) polynomials that move an MT19937 key block
// 624 * chunk_blocks * k words forward, so that chunk k of a long draw can start without generating
// everything before it.
//
// Viewed as one word sequence x[0..], MT19937 is linear over GF(2): x[n] = x[n-227] ^ mix(x[n-624],
// x[n-623]).  The step T: window (x[n..n+623]) -> (x[n+1..n+624]) has characteristic polynomial phi
// of degree 19937 on the 19937 bits that matter (the low 31 bits of a window's first word never
// reach the output), so T^D = r(T) with r = x^D mod phi, i.e. window(D) = XOR of window(i) over the
// set bits i of r (Cayley-Hamilton).  phi comes from Berlekamp-Massey on one output bit of the
// stream (its minimal polynomial is phi, which is irreducible); x^D mod phi by square-and-multiply
// with Barrett reduction on carry-less (PCLMUL) products.  A one-time check against a directly
// generated block guards the whole construction: on a mismatch the caller gets no table.
#include <immintrin.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <vector>

namespace tts {
namespace {

typedef unsigned long long u64;
constexpr int N = 624, MM = 397;
constexpr int DEG = 19937;
constexpr int PW = (DEG + 63) / 64;  // 312 words per polynomial of degree < DEG

// raw (untempered) words of the stream from init_genrand(5489)
std::vector<uint32_t> raw_stream(size_t n) {
    std::vector<uint32_t> x(std::max(n, (size_t)N));
    x[0] = 5489u;
    for (int i = 1; i < N; ++i) x[i] = 1812433253u * (x[i - 1] ^ (x[i - 1] >> 30)) + (uint32_t)i;
    for (size_t i = N; i < x.size(); ++i) {
        const uint32_t y = (x[i - N] & 0x80000000u) | (x[i - N + 1] & 0x7fffffffu);
        x[i] = x[i - N + MM] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    return x;
}

inline int bit(const std::vector<u64>& v, long long i) {
    return i < 0 || (size_t)(i >> 6) >= v.size() ? 0 : (int)((v[i >> 6] >> (i & 63)) & 1u);
}
// 64 bits of v from bit position p (positions outside v read as zero)
inline u64 get64(const std::vector<u64>& v, long long p) {
    const long long w = p >> 6;  // arithmetic shift: floor
    const int s = (int)(p & 63);
    auto at = [&](long long i) -> u64 { return i < 0 || (size_t)i >= v.size() ? 0ull : v[i]; };
    return s == 0 ? at(w) : (at(w) >> s) | (at(w + 1) << (64 - s));
}

// phi from Berlekamp-Massey on bit 0 of the stream; empty on failure
std::vector<u64> char_poly() {
    const int NB = 2 * DEG + 128;
    const std::vector<uint32_t> x = raw_stream(N + NB);
    const int CW = (NB / 2 + 256) / 64;
    std::vector<u64> rs((NB + 63) / 64 + 2, 0);  // reversed sequence: bit j = s[NB - 1 - j]
    for (int j = 0; j < NB; ++j)
        if (x[N + NB - 1 - j] & 1u) rs[j >> 6] |= 1ull << (j & 63);
    std::vector<u64> C(CW, 0), B(CW, 0), T;
    C[0] = B[0] = 1;
    int L = 0, m = 1;
    for (int n = 0; n < NB; ++n) {
        // discrepancy s[n] + sum_{i=1..L} C_i s[n-i] = parity(C & reversed window at NB-1-n)
        u64 acc = 0;
        const int wmax = std::min(CW - 1, (n + 1) >> 6);
        for (int w = 0; w <= wmax; ++w) acc ^= C[w] & get64(rs, (long long)(NB - 1 - n) + 64 * w);
        if (__builtin_popcountll(acc) & 1) {
            T = C;
            for (int w = 0; w < CW; ++w) C[w] ^= get64(B, 64ll * w - m);
            if (2 * L <= n) {
                L = n + 1 - L;
                B = T;
                m = 1;
            } else {
                ++m;
            }
        } else {
            ++m;
        }
    }
    if (L != DEG || !bit(C, L)) return {};
    std::vector<u64> phi(PW, 0);  // x^j coefficient = C_{L-j}; bit DEG lives in word 311
    for (int j = 0; j <= L; ++j)
        if (bit(C, L - j)) phi[j >> 6] |= 1ull << (j & 63);
    return phi;
}

__attribute__((target("pclmul,sse4.1"))) void pmul(const u64* a, int na, const u64* b, int nb, u64* r) {
    std::fill(r, r + na + nb, 0ull);
    for (int i = 0; i < na; ++i) {
        if (!a[i]) continue;
        const __m128i ai = _mm_set_epi64x(0, (long long)a[i]);
        for (int j = 0; j < nb; ++j) {
            const __m128i p = _mm_clmulepi64_si128(ai, _mm_set_epi64x(0, (long long)b[j]), 0x00);
            r[i + j] ^= (u64)_mm_cvtsi128_si64(p);
            r[i + j + 1] ^= (u64)_mm_extract_epi64(p, 1);
        }
    }
}

struct Field {
    std::vector<u64> phi, mu;  // phi (degree DEG), mu = floor(x^(2 DEG) / phi) (degree DEG)
    bool init() {
        phi = char_poly();
        if (phi.empty()) return false;
        // long division of x^(2 DEG) by phi, bit-serial (once)
        std::vector<u64> R(2 * PW + 2, 0);
        R[(2 * DEG) >> 6] |= 1ull << ((2 * DEG) & 63);
        mu.assign(PW, 0);
        for (int i = 2 * DEG; i >= DEG; --i) {
            if (!bit(R, i)) continue;
            const int sh = i - DEG;
            mu[sh >> 6] |= 1ull << (sh & 63);
            const int ws = sh >> 6, bs = sh & 63;
            for (int w = 0; w < PW; ++w) {
                R[w + ws] ^= phi[w] << bs;
                if (bs) R[w + ws + 1] ^= phi[w] >> (64 - bs);
            }
        }
        return true;
    }
    // v >> DEG, PW words
    static void shr_deg(const std::vector<u64>& v, u64* out) {
        for (int w = 0; w < PW; ++w) out[w] = get64(v, DEG + 64ll * w);
    }
    // a * b mod phi (Barrett); false if the reduction left bits at or above DEG (never expected)
    bool mulmod(const std::vector<u64>& a, const std::vector<u64>& b, std::vector<u64>& r) const {
        std::vector<u64> p(2 * PW), q1(PW), t(2 * PW), q(PW), qp(2 * PW);
        pmul(a.data(), PW, b.data(), PW, p.data());
        shr_deg(p, q1.data());
        pmul(q1.data(), PW, mu.data(), PW, t.data());
        shr_deg(t, q.data());
        pmul(q.data(), PW, phi.data(), PW, qp.data());
        for (int w = 0; w < 2 * PW; ++w) p[w] ^= qp[w];
        for (int w = DEG >> 6; w < 2 * PW; ++w) {
            const u64 hi = w == (DEG >> 6) ? p[w] >> (DEG & 63) : p[w];
            if (hi) return false;
        }
        r.assign(p.begin(), p.begin() + PW);
        return true;
    }
    bool xpow(u64 e, std::vector<u64>& r) const {
        r.assign(PW, 0);
        r[0] = 1;
        for (int b = 63; b >= 0; --b) {
            if (!mulmod(r, r, r)) return false;
            if ((e >> b) & 1u) {  // r * x
                u64 carry = 0;
                for (int w = 0; w < PW; ++w) {
                    const u64 nc = r[w] >> 63;
                    r[w] = (r[w] << 1) | carry;
                    carry = nc;
                }
                if (bit(r, DEG))
                    for (int w = 0; w < PW; ++w) r[w] ^= phi[w];
            }
        }
        return true;
    }
};

// the jumped block must equal the directly generated one (all bits but the dead low 31 of word 0)
bool self_check(const std::vector<u64>& c, int chunk_blocks) {
    const size_t D = (size_t)N * chunk_blocks;
    const std::vector<uint32_t> x = raw_stream(N + D + N + 1);
    for (int w = 0; w < N; ++w) {
        uint32_t acc = 0;
        for (int i = 0; i < DEG; ++i)
            if ((c[i >> 6] >> (i & 63)) & 1u) acc ^= x[N + i + w];
        const uint32_t want = x[N + D + w];
        if (w == 0 ? ((acc ^ want) & 0x80000000u) : (acc ^ want)) return false;
    }
    return true;
}

struct Table {
    std::mutex mu;
    int chunk_blocks = 0;
    bool failed = false;
    Field f;
    std::vector<u64> step;   // x^(624 chunk_blocks) mod phi
    std::vector<u64> polys;  // [n][PW]: x^(624 chunk_blocks k) mod phi, k = 1..n
};
Table& table() {
    static Table t;
    return t;
}

}  // namespace

// the first n jump polynomials (k = 1..n) of chunks of chunk_blocks key blocks, PW words each;
// false if the construction failed its check (the caller then draws without jumps)
bool mt_jump_polys(int chunk_blocks, int n, std::vector<unsigned long long>* out) {
    Table& t = table();
    std::lock_guard<std::mutex> lk(t.mu);
    if (t.failed) return false;
    if (t.chunk_blocks == 0) {
        t.chunk_blocks = chunk_blocks;
        if (!t.f.init() || !t.f.xpow((u64)N * chunk_blocks, t.step) || !self_check(t.step, chunk_blocks)) {
            t.failed = true;
            return false;
        }
        t.polys = t.step;
    }
    if (chunk_blocks != t.chunk_blocks) return false;
    std::vector<u64> r;
    while ((int)(t.polys.size() / PW) < n) {
        const std::vector<u64> last(t.polys.end() - PW, t.polys.end());
        if (!t.f.mulmod(last, t.step, r)) {
            t.failed = true;
            return false;
        }
        t.polys.insert(t.polys.end(), r.begin(), r.end());
    }
    out->assign(t.polys.begin(), t.polys.begin() + (size_t)n * PW);
    return true;
}

}  // namespace tts
