// mt_poly.cpp — host-side GF(2)[x] arithmetic for the MT19937 jump-ahead of
// the parallel torch-parity stream (mt_jump.hip).
//
// torch's CPU generator (at::mt19937; seed.py:6-11 torch.manual_seed, consumed
// by torch.bernoulli at compressors.py:310) is a linear recurrence on a
// 19937-bit state S_t: S_{t+1} = A S_t.  Its characteristic polynomial P (degree
// 19937, irreducible) annihilates every bit sequence of the stream, so by
// Cayley-Hamilton A^m = a(A) with a(x) = x^m mod P, and every raw word obeys
//     x_{m+j} = XOR_{k : a_k = 1} x_{k+j}          (1 <= j <= 624)
// — the 624-word window m positions ahead is a GF(2) convolution of the
// current stream with the coefficients of x^m mod P.  This file computes
//   * P, by Berlekamp-Massey on one bit of the raw stream (once per process);
//   * the jump table: for generator g >= 1 of the parallel stream, the
//     coefficients of x^(g*J - 1) mod P (J = GC_MT_JUMP_DRAWS), so that the
//     window starting at draw g*J is the convolution above with m = g*J - 1.
// The table depends only on g and J, never on the state: callers build it once
// and keep it on the device.
//
// Polynomials are little-endian arrays of 64-bit words (bit k of word w is the
// coefficient of x^(64w + k)).  Products use PCLMULQDQ when the host CPU has it
// (a portable carry-less multiply otherwise); reduction is Barrett's with
// mu = floor(x^(2D) / P), exact over GF(2).
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "gcodec.h"

namespace {

constexpr int D = 19937;               // degree of P
constexpr int NW = (D + 63) / 64;      // words of a reduced polynomial (312)
constexpr int NW2 = 2 * NW;            // words of a product
typedef std::vector<uint64_t> Poly;

// ---- carry-less 64 x 64 -> 128 ------------------------------------------------
__attribute__((target("pclmul,sse2"))) void clmul_hw(uint64_t a, uint64_t b, uint64_t *lo, uint64_t *hi)
{
    const __m128i r = _mm_clmulepi64_si128(_mm_set_epi64x(0, (long long)a), _mm_set_epi64x(0, (long long)b), 0);
    *lo = (uint64_t)_mm_cvtsi128_si64(r);
    *hi = (uint64_t)_mm_cvtsi128_si64(_mm_unpackhi_epi64(r, r));
}

void clmul_sw(uint64_t a, uint64_t b, uint64_t *lo, uint64_t *hi)
{
    uint64_t l = 0, h = 0;
    for (int i = 0; i < 64; ++i)
        if ((b >> i) & 1u) {
            l ^= a << i;
            if (i)
                h ^= a >> (64 - i);
        }
    *lo = l;
    *hi = h;
}

bool have_pclmul() { return __builtin_cpu_supports("pclmul"); }

__attribute__((target("pclmul,sse2"))) void mul_hw(const uint64_t *a, int na, const uint64_t *b, int nb, uint64_t *r)
{
    memset(r, 0, sizeof(uint64_t) * (na + nb));
    for (int i = 0; i < na; ++i) {
        if (!a[i])
            continue;
        const __m128i ai = _mm_set_epi64x(0, (long long)a[i]);
        for (int j = 0; j < nb; ++j) {
            const __m128i p = _mm_clmulepi64_si128(ai, _mm_set_epi64x(0, (long long)b[j]), 0);
            r[i + j] ^= (uint64_t)_mm_cvtsi128_si64(p);
            r[i + j + 1] ^= (uint64_t)_mm_cvtsi128_si64(_mm_unpackhi_epi64(p, p));
        }
    }
}

// r[na + nb] = a * b
void mul(const uint64_t *a, int na, const uint64_t *b, int nb, uint64_t *r)
{
    static const bool hw = have_pclmul();
    if (hw) {
        mul_hw(a, na, b, nb, r);
        return;
    }
    (void)clmul_hw;
    memset(r, 0, sizeof(uint64_t) * (na + nb));
    for (int i = 0; i < na; ++i)
        for (int j = 0; j < nb; ++j) {
            uint64_t lo, hi;
            clmul_sw(a[i], b[j], &lo, &hi);
            r[i + j] ^= lo;
            r[i + j + 1] ^= hi;
        }
}

// bits [s, s + 64*nout) of a (words na) into out (zero beyond a)
void shr_bits(const uint64_t *a, int na, int s, uint64_t *out, int nout)
{
    const int q = s >> 6, r = s & 63;
    for (int w = 0; w < nout; ++w) {
        const int i = q + w;
        const uint64_t lo = i < na ? a[i] : 0, hi = i + 1 < na ? a[i + 1] : 0;
        out[w] = r ? (lo >> r) | (hi << (64 - r)) : lo;
    }
}

void mask_low(uint64_t *a, int nwords, int bits)
{
    for (int w = 0; w < nwords; ++w) {
        const int lo = w * 64;
        if (lo >= bits)
            a[w] = 0;
        else if (lo + 64 > bits)
            a[w] &= (~0ull) >> (64 - (bits - lo));
    }
}

struct Field {
    Poly P;   // NW + 1 words (x^D term included)
    Poly mu;  // floor(x^(2D) / P), NW + 1 words
};

// ---- the MT19937 raw stream (untempered state words) ---------------------------
void mt_raw(uint32_t seed, int count, std::vector<uint32_t> &out)
{
    uint32_t mt[624];
    mt[0] = seed;
    for (int i = 1; i < 624; ++i)
        mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    out.resize(count);
    int k = 624;
    for (int t = 0; t < count; ++t) {
        if (k == 624) {
            for (int i = 0; i < 624; ++i) {
                const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
                mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            k = 0;
        }
        out[t] = mt[k++];
    }
}

// Berlekamp-Massey over GF(2) on bit 0 of the raw stream -> the connection
// polynomial C (C_0 = 1); P(x) = x^L C(1/x).  Word-parallel: the sequence is
// stored reversed so the discrepancy is an AND + parity over whole words.
Poly char_poly()
{
    const int N = 2 * D + 128;
    std::vector<uint32_t> raw;
    mt_raw(5489u, N, raw);
    const int NS = (N + 63) / 64 + 2;
    std::vector<uint64_t> rs(NS, 0);  // rs bit k = s[N - 1 - k]
    for (int n = 0; n < N; ++n)
        if (raw[n] & 1u) {
            const int k = N - 1 - n;
            rs[k >> 6] |= 1ull << (k & 63);
        }
    const int CW = NW + 4;
    std::vector<uint64_t> C(CW, 0), B(CW, 0), T(CW), sh(CW);
    C[0] = B[0] = 1;
    int L = 0, m = 1;
    std::vector<uint64_t> win(CW);
    for (int n = 0; n < N; ++n) {
        // d = parity(C[0..L] & s[n], s[n-1], ..., s[n-L]) = parity(C & rs[N-1-n ..])
        const int nw = (L >> 6) + 1;
        shr_bits(rs.data(), NS, N - 1 - n, win.data(), nw);
        uint64_t acc = 0;
        for (int w = 0; w < nw; ++w)
            acc ^= C[w] & win[w];
        const int d = __builtin_parityll(acc);
        if (!d) {
            ++m;
            continue;
        }
        // sh = B << m
        memset(sh.data(), 0, sizeof(uint64_t) * CW);
        const int q = m >> 6, r = m & 63;
        for (int w = CW - 1; w >= q; --w) {
            const uint64_t lo = B[w - q], lo2 = (w - q - 1 >= 0) ? B[w - q - 1] : 0;
            sh[w] = r ? (lo << r) | (lo2 >> (64 - r)) : lo;
        }
        if (2 * L <= n) {
            T = C;
            for (int w = 0; w < CW; ++w)
                C[w] ^= sh[w];
            L = n + 1 - L;
            B = T;
            m = 1;
        } else {
            for (int w = 0; w < CW; ++w)
                C[w] ^= sh[w];
            ++m;
        }
    }
    Poly P(NW + 1, 0);
    if (L != D)
        return Poly();  // cannot happen for MT19937 (P irreducible of degree D)
    for (int k = 0; k <= D; ++k)  // P_k = C_{L-k}
        if ((C[(D - k) >> 6] >> ((D - k) & 63)) & 1u)
            P[k >> 6] |= 1ull << (k & 63);
    return P;
}

// floor(x^(2D) / P) by long division (once)
Poly barrett_mu(const Poly &P)
{
    const int RW = (2 * D) / 64 + 2;
    std::vector<uint64_t> rem(RW, 0);
    rem[(2 * D) >> 6] |= 1ull << ((2 * D) & 63);
    // 64 shifted copies of P
    std::vector<std::vector<uint64_t>> Ps(64, std::vector<uint64_t>(NW + 2, 0));
    for (int s = 0; s < 64; ++s)
        for (int w = NW + 1; w >= 0; --w) {
            const uint64_t lo = w < (int)P.size() ? P[w] : 0, lo2 = (w >= 1 && w - 1 < (int)P.size()) ? P[w - 1] : 0;
            Ps[s][w] = s ? (lo << s) | (lo2 >> (64 - s)) : lo;
        }
    Poly mu(NW + 2, 0);
    for (int d = 2 * D; d >= D; --d) {
        if (!((rem[d >> 6] >> (d & 63)) & 1u))
            continue;
        const int sft = d - D;  // rem ^= P << sft
        mu[sft >> 6] |= 1ull << (sft & 63);
        const int q = sft >> 6, r = sft & 63;
        for (int w = 0; w < NW + 2 && q + w < RW; ++w)
            rem[q + w] ^= Ps[r][w];
    }
    mu.resize(NW + 1);
    return mu;
}

const Field &field()
{
    static Field f;
    static std::once_flag once;
    std::call_once(once, [] {
        f.P = char_poly();
        if (!f.P.empty())
            f.mu = barrett_mu(f.P);
    });
    return f;
}

// r (NW words, deg < D) = R mod P, R of NW2 words (deg < 2D)
void reduce(const Field &F, const uint64_t *R, uint64_t *r)
{
    uint64_t hi[NW + 1], q[NW2 + 2], t[NW2 + 2];
    shr_bits(R, NW2, D, hi, NW + 1);  // floor(R / x^D), deg < D
    mul(hi, NW + 1, F.mu.data(), NW + 1, q);
    uint64_t qq[NW + 1];
    shr_bits(q, 2 * (NW + 1), D, qq, NW + 1);  // quotient, deg < D
    mul(qq, NW + 1, F.P.data(), NW + 1, t);
    for (int w = 0; w < NW; ++w)
        r[w] = R[w] ^ t[w];
    mask_low(r, NW, D);
}

void mulmod(const Field &F, const uint64_t *a, const uint64_t *b, uint64_t *r)
{
    uint64_t p[NW2];
    mul(a, NW, b, NW, p);
    reduce(F, p, r);
}

// x^e mod P
void xpow(const Field &F, uint64_t e, uint64_t *r)
{
    memset(r, 0, sizeof(uint64_t) * NW);
    r[0] = 1;
    int top = 63;
    while (top >= 0 && !((e >> top) & 1u))
        --top;
    uint64_t p[NW2];
    for (int b = top; b >= 0; --b) {
        mul(r, NW, r, NW, p);  // square
        reduce(F, p, r);
        if ((e >> b) & 1u) {  // * x: shift by one, fold x^D
            uint64_t carry = 0;
            for (int w = 0; w < NW; ++w) {
                const uint64_t v = r[w];
                r[w] = (v << 1) | carry;
                carry = v >> 63;
            }
            if ((r[D >> 6] >> (D & 63)) & 1u) {
                for (int w = 0; w < NW; ++w)
                    r[w] ^= F.P[w];
            }
            mask_low(r, NW, D);
        }
    }
}

}  // namespace

namespace gc {
int fail(int code, const char *fmt, ...);
}

extern "C" {

int gc_mt19937_jump_table_j(uint64_t J, uint64_t first, uint64_t count, uint32_t *table)
{
    if (count && !table)
        return gc::fail(GC_EINVAL, "gc_mt19937_jump_table: null table");
    if (J == 0 || J % 624 != 0)
        return gc::fail(GC_EINVAL, "gc_mt19937_jump_table: J = %llu is not a positive multiple of 624",
                        (unsigned long long)J);
    if (first < 1)
        return gc::fail(GC_EINVAL, "gc_mt19937_jump_table: generators start at 1 (generator 0 is the state itself)");
    if (!count)
        return GC_OK;
    const Field &F = field();
    if (F.P.empty())
        return gc::fail(GC_EINVAL, "gc_mt19937_jump_table: characteristic polynomial not found");
    uint64_t cur[NW], RJ[NW], nxt[NW];
    xpow(F, first * J - 1, cur);
    if (count > 1)
        xpow(F, J, RJ);
    for (uint64_t i = 0; i < count; ++i) {
        memcpy(table + i * 624, cur, sizeof(uint64_t) * NW);  // little-endian: 312 x u64 = 624 x u32
        if (i + 1 < count) {
            mulmod(F, cur, RJ, nxt);
            memcpy(cur, nxt, sizeof(cur));
        }
    }
    return GC_OK;
}

int gc_mt19937_jump_table(uint64_t first, uint64_t count, uint32_t *table)
{
    return gc_mt19937_jump_table_j(GC_MT_JUMP_DRAWS, first, count, table);
}

}  // extern "C"
