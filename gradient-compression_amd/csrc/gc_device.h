// gc_device.h — device-side building blocks shared by the gcodec kernels.
//
// gfx950 (CDNA4) only: 64-lane waves, fp32 denormals preserved (no FTZ), no
// FMA contraction (built with -ffp-contract=off), IEEE correctly-rounded fp32
// division (hipcc default for HIP device code).  The per-element arithmetic is
// the reference's, operation for operation (compressors.py:299-316).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gc {

constexpr int kBlock = 256;  // 4 waves of 64

// ---------------------------------------------------------------------------
// Random draws.  KIND 0 = Philox4x32-10 (counter-based, launch-invariant),
// KIND 1 = caller stream (level-major: stream[level*n + i]).
// ---------------------------------------------------------------------------
struct RngArgs {
    uint64_t seed;
    uint64_t offset;
    const uint32_t *stream;
    uint64_t n;  // elements per level in the stream
};

// Philox4x32-10 round function; IMPL selects the instruction mix only (the
// outputs are identical): 0 = 64-bit products + 2-input XORs, 1 = 64-bit
// products (v_mad_u64_u32) + 3-input XOR (v_bitop3_b32 0x96), 2 = 32-bit
// mul_hi / mul_lo + v_bitop3_b32.
#ifndef GC_PHILOX_IMPL
#define GC_PHILOX_IMPL 1
#endif

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

template <int IMPL = GC_PHILOX_IMPL>
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1)
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, lo0, hi1, lo1;
        if constexpr (IMPL == 2) {
            hi0 = __umulhi(0xD2511F53u, c.x);
            lo0 = 0xD2511F53u * c.x;
            hi1 = __umulhi(0xCD9E8D57u, c.z);
            lo1 = 0xCD9E8D57u * c.z;
        } else {
            const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
            const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
            hi0 = (uint32_t)(p0 >> 32);
            lo0 = (uint32_t)p0;
            hi1 = (uint32_t)(p1 >> 32);
            lo1 = (uint32_t)p1;
        }
        uint4 o;
        if constexpr (IMPL == 0) {
            o.x = hi1 ^ c.y ^ k0;
            o.z = hi0 ^ c.w ^ k1;
        } else {
            o.x = xor3(hi1, c.y, k0);
            o.z = xor3(hi0, c.w, k1);
        }
        o.y = lo1;
        o.w = lo0;
        c = o;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// Philox4x32-10 of the counter (g, y, z, w) when only g varies across the
// wave and y, z, w and the key are uniform (the draws4 counter: quad index,
// level, call offset): the same outputs as philox4x32_10, with the uniform
// halves of rounds 1-3 kept on the scalar unit and every XOR of two uniform
// terms folded before it meets a per-lane one (round 1: one product and one
// XOR per lane; round 2: one product, two XORs; round 3: the full round with
// one 2-input XOR).  About 3 VALU instructions fewer per block than the
// generic rounds, which leave the compiler 3-input XORs of two SGPRs (a
// v_mov each, the constant-bus limit) and no pre-folding.
__device__ __forceinline__ uint4 philox4x32_10_g(uint32_t g, uint32_t y, uint32_t z, uint32_t w, uint32_t k0,
                                                 uint32_t k1)
{
    constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, C0 = 0x9E3779B9u, C1 = 0xBB67AE85u;
    // the folded uniform terms pass through an empty asm on an SGPR, so the
    // compiler cannot re-associate them back into two per-lane XORs
    auto fold = [](uint32_t v) {
        asm("" : "+s"(v));
        return v;
    };
    // round 1: p1 = M1 z is uniform
    const uint64_t a0 = (uint64_t)M0 * g;
    const uint64_t a1 = (uint64_t)M1 * z;
    const uint32_t ux = (uint32_t)(a1 >> 32) ^ y ^ k0;  // uniform
    const uint32_t uy = (uint32_t)a1;                   // uniform
    const uint32_t vz = (uint32_t)(a0 >> 32) ^ fold(w ^ k1);
    const uint32_t vw = (uint32_t)a0;
    // round 2: p0 = M0 ux is uniform
    const uint64_t b0 = (uint64_t)M0 * ux;
    const uint64_t b1 = (uint64_t)M1 * vz;
    uint4 c;
    c.x = (uint32_t)(b1 >> 32) ^ fold(uy ^ (k0 + C0));
    c.y = (uint32_t)b1;
    c.z = vw ^ fold((uint32_t)(b0 >> 32) ^ (k1 + C1));
    const uint32_t uw = (uint32_t)b0;  // uniform
    // round 3: c.w uniform
    {
        const uint64_t p0 = (uint64_t)M0 * c.x;
        const uint64_t p1 = (uint64_t)M1 * c.z;
        uint4 o;
        o.x = xor3((uint32_t)(p1 >> 32), c.y, k0 + 2u * C0);
        o.z = (uint32_t)(p0 >> 32) ^ fold(uw ^ (k1 + 2u * C1));
        o.y = (uint32_t)p1;
        o.w = (uint32_t)p0;
        c = o;
    }
    k0 += 3u * C0;
    k1 += 3u * C1;
#pragma unroll
    for (int r = 3; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)M0 * c.x;
        const uint64_t p1 = (uint64_t)M1 * c.z;
        uint4 o;
        o.x = xor3((uint32_t)(p1 >> 32), c.y, k0);
        o.z = xor3((uint32_t)(p0 >> 32), c.w, k1);
        o.y = (uint32_t)p1;
        o.w = (uint32_t)p0;
        c = o;
        k0 += C0;
        k1 += C1;
    }
    return c;
}

// ---------------------------------------------------------------------------
// KIND 2: the dense two-level Philox stream of the 2-level multi-scale /
// two-scale codecs (levels 0 and 1 only).  The 16 draws of elements
// 8g..8g+7 at both levels are 24-bit fields of 3 Philox4x32-10 blocks,
// counter (lo32 g, (hi16 g) | b << 16, lo32 offset, hi32 offset), b = 0, 1, 2,
// key = seed: with w_0..w_11 the blocks' words in order, draw (level l,
// element 8g + e) is bits 24 (8 l + e) .. +23 of w_0 | w_1 << 32 | ... .  The
// rounding reads only the low 24 bits of a draw (r & 0xFFFFFF), so 16 draws
// cost 3 blocks instead of 4 (ms2_octet: 1.5 blocks per 4 elements and level
// pair).  Quad h (elements 8g + 4h ..) at level l is the 3 words from
// w_(6l + 3h): draws (a, alignbit(b, a, 24), alignbit(c, b, 16), c >> 8)
// (the top byte of the first three is not part of the draw).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint4 ms2_quad(uint32_t a, uint32_t b, uint32_t c)
{
    return make_uint4(a, __builtin_amdgcn_alignbit(b, a, 24), __builtin_amdgcn_alignbit(c, b, 16), c >> 8);
}

template <int IMPL = GC_PHILOX_IMPL>
__device__ __forceinline__ uint4 ms2_block(const RngArgs &r, uint64_t g, uint32_t b)
{
    if constexpr (IMPL == 1) {
        if (g < (1ull << 32))
            return philox4x32_10_g((uint32_t)g, b << 16, (uint32_t)r.offset, (uint32_t)(r.offset >> 32),
                                   (uint32_t)r.seed, (uint32_t)(r.seed >> 32));
    }
    uint4 c;
    c.x = (uint32_t)g;
    c.y = ((uint32_t)(g >> 32) & 0xffffu) | (b << 16);
    c.z = (uint32_t)r.offset;
    c.w = (uint32_t)(r.offset >> 32);
    return philox4x32_10<IMPL>(c, (uint32_t)r.seed, (uint32_t)(r.seed >> 32));
}

// both levels' draws of the 8 elements 8g..8g+7: d[l][h] = quad h at level l
__device__ __forceinline__ void ms2_octet(const RngArgs &r, uint64_t g, uint4 (&d)[2][2])
{
    const uint4 b0 = ms2_block(r, g, 0), b1 = ms2_block(r, g, 1), b2 = ms2_block(r, g, 2);
    d[0][0] = ms2_quad(b0.x, b0.y, b0.z);
    d[0][1] = ms2_quad(b0.w, b1.x, b1.y);
    d[1][0] = ms2_quad(b1.z, b1.w, b2.x);
    d[1][1] = ms2_quad(b2.y, b2.z, b2.w);
}

// one level's draws of the 8 elements (2 blocks: 0 and 1, or 1 and 2)
__device__ __forceinline__ void ms2_octet_level(const RngArgs &r, uint64_t g, uint32_t level, uint4 (&d)[2])
{
    if (level == 0) {
        const uint4 b0 = ms2_block(r, g, 0), b1 = ms2_block(r, g, 1);
        d[0] = ms2_quad(b0.x, b0.y, b0.z);
        d[1] = ms2_quad(b0.w, b1.x, b1.y);
    } else {
        const uint4 b1 = ms2_block(r, g, 1), b2 = ms2_block(r, g, 2);
        d[0] = ms2_quad(b1.z, b1.w, b2.x);
        d[1] = ms2_quad(b2.y, b2.z, b2.w);
    }
}

// ---------------------------------------------------------------------------
// KIND 4 / 5: split-plane draws (GC_RNG_SPLIT8 / GC_RNG_SPLIT16).  Of each
// draw only the 24 bits the rounding reads are kept, cut in two planes: the
// HI plane holds bits 24-HB .. 23 (HB = 8: one byte per draw, 16: two), padded
// to 16 bytes, then the LO plane holds bits 0 .. 23-HB.  The encode decides
// [r24 < F] from the HI plane alone unless HI equals the top HB bits of F-1
// (about 1 draw in 2^HB), and reads the LO plane only for those quads
// (enc_tile_int_split).  One level; n = the call's draws.
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t split_hpad(uint64_t n, uint32_t hb)
{
    return (n * (hb / 8) + 15) & ~(uint64_t)15;
}
__host__ __device__ __forceinline__ uint64_t split_bytes(uint64_t n, uint32_t hb)
{
    return split_hpad(n, hb) + ((n * ((24 - hb) / 8) + 15) & ~(uint64_t)15);
}

// the full 24-bit draws of quad i0 .. i0+3 (left of them in range) from both planes
template <uint32_t HB>
__device__ __forceinline__ uint4 split_quad(const RngArgs &r, uint64_t i0, uint64_t left)
{
    const uint8_t *h = reinterpret_cast<const uint8_t *>(r.stream);
    const uint8_t *l = h + split_hpad(r.n, HB);
    uint4 d = make_uint4(0u, 0u, 0u, 0u);
    uint32_t *dp = &d.x;
    if (left >= 4) {
        if constexpr (HB == 8) {
            const uint32_t hq = *reinterpret_cast<const uint32_t *>(h + i0);
            const uint2 lq = *reinterpret_cast<const uint2 *>(l + 2 * i0);
            d.x = (hq & 0xFFu) << 16 | (lq.x & 0xFFFFu);
            d.y = ((hq >> 8) & 0xFFu) << 16 | (lq.x >> 16);
            d.z = ((hq >> 16) & 0xFFu) << 16 | (lq.y & 0xFFFFu);
            d.w = (hq >> 24) << 16 | (lq.y >> 16);
        } else {
            const uint2 hq = *reinterpret_cast<const uint2 *>(h + 2 * i0);
            const uint32_t lq = *reinterpret_cast<const uint32_t *>(l + i0);
            d.x = (hq.x & 0xFFFFu) << 8 | (lq & 0xFFu);
            d.y = (hq.x >> 16) << 8 | ((lq >> 8) & 0xFFu);
            d.z = (hq.y & 0xFFFFu) << 8 | ((lq >> 16) & 0xFFu);
            d.w = (hq.y >> 16) << 8 | (lq >> 24);
        }
        return d;
    }
    for (uint32_t e = 0; e < (uint32_t)min(left, (uint64_t)4); ++e) {
        const uint64_t i = i0 + e;
        if constexpr (HB == 8)
            dp[e] = (uint32_t)h[i] << 16 | (uint32_t)reinterpret_cast<const uint16_t *>(l)[i];
        else
            dp[e] = (uint32_t)reinterpret_cast<const uint16_t *>(h)[i] << 8 | (uint32_t)l[i];
    }
    return d;
}

// Four draws for elements i0..i0+3 (i0 % 4 == 0) at scale `level`.
// KIND 0: Philox, one block per quad and level; 1: a draw stream; 2: the
// dense two-level Philox stream above (one or two blocks per quad and level:
// the generic kernels' path; the octet kernels of ms_fast.h share blocks);
// 3: a draw stream packed to 24 bits (GC_RNG_STREAM24); 4 / 5: split-plane
// draws (both planes read: the generic paths; one level).
template <int KIND, int IMPL = GC_PHILOX_IMPL>
__device__ __forceinline__ uint4 draws4(const RngArgs &r, uint32_t level, uint64_t i0)
{
    if constexpr (KIND == 4 || KIND == 5) {
        return split_quad<KIND == 4 ? 8u : 16u>(r, i0, i0 < r.n ? r.n - i0 : 0);
    } else if constexpr (KIND == 2) {
        // block numbers stay wave-uniform (philox4x32_10_g keeps y on the
        // scalar unit); the quad half h = bit 2 of i0 is per lane
        const uint64_t g = i0 >> 3;
        const bool h = (i0 & 4u) != 0;
        if (level == 0) {  // words 0-2 (h = 0) or 3-5
            const uint4 a = ms2_block<IMPL>(r, g, 0);
            if (!h)
                return ms2_quad(a.x, a.y, a.z);
            const uint4 b = ms2_block<IMPL>(r, g, 1);
            return ms2_quad(a.w, b.x, b.y);
        }
        const uint4 c = ms2_block<IMPL>(r, g, 2);  // level 1: words 6-8 (h = 0) or 9-11
        if (h)
            return ms2_quad(c.y, c.z, c.w);
        const uint4 b = ms2_block<IMPL>(r, g, 1);
        return ms2_quad(b.z, b.w, c.x);
    } else if constexpr (KIND == 3) {
        // GC_RNG_STREAM24: draw j = bytes 3j .. 3j+2; a quad's 12 bytes start
        // 4-byte aligned (level n + i0 is a multiple of 4: one level)
        const uint64_t j = (uint64_t)level * r.n + i0;
        const uint64_t left = i0 < r.n ? r.n - i0 : 0;
        const uint8_t *b = reinterpret_cast<const uint8_t *>(r.stream) + 3 * j;
        if (left >= 4) {
            const uint3 w = *reinterpret_cast<const uint3 *>(b);
            return ms2_quad(w.x, w.y, w.z);
        }
        uint4 d = make_uint4(0u, 0u, 0u, 0u);
        uint32_t *dp = &d.x;
        for (uint32_t e = 0; e < (uint32_t)left; ++e)
            dp[e] = b[3 * e] | (uint32_t)b[3 * e + 1] << 8 | (uint32_t)b[3 * e + 2] << 16;
        return d;
    } else if constexpr (KIND == 0) {
        const uint64_t g = i0 >> 2;
        uint4 c;
        c.x = (uint32_t)g;
        c.y = ((uint32_t)(g >> 32) & 0xffffu) | (level << 16);
        c.z = (uint32_t)r.offset;
        c.w = (uint32_t)(r.offset >> 32);
        if constexpr (IMPL == 1) {
            if (i0 < (1ull << 34))  // g < 2^32: c.y is the uniform level word
                return philox4x32_10_g(c.x, level << 16, c.z, c.w, (uint32_t)r.seed, (uint32_t)(r.seed >> 32));
        }
        return philox4x32_10<IMPL>(c, (uint32_t)r.seed, (uint32_t)(r.seed >> 32));
    } else {
        const uint32_t *p = r.stream + (uint64_t)level * r.n + i0;
        const uint64_t left = i0 < r.n ? r.n - i0 : 0;
        if (left >= 4 && (reinterpret_cast<uintptr_t>(p) & 15u) == 0) {  // streamed once: one 16-byte NT load
            typedef uint32_t u4v __attribute__((ext_vector_type(4)));
            const u4v v = __builtin_nontemporal_load(reinterpret_cast<const u4v *>(p));
            return make_uint4(v.x, v.y, v.z, v.w);
        }
        uint4 d;
        d.x = left > 0 ? p[0] : 0u;
        d.y = left > 1 ? p[1] : 0u;
        d.z = left > 2 ? p[2] : 0u;
        d.w = left > 3 ? p[3] : 0u;
        return d;
    }
}

// One draw (gather / unaligned paths).
template <int KIND>
__device__ __forceinline__ uint32_t draw1(const RngArgs &r, uint32_t level, uint64_t i)
{
    if constexpr (KIND == 0 || KIND == 2) {
        const uint4 d = draws4<KIND>(r, level, i & ~(uint64_t)3);
        const uint32_t j = (uint32_t)(i & 3);
        return j == 0 ? d.x : (j == 1 ? d.y : (j == 2 ? d.z : d.w));
    } else if constexpr (KIND == 4 || KIND == 5) {
        return split_quad<KIND == 4 ? 8u : 16u>(r, i, 1).x;
    } else if constexpr (KIND == 3) {
        const uint8_t *b = reinterpret_cast<const uint8_t *>(r.stream) + 3 * ((uint64_t)level * r.n + i);
        return b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16;
    } else {
        return r.stream[(uint64_t)level * r.n + i];
    }
}

__device__ __forceinline__ uint32_t pick(const uint4 &v, int j)
{
    return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}
__device__ __forceinline__ float pickf(const float4 &v, int j)
{
    return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

// ---------------------------------------------------------------------------
// One element of the stochastic quantizer (compressors.py:299-316):
//   l = RN(RN(|x| / norm) * s); fl = trunc(l); p = l - fl (exact, in [0,1));
//   xi = fl + (u < p), u = (r & 0xFFFFFF) * 2^-24; q = sign(x) * xi.
// Returns xi (>= 0) and the sign separately.  A NaN quotient (0/0 for a
// zero bucket, NaN inputs) gives 0 where the reference raises (documented
// divergence); l is clamped to 2^30 (no-op when |x| <= norm).
// ---------------------------------------------------------------------------
struct QElem {
    int32_t xi;
    int32_t sg;
};

__device__ __forceinline__ QElem q_elem(float x, float norm, float s, uint32_t r)
{
    const float a = fabsf(x);
    const float ql = a / norm;  // IEEE division, as torch's div
    const bool ok = ql == ql;
    const float l = fminf(ql * s, 1073741824.0f);
    const int32_t fl = (int32_t)l;
    const float p = l - (float)fl;
    const float u = (float)(r & 0xFFFFFFu) * 0x1p-24f;
    QElem e;
    e.xi = ok ? fl + (u < p ? 1 : 0) : 0;
    e.sg = (x > 0.0f) ? 1 : ((x < 0.0f) ? -1 : 0);
    return e;
}

__device__ __forceinline__ int32_t q_signed(float x, float norm, float s, uint32_t r)
{
    const QElem e = q_elem(x, norm, s, r);
    return e.sg * e.xi;
}

// Division by the bucket-constant norm.  hipcc lowers a / b (IEEE, denormals
// on) to: D = div_scale(b), N = div_scale(a), r = rcp(D), r += r*(1 - D*r),
// q = N*r, q += r*(N - D*q), q = div_fmas(r*(N - D*q) + q), div_fixup.  With
// b normal, 1/b normal and a >= 2^-100 (or a == 0) div_scale is the identity
// and div_fmas a plain fma, so hoisting the reciprocal out of the loop gives
// bit-identical quotients for 1 mul + 4 fma.  Anything else takes the
// compiler's full division.
struct DivNorm {
    float norm;
    float r;       // 1/norm refined by one Newton step (the compiler's div sequence)
    float rr;      // RN(1/norm), IEEE division (Markstein's one-correction quotient)
    uint32_t lo1;  // bits(thr_lo) - 1: |x| in (0, thr_lo) takes the full division
    uint32_t hi;   // bits(thr_hi): |x| above (and inf / NaN) takes the full division
    bool fast;     // uniform: norm in [2^-100, 2^100]
};

__device__ __forceinline__ DivNorm make_div(float norm)
{
    DivNorm d;
    d.norm = norm;
    d.fast = norm >= 0x1p-100f && norm <= 0x1p100f;
    float r = __builtin_amdgcn_rcpf(norm);
    const float e = fmaf(-norm, r, 1.0f);
    d.r = fmaf(e, r, r);
    d.rr = 1.0f / norm;  // correctly rounded (-fhip-fp32-correctly-rounded-divide-sqrt)
    // thr_lo keeps |x| >= 2^-100 (no numerator scaling) and |x|/norm >= 2^-120
    // (normal quotient); thr_hi keeps |x|/norm <= 2^64 (no overflow scaling)
    d.lo1 = __float_as_uint(fmaxf(0x1p-100f, norm * 0x1p-120f)) - 1u;
    d.hi = __float_as_uint(fminf(norm * 0x1p64f, 3.4028234e38f));
    return d;
}

// the compiler's IEEE sequence with div_scale / div_fixup as identities:
// two Newton corrections on a refined reciprocal (kept for the lab A/B)
__device__ __forceinline__ float div_fast2(float a, const DivNorm &d)
{
    float q = a * d.r;
    float e = fmaf(-d.norm, q, a);
    q = fmaf(e, d.r, q);
    e = fmaf(-d.norm, q, a);
    return fmaf(e, d.r, q);
}

// Markstein (IBM J. Res. Dev. 34(1), 1990; Muller et al., Handbook of FP
// arithmetic, Thm. 4.13): with y = RN(1/b) and q = RN(a*y) within one ulp
// of a/b, e = a - b*q is exact (fma) and RN(q + e*y) = RN(a/b) — provided
// nothing over/underflows, which the same Range check as div_fast guarantees.
// One multiply + two fma instead of div_fast2's one + four; checked bit for
// bit against IEEE division on 3.4e10 random in-range pairs (tools/encode_lab
// divcheck, profiles/r01k_encode_lab.log).
__device__ __forceinline__ float div_fast(float a, const DivNorm &d)
{
    const float q = a * d.rr;
    const float e = fmaf(-d.norm, q, a);
    return fmaf(e, d.rr, q);
}

// running range of |x| bit patterns for the fast-division check:
// mn = min(bits - 1) (zero wraps to 0xFFFFFFFF and never triggers), mx = max(bits)
struct Range {
    uint32_t mn = 0xffffffffu, mx = 0u;
    __device__ __forceinline__ void add4(const float4 &v)
    {
        const uint32_t a = __float_as_uint(v.x) & 0x7fffffffu, b = __float_as_uint(v.y) & 0x7fffffffu;
        const uint32_t c = __float_as_uint(v.z) & 0x7fffffffu, e = __float_as_uint(v.w) & 0x7fffffffu;
        mn = min(min(mn, a - 1u), min(min(b - 1u, c - 1u), e - 1u));
        mx = max(max(mx, a), max(max(b, c), e));
    }
    __device__ __forceinline__ bool slow(const DivNorm &d) const { return (mn < d.lo1) | (mx > d.hi); }
};

__device__ __forceinline__ float4 quot4_ieee(const float4 &v, float norm)
{
    float4 q;
    q.x = fabsf(v.x) / norm;
    q.y = fabsf(v.y) / norm;
    q.z = fabsf(v.z) / norm;
    q.w = fabsf(v.w) / norm;
    return q;
}

// exact RN(|x| / norm) for 4 elements: fast path when the norm and the tile
// are in range, the compiler's IEEE division otherwise
__device__ __forceinline__ float4 quot4_exact(const float4 &v, const DivNorm &d)
{
    if (d.fast) {
        Range rg;
        rg.add4(v);
        if (!rg.slow(d)) {
            float4 q;
            q.x = div_fast(fabsf(v.x), d);
            q.y = div_fast(fabsf(v.y), d);
            q.z = div_fast(fabsf(v.z), d);
            q.w = div_fast(fabsf(v.w), d);
            return q;
        }
    }
    return quot4_ieee(v, d.norm);
}

// xi = stochastic round of l = |x|/norm * s (compressors.py:304-312) from the
// quotient: l clamped to [0, 2^30] by v_med3 (NaN quotient -> 0, inf -> 2^30,
// as the oracle), fl = trunc(l), p = l - fl exactly (v_fract_f32)
__device__ __forceinline__ int32_t xi_from_q(float ql, float s, uint32_t r)
{
    const float l = __builtin_amdgcn_fmed3f(ql * s, 0.0f, 1073741824.0f);
    const int32_t fl = (int32_t)l;
    const float p = __builtin_amdgcn_fractf(l);
    const float u = (float)(r & 0xFFFFFFu) * 0x1p-24f;
    return fl + (u < p ? 1 : 0);
}

__device__ __forceinline__ int32_t sgn_of(float x) { return (x > 0.0f) ? 1 : ((x < 0.0f) ? -1 : 0); }

// nontemporal 16-byte load: streamed inputs read once per pass (x)
__device__ __forceinline__ float4 ld_nt(const float4 *p)
{
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v r = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(p));
    return make_float4(r.x, r.y, r.z, r.w);
}

// nontemporal 16-byte store: streamed outputs written once (decoded floats,
// packed words) bypass the cache hierarchy's allocation; 400 MB of decode
// stores take 69 instead of 92 us (profiles/r01n_lab2_nt.log)
__device__ __forceinline__ void st_nt4(float *p, const float4 &v)
{
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v r = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(r, reinterpret_cast<f4v *>(p));
}

// ---------------------------------------------------------------------------
// GlobalRandK gathers / scatters (MODE 2).  A thread's quads in C planes
// (elements k*M + i0 .. +3, k = k0 .. k0+C-1): every index load is issued
// before any value load, so the thread waits two dependent round trips
// instead of 2C.  Addresses past n are clamped to n-1 (always valid, n > 0)
// so the loads stay unconditional and issue back to back; the caller masks
// those lanes.
// ---------------------------------------------------------------------------
// planes per gather batch: up to 8 (8 x 4 int64 indices = 64 VGPRs)
constexpr int gather_chunk(int L) { return L < 8 ? L : 8; }

template <int C>
__device__ __forceinline__ void gather_idx(const int64_t *__restrict__ idx, uint64_t n, uint64_t M, uint64_t i0,
                                           int k0, int64_t (&id)[C][4])
{
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e)
            id[c][e] = idx[min((uint64_t)(k0 + c) * M + i0 + e, n - 1)];
}

template <int C>
__device__ __forceinline__ void gather_planes(const float *__restrict__ x, const int64_t *__restrict__ idx,
                                              uint64_t n, uint64_t M, uint64_t i0, int k0, float4 (&v)[C])
{
    int64_t id[C][4];
    gather_idx<C>(idx, n, M, i0, k0, id);
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const uint64_t b = (uint64_t)(k0 + c) * M + i0;
        v[c].x = b + 0 < n ? x[id[c][0]] : 0.0f;
        v[c].y = b + 1 < n ? x[id[c][1]] : 0.0f;
        v[c].z = b + 2 < n ? x[id[c][2]] : 0.0f;
        v[c].w = b + 3 < n ? x[id[c][3]] : 0.0f;
    }
}

// ---------------------------------------------------------------------------
// wave64 / block reductions
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}

}  // namespace gc
