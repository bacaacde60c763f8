// qsgd_encode.h — the fused QSGD-MaxNorm encode kernel (quantize + stochastic
// round + carry-free planar pack), compressors.py:299-316.
//
// The product kernel only: full tiles take the integer stochastic rounding,
// nontemporal loads of x and nontemporal stores of the words (tools/lab2,
// profiles/r01m_*, r01n_*).  The measurement variants of earlier rounds
// (ablations, instruction mixes, schedules) live in tools/encode_lab_kernel.h.
//
// Per element, the reference's arithmetic in its own order:
//   ql = RN(|x| / norm)        IEEE division (see div_norm below)
//   l  = RN(ql * s)            then min(l, s) (lane safety; no-op in contract)
//   fl = trunc(l), p = l - fl  (v_cvt_i32_f32, v_fract_f32: exact for l >= 0)
//   xi = fl + [ (r & 0xFFFFFF) * 2^-24 < p ]
//   lane = qmax + sign(x) * xi
// A NaN quotient gives xi = 0 (the oracle's q = 0); over-range values saturate.
#pragma once

#include "gc_device.h"

namespace gc {

// the packed words: written once, never read back by this kernel (NT store)
__device__ __forceinline__ void store_words(uint32_t *p, const uint4 &v)
{
    typedef uint32_t u4v __attribute__((ext_vector_type(4)));
    const u4v r = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(r, reinterpret_cast<u4v *>(p));
}

// ---------------------------------------------------------------------------
// Integer form of the stochastic rounding (full tiles), bit-identical to
// enc_lane on the fast path (|x| <= norm, no tiny |x|, norm in range):
//   q  = RN(x / norm)                 signed Markstein quotient (RN is odd)
//   Ls = RN(q * s*2^24)               = RN(|x|/norm * s) * 2^24 exactly (power-of-two
//                                       scaling of a normal product; |Ls| <= s*2^24)
//   Ac = ceil(|Ls|) = fl*2^24 + F     F = ceil(p*2^24): for l >= 1/2, Ls is an
//                                       integer; below, fl = 0 and F = ceil(l*2^24)
//   [u < p] = [m < F]                 u = m*2^-24, m = r & 0xFFFFFF integer
//   h  = (floor(-|Ls|) + m) >> 24     = -fl - [m < F] = -xi   (arithmetic shift)
// so the lane needs one v_cvt_flr_i32_f32 (-|Ls| as a source modifier), one
// and, one add and a 24-bit multiply whose SDWA byte-3 select is the shift.
// The sign is folded into that multiply: sgk = med3(bits(x), -2^sh, 2^sh) is
// +-2^sh for every nonzero fast-path x (|x| >= 2^-100 has bits >= 2^27 > 2^sh)
// and h = 0 whenever x is +-0, so  h * sgk = -q * 2^sh.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int32_t cvt_flr_neg_abs(float v)
{
    int32_t r;
    asm("v_cvt_flr_i32_f32_e64 %0, -|%1|" : "=v"(r) : "v"(v));
    return r;
}

__device__ __forceinline__ int32_t med3_i32(int32_t a, int32_t lo, int32_t hi)
{
    int32_t r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(lo), "s"(hi));
    return r;
}

// (r & 0xFFFFFF) + c in one op: v_mad_u32_u24 reads only the low 24 bits
__device__ __forceinline__ int32_t add_low24(uint32_t r, int32_t c)
{
    int32_t o;
    asm("v_mad_u32_u24 %0, %1, 1, %2" : "=v"(o) : "v"(r), "v"(c));
    return o;
}

// -q * 2^sh for one element (see above) from Ls = RN(q * s*2^24); lo = -2^sh, hi = 2^sh
__device__ __forceinline__ int32_t enc_negq_int(float x, float Ls, uint32_t r, int32_t lo, int32_t hi)
{
    const int32_t t = add_low24(r, cvt_flr_neg_abs(Ls));
    return __mul24(t >> 24, med3_i32(__float_as_int(x), lo, hi));
}

typedef float gc_f2 __attribute__((ext_vector_type(2)));

// Ls = RN(RN(x / norm) * S24) for a pair, as packed fp32 (v_pk_mul_f32 /
// v_pk_fma_f32): the signed Markstein quotient (RN is odd), then the scale
__device__ __forceinline__ gc_f2 ls2(float a, float b, const DivNorm &d, float S24)
{
    const gc_f2 x = {a, b};
    const gc_f2 y = {d.rr, d.rr};
    const gc_f2 nb = {-d.norm, -d.norm};
    const gc_f2 q0 = x * y;
    const gc_f2 e = __builtin_elementwise_fma(nb, q0, x);
    const gc_f2 q = __builtin_elementwise_fma(e, y, q0);
    const gc_f2 sc = {S24, S24};
    return q * sc;
}

// b = 8 (s*2^24 >= 2^31): the unsigned form.  Ac = ceil(|Ls|) <= 255*2^24,
// t = Ac + (~r & 0xFFFFFF) < 2^32, xi = t >> 24 = fl + [m < F]; returns +q * 2^sh
__device__ __forceinline__ int32_t enc_q_wide(float x, float Ls, uint32_t r, int32_t lo, int32_t hi)
{
    const uint32_t ac = (uint32_t)__builtin_ceilf(fabsf(Ls));
    const uint32_t t = (uint32_t)add_low24(~r, (int32_t)ac);
    return __mul24((int32_t)(t >> 24), med3_i32(__float_as_int(x), lo, hi));
}

// One full tile from split-plane draws (KIND 4 / 5, gc_device.h).  With c =
// ceil(|Ls|) = fl*2^24 + F the bit is [m < F], m = the 24-bit draw.  Knowing
// only m's top HB bits hm (low bits zero), [hm < F] is already right unless
// F - 1 and m share their top HB bits (then hm <= F - 1 < hm + 2^(24-HB) and
// the low bits decide).  Pass 1 reads the HI plane and checks every element
// of the tile for that tie; a tile with one returns false and the caller's
// general path encodes it from both planes (about 24 / 2^HB of the tiles: 1 in
// 2,700 for HB = 16).  Pass 2 recomputes Ls (cheaper than holding 4L values
// across the check) and packs with the HI bits alone: the LO plane is never
// read for such tiles.  A flag where F = 0 is harmless (the general path is
// exact either way).  Otherwise enc_tile_int's arithmetic.
__device__ __forceinline__ uint32_t ld_nt_u32(const uint8_t *p)
{
    return __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(p));
}
__device__ __forceinline__ uint2 ld_nt_u2(const uint8_t *p)
{
    typedef uint32_t u2v __attribute__((ext_vector_type(2)));
    const u2v v = __builtin_nontemporal_load(reinterpret_cast<const u2v *>(p));
    return make_uint2(v.x, v.y);
}

// the HI bits of draw e (0..3) of a plane's quad, in place (low 24-HB bits zero)
template <uint32_t HB>
__device__ __forceinline__ uint32_t split_hi(const uint32_t (&hw)[HB / 8], int e)
{
    constexpr uint32_t HM = ((1u << HB) - 1u) << (24u - HB);
    if constexpr (HB == 8)
        return e == 0 ? (hw[0] << 16) & HM : e == 1 ? (hw[0] << 8) & HM : e == 2 ? hw[0] & HM : (hw[0] >> 8) & HM;
    else
        return e == 0 ? (hw[0] << 8) & HM : e == 1 ? (hw[0] >> 8) & HM
             : e == 2 ? (hw[HB / 8 - 1] << 8) & HM : (hw[HB / 8 - 1] >> 8) & HM;
}

// c (WIDE) or -c (narrow) of one element from its Ls
template <bool WIDE>
__device__ __forceinline__ int32_t split_c(float ls)
{
    if constexpr (WIDE)
        return (int32_t)(uint32_t)__builtin_ceilf(fabsf(ls));
    else
        return cvt_flr_neg_abs(ls);
}

template <int L, int KIND, bool WIDE>
__device__ __forceinline__ bool enc_tile_int_split(const float4 (&xv)[L], uint32_t t4, uint32_t M32, const DivNorm &dv,
                                                   float S24, uint32_t w, uint32_t Cw, const RngArgs &rng, uint4 &acc)
{
    constexpr uint32_t HB = KIND == 4 ? 8u : 16u, LB = 24u - HB;
    constexpr uint32_t HM = ((1u << HB) - 1u) << LB;
    constexpr int H = L / 2;
    const uint8_t *hp = reinterpret_cast<const uint8_t *>(rng.stream);
    uint32_t hw[L][HB / 8];
#pragma unroll
    for (int k = 0; k < L; ++k) {
        const uint32_t i0 = k * M32 + t4;
        if constexpr (HB == 8) {
            hw[k][0] = ld_nt_u32(hp + i0);
        } else {
            const uint2 v = ld_nt_u2(hp + 2u * i0);
            hw[k][0] = v.x;
            hw[k][HB / 8 - 1] = v.y;
        }
    }
    // pass 1: c per element (xv dies here), the signs, the tie check
    int32_t cc[L][4];
    uint64_t neg = 0;  // bit 4k + e: x < 0 (or -0, whose c is 0: no effect); L <= 16
    bool tie = false;
#pragma unroll
    for (int k = 0; k < L; ++k) {
        const gc_f2 l01 = ls2(xv[k].x, xv[k].y, dv, S24);
        const gc_f2 l23 = ls2(xv[k].z, xv[k].w, dv, S24);
        const float ls[4] = {l01.x, l01.y, l23.x, l23.y};
        const float xs[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            cc[k][e] = split_c<WIDE>(ls[e]);
            neg |= (uint64_t)(__float_as_uint(xs[e]) >> 31) << (4 * k + e);
            const uint32_t cm1 = WIDE ? (uint32_t)cc[k][e] - 1u : ~(uint32_t)cc[k][e];  // c - 1
            tie |= ((cm1 ^ split_hi<HB>(hw[k], e)) & HM) == 0u;
        }
    }
    if (__builtin_expect(tie, 0))
        return false;
    // pass 2: the lanes from the HI bits alone (x = +-0 has c = 0 and xi = 0)
    int32_t lo[4] = {0, 0, 0, 0}, hi[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < L; ++k) {
        const uint32_t sh = (uint32_t)(k < H ? k : k - H) * w;
        int32_t *a = k < H ? lo : hi;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint32_t rd = split_hi<HB>(hw[k], e);
            int32_t v;
            if constexpr (WIDE)  // xi = (c + (~m & 0xFFFFFF)) >> 24 = fl + [m < F]
                v = (int32_t)((uint32_t)add_low24(~rd, cc[k][e]) >> 24);
            else  // (m - c) >> 24 = -xi (m < 2^24 here)
                v = ((int32_t)rd + cc[k][e]) >> 24;
            v <<= sh;
            a[e] += ((neg >> (4 * k + e)) & 1u) ? -v : v;
        }
    }
    const uint32_t hs = (uint32_t)H * w;
    if constexpr (WIDE) {
        acc.x = Cw + ((uint32_t)lo[0] + ((uint32_t)hi[0] << hs));
        acc.y = Cw + ((uint32_t)lo[1] + ((uint32_t)hi[1] << hs));
        acc.z = Cw + ((uint32_t)lo[2] + ((uint32_t)hi[2] << hs));
        acc.w = Cw + ((uint32_t)lo[3] + ((uint32_t)hi[3] << hs));
    } else {
        acc.x = Cw - ((uint32_t)lo[0] + ((uint32_t)hi[0] << hs));
        acc.y = Cw - ((uint32_t)lo[1] + ((uint32_t)hi[1] << hs));
        acc.z = Cw - ((uint32_t)lo[2] + ((uint32_t)hi[2] << hs));
        acc.w = Cw - ((uint32_t)lo[3] + ((uint32_t)hi[3] << hs));
    }
    return true;
}

// one full tile (L planes x 4 words) on the integer path.  Lanes k < H
// accumulate at shift k*w, lanes k >= H at (k-H)*w, so every 24-bit
// multiplier is +-2^sh with sh <= 15; word = C -+ (lo + (hi << H*w)).
template <int L, int KIND, bool WIDE>
__device__ __forceinline__ uint4 enc_tile_int(const float4 (&xv)[L], uint32_t t4, uint32_t M32, const DivNorm &dv,
                                              float S24, uint32_t w, uint32_t Cw, const RngArgs &rng)
{
    constexpr int H = L / 2;
    int32_t lo[4] = {0, 0, 0, 0}, hi[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < L; ++k) {
        const gc_f2 l01 = ls2(xv[k].x, xv[k].y, dv, S24);
        const gc_f2 l23 = ls2(xv[k].z, xv[k].w, dv, S24);
        const uint4 r = draws4<KIND>(rng, 0, k * M32 + t4);
        const uint32_t sh = (uint32_t)(k < H ? k : k - H) * w;
        const int32_t bl = -(1 << sh), bh = 1 << sh;
        int32_t *a = k < H ? lo : hi;
        if constexpr (WIDE) {
            a[0] += enc_q_wide(xv[k].x, l01.x, r.x, bl, bh);
            a[1] += enc_q_wide(xv[k].y, l01.y, r.y, bl, bh);
            a[2] += enc_q_wide(xv[k].z, l23.x, r.z, bl, bh);
            a[3] += enc_q_wide(xv[k].w, l23.y, r.w, bl, bh);
        } else {
            a[0] += enc_negq_int(xv[k].x, l01.x, r.x, bl, bh);
            a[1] += enc_negq_int(xv[k].y, l01.y, r.y, bl, bh);
            a[2] += enc_negq_int(xv[k].z, l23.x, r.z, bl, bh);
            a[3] += enc_negq_int(xv[k].w, l23.y, r.w, bl, bh);
        }
    }
    const uint32_t hs = (uint32_t)H * w;
    uint4 acc;
    if constexpr (WIDE) {
        acc.x = Cw + ((uint32_t)lo[0] + ((uint32_t)hi[0] << hs));
        acc.y = Cw + ((uint32_t)lo[1] + ((uint32_t)hi[1] << hs));
        acc.z = Cw + ((uint32_t)lo[2] + ((uint32_t)hi[2] << hs));
        acc.w = Cw + ((uint32_t)lo[3] + ((uint32_t)hi[3] << hs));
    } else {
        acc.x = Cw - ((uint32_t)lo[0] + ((uint32_t)hi[0] << hs));
        acc.y = Cw - ((uint32_t)lo[1] + ((uint32_t)hi[1] << hs));
        acc.z = Cw - ((uint32_t)lo[2] + ((uint32_t)hi[2] << hs));
        acc.w = Cw - ((uint32_t)lo[3] + ((uint32_t)hi[3] << hs));
    }
    return acc;
}

// fast-path tile check of the integer form: every |x| <= norm (inf / NaN excluded by
// the bit compare) and no nonzero |x| below the division's low threshold.
// 2*bits drops the sign; 2*bits - 2 wraps +-0 to 0xFFFFFFFE.
struct RangeI {
    uint32_t mn = 0xffffffffu, mx = 0u;
    __device__ __forceinline__ void add4(const float4 &v)
    {
        const uint32_t a = __float_as_uint(v.x), b = __float_as_uint(v.y);
        const uint32_t c = __float_as_uint(v.z), e = __float_as_uint(v.w);
        mn = min(min(mn, 2u * a - 2u), min(min(2u * b - 2u, 2u * c - 2u), 2u * e - 2u));
        mx = max(max(mx, 2u * a), max(max(2u * b, 2u * c), 2u * e));
    }
    // lo2 = 2 * bits(thr_lo) - 2, hi2 = 2 * bits(norm)
    __device__ __forceinline__ bool slow(uint32_t lo2, uint32_t hi2) const { return (mn < lo2) | (mx > hi2); }
};

// lane value of one element (ql = |x| / norm).  A NaN quotient (0/0, NaN
// input) gives xi = 0 (fmaxf(NaN, 0) = 0); an infinite one saturates at s.
__device__ __forceinline__ uint32_t enc_lane(float x, float ql, float s, int32_t qmax, uint32_t r)
{
    // v_med3_f32(l, 0, s): clamps to [0, s]; a NaN l yields 0 (checked against
    // the oracle by tests/test_gpu_parity.py::test_encode_non_finite_and_tiny_inputs)
    const float l = __builtin_amdgcn_fmed3f(ql * s, 0.0f, s);
    const uint32_t fl = (uint32_t)(int32_t)l;
    const float p = __builtin_amdgcn_fractf(l);
    const float u = (float)(r & 0xFFFFFFu) * 0x1p-24f;
    const uint32_t xi = fl + (u < p ? 1u : 0u);
    // qmax + sign(x)*xi without a multiply: sg = 0 or ~0 from the sign bit
    // (-0.0 and signed NaN give xi = 0 anyway): (xi ^ sg) - sg + qmax
    const uint32_t sg = (uint32_t)(__float_as_int(x) >> 31);
    return (xi ^ sg) + ((uint32_t)qmax - sg);
}

__device__ __forceinline__ float4 quot4_fast(const float4 &v, const DivNorm &d)
{
    float4 q;
    q.x = div_fast(fabsf(v.x), d);
    q.y = div_fast(fabsf(v.y), d);
    q.z = div_fast(fabsf(v.z), d);
    q.w = div_fast(fabsf(v.w), d);
    return q;
}

// Full tiles: every one of the L planes of words 4t..4t+3 is in range, so
// no per-element bounds, 32-bit element indices, L float4 loads in flight
// (nontemporal: x is streamed once per pass), the integer stochastic rounding
// when the tile passes its range check.  Tail quads, gathers, unaligned x and
// the non-fast-division case go through the generic body.
template <int L, int KIND, int MODE, int MINW = 1>
__global__ __launch_bounds__(kBlock, MINW) void k_qsgd_encode(const float *__restrict__ x, const int64_t *__restrict__ idx,
                                                        uint64_t n, const float *__restrict__ normp, float s,
                                                        int32_t qmax, uint32_t w, uint64_t M, RngArgs rng,
                                                        uint32_t *__restrict__ words)
{
    const float norm = *normp;
    const DivNorm dv = make_div(norm);
    const bool fast = dv.fast;
    const uint64_t quads = M >> 2;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;

    // quads whose last plane is full: (L-1)*M + 4t + 3 < n
    const uint64_t last = (uint64_t)(L - 1) * M;
    const uint64_t full = (MODE == 0 && fast && n >= last + 4 && n < (1ull << 32)) ? (n - last) >> 2 : 0;
    const uint32_t M32 = (uint32_t)M;
    // integer-path constants (uniform): b <= 7 (s * 2^24 < 2^31) takes the
    // signed floor form, b = 8 the unsigned ceil form
    const bool intok = s <= 255.0f, narrow = s <= 127.0f;
    const float S24 = s * 16777216.0f;
    const uint32_t lo2 = 2u * dv.lo1, hi2 = 2u * __float_as_uint(norm);
    uint32_t Cw = 0;
    for (int k = 0; k < L; ++k)
        Cw += (uint32_t)qmax << (k * w);
    for (; t < full; t += stride) {
        const uint32_t t4 = (uint32_t)t * 4u;
        float4 xv[L];
#pragma unroll
        for (int k = 0; k < L; ++k)
            xv[k] = ld_nt(reinterpret_cast<const float4 *>(x + (k * M32 + t4)));
        if (intok) {
            RangeI rg;
#pragma unroll
            for (int k = 0; k < L; ++k)
                rg.add4(xv[k]);
            if (__builtin_expect(!rg.slow(lo2, hi2), 1)) {
                const uint4 acc = narrow ? enc_tile_int<L, KIND, false>(xv, t4, M32, dv, S24, w, Cw, rng)
                                         : enc_tile_int<L, KIND, true>(xv, t4, M32, dv, S24, w, Cw, rng);
                store_words(words + t4, acc);
                continue;
            }
        }
        float4 q[L];
        Range rg;
#pragma unroll
        for (int k = 0; k < L; ++k) {
            q[k] = quot4_fast(xv[k], dv);
            rg.add4(xv[k]);
        }
        if (__builtin_expect(rg.slow(dv), 0)) {
#pragma unroll
            for (int k = 0; k < L; ++k)
                q[k] = quot4_ieee(xv[k], norm);
        }
        uint4 acc = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int k = 0; k < L; ++k) {
            const uint4 r = draws4<KIND>(rng, 0, k * M32 + t4);
            const uint32_t sh = (uint32_t)k * w;
            acc.x |= enc_lane(xv[k].x, q[k].x, s, qmax, r.x) << sh;
            acc.y |= enc_lane(xv[k].y, q[k].y, s, qmax, r.y) << sh;
            acc.z |= enc_lane(xv[k].z, q[k].z, s, qmax, r.z) << sh;
            acc.w |= enc_lane(xv[k].w, q[k].w, s, qmax, r.w) << sh;
        }
        *reinterpret_cast<uint4 *>(words + t4) = acc;
    }
    if constexpr (MODE == 2) {
        // GlobalRandK gathers: planes in chunks of up to 8, all index loads
        // then all value loads per chunk (gather_planes)
        constexpr int C = L < 8 ? L : 8;
        for (; t < quads; t += stride) {
            uint4 acc = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (int k0 = 0; k0 < L; k0 += C) {
                float4 v[C];
                gather_planes<C>(x, idx, n, M, 4 * t, k0, v);
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    const int k = k0 + j;
                    const uint64_t i0 = (uint64_t)k * M + 4 * t;
                    if (k < L && i0 < n) {
                        const uint4 r = draws4<KIND>(rng, 0, i0);
                        Range rg;
                        rg.add4(v[j]);
                        const float4 q = fast && !rg.slow(dv) ? quot4_fast(v[j], dv) : quot4_ieee(v[j], norm);
                        const uint32_t sh = (uint32_t)k * w;
                        acc.x |= enc_lane(v[j].x, q.x, s, qmax, r.x) << sh;
                        acc.y |= (i0 + 1 < n ? enc_lane(v[j].y, q.y, s, qmax, r.y) : 0u) << sh;
                        acc.z |= (i0 + 2 < n ? enc_lane(v[j].z, q.z, s, qmax, r.z) : 0u) << sh;
                        acc.w |= (i0 + 3 < n ? enc_lane(v[j].w, q.w, s, qmax, r.w) : 0u) << sh;
                    }
                }
            }
            *reinterpret_cast<uint4 *>(words + 4 * t) = acc;
        }
        return;
    }
    // generic body: tail quads (partial planes), unaligned x, odd norms
    for (; t < quads; t += stride) {
        uint4 acc = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int k = 0; k < L; ++k) {
            const uint64_t i0 = (uint64_t)k * M + 4 * t;
            if (i0 < n) {
                float4 v;
                if (MODE == 0 && i0 + 4 <= n) {
                    v = *reinterpret_cast<const float4 *>(x + i0);
                } else {
                    v.x = MODE == 2 ? x[idx[i0]] : x[i0];
                    v.y = i0 + 1 < n ? (MODE == 2 ? x[idx[i0 + 1]] : x[i0 + 1]) : 0.0f;
                    v.z = i0 + 2 < n ? (MODE == 2 ? x[idx[i0 + 2]] : x[i0 + 2]) : 0.0f;
                    v.w = i0 + 3 < n ? (MODE == 2 ? x[idx[i0 + 3]] : x[i0 + 3]) : 0.0f;
                }
                const uint4 r = draws4<KIND>(rng, 0, i0);
                float4 q;
                Range rg;
                rg.add4(v);
                if (fast && !rg.slow(dv))
                    q = quot4_fast(v, dv);
                else
                    q = quot4_ieee(v, norm);
                const uint32_t sh = (uint32_t)k * w;
                acc.x |= enc_lane(v.x, q.x, s, qmax, r.x) << sh;
                acc.y |= (i0 + 1 < n ? enc_lane(v.y, q.y, s, qmax, r.y) : 0u) << sh;
                acc.z |= (i0 + 2 < n ? enc_lane(v.z, q.z, s, qmax, r.z) : 0u) << sh;
                acc.w |= (i0 + 3 < n ? enc_lane(v.w, q.w, s, qmax, r.w) : 0u) << sh;
            }
        }
        *reinterpret_cast<uint4 *>(words + 4 * t) = acc;
    }
}

// the exact encode of word quad tq from split-plane draws, a plane at a time
// (partial planes: n): the path of tiles with a tie, slow ranges, b > 8 and
// tails.  Not inlined: the split tile's registers are not shared with it.
template <int L, int KIND>
__device__ __noinline__ void split_exact_quad(const float *__restrict__ x, uint64_t n, const DivNorm &dv, float s,
                                              int32_t qmax, uint32_t w, uint64_t M, const RngArgs &rng,
                                              uint32_t *__restrict__ words, uint64_t tq)
{
    uint4 acc = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll 1
    for (int k = 0; k < L; ++k) {
        const uint64_t i0 = (uint64_t)k * M + 4 * tq;
        if (i0 >= n)
            break;
        float4 v;
        if (i0 + 4 <= n) {
            v = ld_nt(reinterpret_cast<const float4 *>(x + i0));
        } else {
            v.x = x[i0];
            v.y = i0 + 1 < n ? x[i0 + 1] : 0.0f;
            v.z = i0 + 2 < n ? x[i0 + 2] : 0.0f;
            v.w = 0.0f;
        }
        const float4 q = quot4_exact(v, dv);
        const uint4 r = draws4<KIND>(rng, 0, i0);
        const uint32_t sh = (uint32_t)k * w;
        acc.x |= enc_lane(v.x, q.x, s, qmax, r.x) << sh;
        acc.y |= (i0 + 1 < n ? enc_lane(v.y, q.y, s, qmax, r.y) : 0u) << sh;
        acc.z |= (i0 + 2 < n ? enc_lane(v.z, q.z, s, qmax, r.z) : 0u) << sh;
        acc.w |= (i0 + 3 < n ? enc_lane(v.w, q.w, s, qmax, r.w) : 0u) << sh;
    }
    *reinterpret_cast<uint4 *>(words + 4 * tq) = acc;
}

// The encode from split-plane draws (GC_RNG_SPLIT8 / SPLIT16): a kernel of its
// own, so the one heavy path (enc_tile_int_split) does not share its register
// allocation with the Philox / stream paths (125 VGPRs: 4 waves per SIMD).
// Full tiles in range take the split tile; a tile with a tie, a slow range,
// b > 8, or a tail quad takes split_exact_quad, a separate function, so the
// compiler can neither hoist its LO-plane loads above the tie check nor hold
// its values across the split tile.
template <int L, int KIND>
__global__ __launch_bounds__(kBlock) void k_qsgd_encode_split(const float *__restrict__ x, uint64_t n,
                                                              const float *__restrict__ normp, float s, int32_t qmax,
                                                              uint32_t w, uint64_t M, RngArgs rng,
                                                              uint32_t *__restrict__ words)
{
    static_assert(KIND == 4 || KIND == 5, "split-plane draws only");
    static_assert(L <= 16, "the sign mask holds 4 L bits");
    const float norm = *normp;
    const DivNorm dv = make_div(norm);
    const uint64_t quads = M >> 2;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint64_t last = (uint64_t)(L - 1) * M;
    const uint64_t full = (dv.fast && n >= last + 4 && n < (1ull << 32)) ? (n - last) >> 2 : 0;
    const uint32_t M32 = (uint32_t)M;
    const bool intok = s <= 255.0f, narrow = s <= 127.0f;
    const float S24 = s * 16777216.0f;
    const uint32_t lo2 = 2u * dv.lo1, hi2 = 2u * __float_as_uint(norm);
    uint32_t Cw = 0;
    for (int k = 0; k < L; ++k)
        Cw += (uint32_t)qmax << (k * w);
    for (; t < full; t += stride) {
        const uint32_t t4 = (uint32_t)t * 4u;
        bool done = false;
        if (intok) {
            float4 xv[L];
#pragma unroll
            for (int k = 0; k < L; ++k)
                xv[k] = ld_nt(reinterpret_cast<const float4 *>(x + (k * M32 + t4)));
            RangeI rg;
#pragma unroll
            for (int k = 0; k < L; ++k)
                rg.add4(xv[k]);
            if (__builtin_expect(!rg.slow(lo2, hi2), 1)) {
                uint4 acc;
                done = narrow ? enc_tile_int_split<L, KIND, false>(xv, t4, M32, dv, S24, w, Cw, rng, acc)
                              : enc_tile_int_split<L, KIND, true>(xv, t4, M32, dv, S24, w, Cw, rng, acc);
                if (done)
                    store_words(words + t4, acc);
            }
        }
        if (__builtin_expect(!done, 0))
            split_exact_quad<L, KIND>(x, n, dv, s, qmax, w, M, rng, words, t);
    }
    for (; t < quads; t += stride)
        split_exact_quad<L, KIND>(x, n, dv, s, qmax, w, M, rng, words, t);
}

}  // namespace gc
