// ms_fast.h — dense fast paths of the multi-scale / two-scale kernels
// (multiscale.hip; compressors.py:754-826 and 612-680).  Same outputs as the
// generic kernels, bit for bit; what changes is the cost per element:
//   * the level decision and the selected level's rounding use the integer
//     stochastic rounding of qsgd_encode.h (the integer form): one signed Markstein
//     quotient per element, then per level one packed scale, one
//     v_cvt_flr_i32_f32 and one v_mad_u32_u24;
//   * the mask-plane position of an element (i / M_mask) is a multiply-high
//     division by the plane size (no 64-bit divide);
//   * the order-0 decode RN(RN(Q*norm) / s) divides by the level scale with
//     Markstein's one-correction quotient (y = RN(1/s) per level);
//   * x, the mask words and the decoded floats are streamed nontemporally.
// Work split: a block owns 64 word quads; its 4 waves take the planes
// p = wave, wave+4, ... of those quads (lanes = consecutive quads, so every
// load is a 1 KB contiguous wave access).  A thread walks at most
// ceil(planes/4) planes instead of all of them: one thread per quad and 32
// sequential plane loads (the mask at W=1) ran 41 us at 23.5M floats, latency
// bound on 11 waves per CU (profiles/r01q_lab_ms*.log).  Encoders combine the
// waves' partial words through LDS; the decode needs no combine.
// Taken when: dense aligned x (MODE 0), n < 2^32, 2 or 3 levels (NL, a
// template argument: level tables and mask fields resolve at compile time),
// every level <= 7 bits (s * 2^24 < 2^31; the decode, which does no rounding,
// up to 16 bits).  Levels of 8-24 bits run the same kernels with MSV_WIDE:
// the wave split and the streaming, with the generic per-element rounding.
// Anything else, and any quad whose |x| fail the RangeI check (or whose norm
// is outside the Markstein range), runs the generic per-element code.
#pragma once

#include "gc_device.h"
#include "ms_common.h"
#include "qsgd_encode.h"

namespace gc {

// x / d for any 32-bit x, d >= 2 (the "round-up" multiply-high method with
// the add-and-halve fix; m = floor(2^32 (2^s - d) / d) + 1, s = ceil(log2 d))
struct FastDiv {
    uint32_t m, s1, d;
};

__device__ __forceinline__ uint32_t fdiv(uint32_t x, const FastDiv &f)
{
    const uint32_t t = __umulhi(x, f.m);
    return (t + ((x - t) >> 1)) >> f.s1;
}

inline FastDiv make_fastdiv(uint32_t d)
{
    uint32_t s = 0;
    while ((1ull << s) < d)
        ++s;
    FastDiv f;
    f.d = d;
    f.s1 = s - 1;
    f.m = (uint32_t)((((1ull << s) - d) << 32) / d + 1);
    return f;
}

// kernel variants: the product uses VAR = 0 (levels <= 7 bits) or MSV_WIDE,
// and MSV_EAGER0 for the one-pass encode with Philox draws (33.5 against
// 34.9 us on the ResNet50 bucket, profiles/r03l_lab_ms.log: the two Philox
// chains interleave, and the level-0 block is needed by nearly every wave
// anyway); the others are lab variants (tools/lab_ms.hip)
enum : int {
    MSV_PERTHREAD = 1,  // one thread walks all planes of its word quad (no wave split)
    MSV_NORNG = 2,      // measurement only: draws = a hash of the element index (no Philox)
    MSV_NOSLOW = 4,     // measurement only: no generic fallback (assumes every quad is fast)
    MSV_WIDE = 8,       // a lowest level of 8-24 bits: the wave-split kernels with the generic
                        // per-element rounding (quot4_exact + xi_from_q) on every quad
    MSV_DEFER = 16,     // lab: the one-pass kernel with the generic path deferred to after the plane loop
    MSV_EAGER0 = 32,    // the one-pass fast path computes level 0's draws for every quad, interleaved
                        // with the upper levels' (no wave-level branch; same draws and outputs)
    MSV_PREFETCH = 64,  // octet one-pass kernel: the next plane's loads are issued before this plane's
                        // math (the product: 29.1 against 31.6 us, profiles/r04n_lab_ms.log)
    MSV_ROLL = 128,     // octet mask / select kernels: the plane loop is not unrolled (the product:
                        // fewer VGPRs, more waves; mask 22.7 against 27.4 us, with the q cache 32.4
                        // against 45.0 us, profiles/r04n_lab_ms.log)
    MSV_UFLAG = 1024,   // octet mask kernel: the per-lane tail tests behind a wave-uniform flag
                        // (round 5 also measured two planes per loop trip and a second copy of the
                        // plane code for full tiles: slower, removed; DESIGN_HISTORY §5.2)
    MSV_PLAINST = 2048, // plain (temporal) stores of the words / mask words instead of nontemporal ones:
                        // the next kernel of a step reads them at once (profiles/r05zh, r05zj_lab_ms.log)
};

template <int KIND, int VAR>
__device__ __forceinline__ uint4 ms_draws4(const RngArgs &rng, uint32_t level, uint32_t i0)
{
    if constexpr ((VAR & MSV_NORNG) != 0) {
        const uint32_t b = (i0 + level * 0x9E3779B9u) * 2654435761u;
        return make_uint4(b, b ^ 0x5bd1e995u, b + 0x27d4eb2fu, b * 3u);
    } else {
        return draws4<KIND>(rng, level, i0);
    }
}

// per-level constants of the fast path (uniform)
struct MsFastArg {
    float S24[GC_MAX_LEVELS];  // s_l * 2^24
    float y[GC_MAX_LEVELS];    // RN(1 / s_l)
    int32_t thr;               // -maxv * 2^24: level l qualifies iff T_l >= thr
};

// the mask level of 4 elements, from W-summed thermometer fields; the plane
// of element i0 is i0 / M (fast division), all 4 share it (M % 4 == 0)
template <int NL>
__device__ __forceinline__ uint4 mask_levels4_fast(const MaskArg &mk, const FastDiv &fd, uint32_t i0)
{
    const uint32_t plane = fdiv(i0, fd);
    const uint32_t pos = i0 - plane * fd.d;
    const uint32_t sh = plane * mk.w;
    const uint32_t msk = (1u << mk.w) - 1u;
    uint4 m = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int f = 0; f < NL - 1; ++f) {
        const uint4 wd = *reinterpret_cast<const uint4 *>(mk.words + (uint64_t)f * mk.M + pos);
        m.x += ((wd.x >> sh) & msk) == mk.world;
        m.y += ((wd.y >> sh) & msk) == mk.world;
        m.z += ((wd.z >> sh) & msk) == mk.world;
        m.w += ((wd.w >> sh) & msk) == mk.world;
    }
    return m;
}

// T = floor(-|RN(q * S24)|) + (r & 0xFFFFFF); T >> 24 = -xi (qsgd_encode.h)
__device__ __forceinline__ int32_t ms_t(float Ls, uint32_t r) { return add_low24(r, cvt_flr_neg_abs(Ls)); }
// the same as volatile asm: evaluated where written, so a select between two
// T values stays a v_cndmask instead of per-element exec-masked branches
__device__ __forceinline__ int32_t ms_t_v(float Ls, uint32_t r)
{
    int32_t f, o;
    asm volatile("v_cvt_flr_i32_f32_e64 %0, -|%1|" : "=v"(f) : "v"(Ls));
    asm volatile("v_mad_u32_u24 %0, %1, 1, %2" : "=v"(o) : "v"(r), "v"(f));
    return o;
}

// signed Markstein quotient pair RN(x / norm); NEG: -RN(x / norm), bit for
// bit (every step negated: q0' = x (-y) = -q0, e' = fma(norm, q0', x) = e,
// q' = fma(e, -y, q0') = -q; RN is symmetric), at the same cost
template <bool NEG = false>
__device__ __forceinline__ gc_f2 quot2_signed(float a, float b, const DivNorm &d)
{
    const gc_f2 x = {a, b};
    const gc_f2 y = {NEG ? -d.rr : d.rr, NEG ? -d.rr : d.rr};
    const gc_f2 nb = {NEG ? d.norm : -d.norm, NEG ? d.norm : -d.norm};
    const gc_f2 q0 = x * y;
    const gc_f2 e = __builtin_elementwise_fma(nb, q0, x);
    return __builtin_elementwise_fma(e, y, q0);
}

// the fast path's range check, split: the low bound (tiny |x|, where the
// Markstein quotient may be inexact) on the bits, 2 bits(x) - 2 (one
// v_lshl_add per element; +-0 wrap high and pass); the high bound on the
// quotient itself: |q| <= 1 for all four (false for NaN, +-inf and |x| > norm
// alike; where |x| <= norm the quotient is exact, so |q| <= 1 exactly then).
// 11 instructions per quad against RangeI's 14.
struct RangeLo {
    uint32_t mn = 0xffffffffu;
    __device__ __forceinline__ void add4(const float4 &v)
    {
        const uint32_t a = 2u * __float_as_uint(v.x) - 2u, b = 2u * __float_as_uint(v.y) - 2u;
        const uint32_t c = 2u * __float_as_uint(v.z) - 2u, e = 2u * __float_as_uint(v.w) - 2u;
        mn = min(mn, min(min(a, b), min(c, e)));
    }
    __device__ __forceinline__ bool tiny(uint32_t lo2) const { return mn < lo2; }
};

__device__ __forceinline__ bool q_in_unit(const gc_f2 &a, const gc_f2 &b)
{
    return (fabsf(a.x) <= 1.0f) & (fabsf(a.y) <= 1.0f) & (fabsf(b.x) <= 1.0f) & (fabsf(b.y) <= 1.0f);
}

// mask levels of 4 fast-path elements: last level l whose xi_l <= maxv
template <int KIND, int NL, int VAR = 0>
__device__ __forceinline__ uint4 ms_levels4_int(const float4 &v, const DivNorm &dv, const LevelsArg &lv,
                                                const MsFastArg &fa, const RngArgs &rng, uint32_t i0)
{
    const gc_f2 q01 = quot2_signed(v.x, v.y, dv), q23 = quot2_signed(v.z, v.w, dv);
    uint4 m = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int l = 1; l < NL; ++l) {
        const uint4 r = ms_draws4<KIND, VAR>(rng, l, i0);
        const gc_f2 S = {fa.S24[l], fa.S24[l]};
        const gc_f2 a = q01 * S, b = q23 * S;
        m.x = ms_t(a.x, r.x) >= fa.thr ? (uint32_t)l : m.x;
        m.y = ms_t(a.y, r.y) >= fa.thr ? (uint32_t)l : m.y;
        m.z = ms_t(b.x, r.z) >= fa.thr ? (uint32_t)l : m.z;
        m.w = ms_t(b.y, r.w) >= fa.thr ? (uint32_t)l : m.w;
    }
    return m;
}

template <int MODE>
__device__ __forceinline__ float4 load4_nt_tail(const float *__restrict__ x, uint32_t i0, uint32_t n)
{
    if (i0 + 4 <= n)
        return ld_nt(reinterpret_cast<const float4 *>(x + i0));
    float4 v;
    v.x = x[i0];
    v.y = i0 + 1 < n ? x[i0 + 1] : 0.0f;
    v.z = i0 + 2 < n ? x[i0 + 2] : 0.0f;
    v.w = i0 + 3 < n ? x[i0 + 3] : 0.0f;
    return v;
}

__device__ __forceinline__ void st_nt4u(uint32_t *p, const uint4 &v);
// a word quad stored nontemporal (NT) or plain
template <bool NT>
__device__ __forceinline__ void st4u(uint32_t *p, const uint4 &v)
{
    if constexpr (NT)
        st_nt4u(p, v);
    else
        *reinterpret_cast<uint4 *>(p) = v;
}
__device__ __forceinline__ void st_nt4u(uint32_t *p, const uint4 &v)
{
    typedef uint32_t u4v __attribute__((ext_vector_type(4)));
    const u4v r = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(r, reinterpret_cast<u4v *>(p));
}

// lane value qmax + clamp(q, +-qmax): from T of the integer rounding (fast
// path; T >> 24 = -xi) or from q itself (generic path)
__device__ __forceinline__ uint32_t lane_of_t(float x, int32_t T, int32_t qmax)
{
    const int32_t nq = __mul24(T >> 24, med3_i32(__float_as_int(x), -1, 1));  // -q
    return (uint32_t)(qmax - min(max(nq, -qmax), qmax));
}
// the same without the clamp, where |q| <= qmax is known: the W = 1 fused
// fast path (|x| <= norm, and the element's own level has xi <= maxv = qmax)
__device__ __forceinline__ uint32_t lane_of_t_nc(float x, int32_t T, int32_t qmax)
{
    return (uint32_t)(qmax - __mul24(T >> 24, med3_i32(__float_as_int(x), -1, 1)));
}
__device__ __forceinline__ uint32_t lane_of_q(int32_t q, int32_t qmax)
{
    return (uint32_t)(min(max(q, -qmax), qmax) + qmax);
}

// ---------------------------------------------------------------------------
// q cache: the reference's compress_cache (compressors.py:778-797, every
// level's sign*xi as an L x n float32 tensor) in packed form.  Element i
// owns one CBY-byte cell; field l (cb bits at l*cb) = the select's lane value
// at level l, qmax + clamp(q_l, +-qmax).  The mask kernel rounds every level
// anyway except level 0; with the cache it rounds level 0 too and writes the
// cell, and the select reads the cell at the common level instead of x and
// the draws (ms_cache_bytes in multiscale.hip says when the fields fit).
// ---------------------------------------------------------------------------
template <int CBY>
struct CacheCell {
    typedef uint8_t T;
};
template <>
struct CacheCell<2> {
    typedef uint16_t T;
};

// utail = false: the caller knows i0 + 4 <= n (a wave-uniform full tile)
template <int CBY>
__device__ __forceinline__ void cache_store(void *__restrict__ cache, uint32_t i0, uint32_t n, const uint4 &c,
                                            bool utail = true)
{
    typedef typename CacheCell<CBY>::T T;
    T *p = reinterpret_cast<T *>(cache) + i0;
    bool whole = !utail;
    if (!whole) {
        asm volatile("");  // as in mask_plane_d: the per-lane test only in the tail form
        whole = i0 + 4 <= n;
    }
    if (whole) {  // i0 % 4 == 0: 4- / 8-byte aligned
        // v_perm_b32 byte selects: each cell truncated to its CBY bytes (the top
        // field may carry garbage above the cell, mask_plane)
        if constexpr (CBY == 1) {
            const uint32_t lo = __builtin_amdgcn_perm(c.y, c.x, 0x0c0c0400u);  // [x0 y0 0 0]
            const uint32_t hi = __builtin_amdgcn_perm(c.w, c.z, 0x0c0c0400u);  // [z0 w0 0 0]
            *reinterpret_cast<uint32_t *>(p) = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
        } else {
            *reinterpret_cast<uint2 *>(p) = make_uint2(__builtin_amdgcn_perm(c.y, c.x, 0x05040100u),
                                                       __builtin_amdgcn_perm(c.w, c.z, 0x05040100u));
        }
        return;
    }
    p[0] = (T)c.x;
    if (i0 + 1 < n)
        p[1] = (T)c.y;
    if (i0 + 2 < n)
        p[2] = (T)c.z;
}

// the cells of elements i0..i0+3 (0 past n), still packed: CBY = 1 in .x (byte
// e = element e), CBY = 2 in .x / .y (halves).  Unpacked by cache_cells after
// every plane's loads are issued: unpacking inside the load's branch made the
// compiler wait on each load before issuing the next plane's.
template <int CBY>
__device__ __forceinline__ uint2 cache_load(const void *__restrict__ cache, uint32_t i0, uint32_t n)
{
    typedef typename CacheCell<CBY>::T T;
    const T *p = reinterpret_cast<const T *>(cache) + i0;
    if (i0 + 4 <= n) {
        if constexpr (CBY == 1)
            return make_uint2(*reinterpret_cast<const uint32_t *>(p), 0u);
        else
            return *reinterpret_cast<const uint2 *>(p);
    }
    const uint32_t c0 = p[0], c1 = i0 + 1 < n ? p[1] : 0u, c2 = i0 + 2 < n ? p[2] : 0u;
    if constexpr (CBY == 1)
        return make_uint2(c0 | (c1 << 8) | (c2 << 16), 0u);
    else
        return make_uint2(c0 | (c1 << 16), c2);
}

template <int CBY>
__device__ __forceinline__ uint4 cache_cells(const uint2 &u)
{
    if constexpr (CBY == 1)
        return make_uint4(u.x & 0xffu, (u.x >> 8) & 0xffu, (u.x >> 16) & 0xffu, u.x >> 24);
    else
        return make_uint4(u.x & 0xffffu, u.x >> 16, u.y & 0xffffu, u.y >> 16);
}


// ---------------------------------------------------------------------------
// per-plane work (4 elements i0..i0+3 of one plane)
// ---------------------------------------------------------------------------
// resolution levels of 4 elements as thermometer bits: mb[f] = bit or 0 per
// element for [m > f] (0 past n).  CACHE: also the 4 cells into *cv: field l
// (at bit l*cb) = cq + clamp(q_l, +-cq), every level's lane value from the same
// draws and the same fast / generic decision as select_plane, so a cell field
// equals the lane the select would compute at that level.  The fast and generic paths are
// whole branches (each with its own draws), so the common fast path carries
// no per-level divergence.
// DR: the draws, dr(l) = level l's uint4 for elements i0..i0+3 (ms_draws4,
// or an octet kernel's shared blocks)
// utail = false: the caller knows i0 + 4 <= n (a wave-uniform full tile; the
// per-lane tail compares cost about 5 VALU instructions per quad)
template <int NL, int VAR, bool CACHE, typename DR>
__device__ __forceinline__ void mask_plane_d(const float4 &v, uint32_t n, uint32_t i0, const DivNorm &dv,
                                             uint32_t lo2, uint32_t hi2, const LevelsArg &lv, const MsFastArg &fa,
                                             const DR &dr, uint32_t bit, uint4 (&mb)[NL - 1], int32_t cq = 0,
                                             uint32_t cb = 0, uint4 *cv = nullptr, bool utail = true)
{
    RangeLo rg;
    rg.add4(v);
    uint4 c = make_uint4(0u, 0u, 0u, 0u);
    // CACHE: the quotients negated (-q, bit for bit; the fast path's range
    // check and T use |q| only), so their signs are -sign(x) for the cells
    const gc_f2 q01 = quot2_signed<CACHE>(v.x, v.y, dv), q23 = quot2_signed<CACHE>(v.z, v.w, dv);
    if ((VAR & MSV_WIDE) == 0 && ((VAR & MSV_NOSLOW) || (dv.fast && !rg.tiny(lo2) && q_in_unit(q01, q23)))) {
        // cache lanes: q = (T >> 24) * -sign(x) (T >> 24 = -xi; 0 for +-0,
        // whose T is >= 0, so the sign of a zero does not matter); the
        // nonzero fast-path q are normal or subnormal, never 0
        int32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        uint32_t Cf = 0;  // sum_l cq << (l cb): the cells' offsets (uniform)
        if constexpr (CACHE) {
            s0 = med3_i32(__float_as_int(q01.x), -1, 1);
            s1 = med3_i32(__float_as_int(q01.y), -1, 1);
            s2 = med3_i32(__float_as_int(q23.x), -1, 1);
            s3 = med3_i32(__float_as_int(q23.y), -1, 1);
#pragma unroll
            for (int l = 0; l < NL; ++l)
                Cf += (uint32_t)cq << ((uint32_t)l * cb);
        }
        bool k0 = false, k1 = false, k2 = false, k3 = false;  // some level >= l qualifies
#pragma unroll
        for (int l = NL - 1; l >= (CACHE ? 0 : 1); --l) {
            const uint4 r = dr(l);
            const gc_f2 S = {fa.S24[l], fa.S24[l]};
            const gc_f2 a = q01 * S, b = q23 * S;
            const int32_t t0 = ms_t(a.x, r.x), t1 = ms_t(a.y, r.y), t2 = ms_t(b.x, r.z), t3 = ms_t(b.y, r.w);
            if (l > 0) {
                k0 = k0 || t0 >= fa.thr;
                k1 = k1 || t1 >= fa.thr;
                k2 = k2 || t2 >= fa.thr;
                k3 = k3 || t3 >= fa.thr;
                mb[l - 1] = make_uint4(k0 ? bit : 0u, k1 ? bit : 0u, k2 ? bit : 0u, k3 ? bit : 0u);
            }
            if constexpr (CACHE) {
                // c = Cf + sum_l q_l << (l cb): the top level starts it (one
                // v_lshl_add with Cf), level 0 ends it (one v_mad_i32_i24).
                // Level 0 has |q| <= s_0 <= cq (no clamp); the middle levels
                // are clamped (an unchosen level's field is never read, but
                // must not carry into the next field); the top field may hold
                // garbage above its cb bits: nothing reads them and the cell
                // store truncates
                const uint32_t sh = (uint32_t)l * cb;
                int32_t n0 = __mul24(t0 >> 24, s0), n1 = __mul24(t1 >> 24, s1);
                int32_t n2 = __mul24(t2 >> 24, s2), n3 = __mul24(t3 >> 24, s3);
                if (l > 0 && l < NL - 1) {
                    n0 = med3_i32(n0, -cq, cq);
                    n1 = med3_i32(n1, -cq, cq);
                    n2 = med3_i32(n2, -cq, cq);
                    n3 = med3_i32(n3, -cq, cq);
                }
                if (l == NL - 1) {
                    c = make_uint4(((uint32_t)n0 << sh) + Cf, ((uint32_t)n1 << sh) + Cf, ((uint32_t)n2 << sh) + Cf,
                                   ((uint32_t)n3 << sh) + Cf);
                } else {
                    c.x += (uint32_t)n0 << sh;
                    c.y += (uint32_t)n1 << sh;
                    c.z += (uint32_t)n2 << sh;
                    c.w += (uint32_t)n3 << sh;
                }
            }
        }
    } else {
        const float4 ql = quot4_exact(v, dv);
        uint4 m = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int l = CACHE ? 0 : 1; l < NL; ++l) {
            const uint4 r = dr(l);
            const float s = lv.s[l];
            const int32_t x0 = xi_from_q(ql.x, s, r.x), x1 = xi_from_q(ql.y, s, r.y);
            const int32_t x2 = xi_from_q(ql.z, s, r.z), x3 = xi_from_q(ql.w, s, r.w);
            if (l > 0) {
                m.x = x0 <= lv.maxv ? (uint32_t)l : m.x;
                m.y = x1 <= lv.maxv ? (uint32_t)l : m.y;
                m.z = x2 <= lv.maxv ? (uint32_t)l : m.z;
                m.w = x3 <= lv.maxv ? (uint32_t)l : m.w;
            }
            if constexpr (CACHE) {  // the same cells (every level clamped here: exact for the fields)
                const uint32_t sh = (uint32_t)l * cb;
                c.x += lane_of_q(sgn_of(v.x) * x0, cq) << sh;
                c.y += lane_of_q(sgn_of(v.y) * x1, cq) << sh;
                c.z += lane_of_q(sgn_of(v.z) * x2, cq) << sh;
                c.w += lane_of_q(sgn_of(v.w) * x3, cq) << sh;
            }
        }
#pragma unroll
        for (int f = 0; f < NL - 1; ++f)
            mb[f] = make_uint4(m.x > (uint32_t)f ? bit : 0u, m.y > (uint32_t)f ? bit : 0u,
                               m.z > (uint32_t)f ? bit : 0u, m.w > (uint32_t)f ? bit : 0u);
    }
    if (utail) {
        // a wave-uniform branch of its own (the empty asm keeps the compiler
        // from merging it with the per-lane test below and hoisting that
        // test's index arithmetic into the common path)
        asm volatile("");
        if (i0 + 4 > n) {
#pragma unroll
            for (int f = 0; f < NL - 1; ++f) {
                mb[f].y = i0 + 1 < n ? mb[f].y : 0u;
                mb[f].z = i0 + 2 < n ? mb[f].z : 0u;
                mb[f].w = i0 + 3 < n ? mb[f].w : 0u;
            }
        }
    }
    if constexpr (CACHE)
        *cv = c;  // the cells (cache_store truncates them to CBY bytes)
}

template <int KIND, int NL, int VAR = 0, bool CACHE = false>
__device__ __forceinline__ void mask_plane_v(const float4 &v, uint32_t n, uint32_t i0, const DivNorm &dv,
                                             uint32_t lo2, uint32_t hi2, const LevelsArg &lv, const MsFastArg &fa,
                                             const RngArgs &rng, uint32_t bit, uint4 (&mb)[NL - 1], int32_t cq = 0,
                                             uint32_t cb = 0, uint4 *cv = nullptr)
{
    mask_plane_d<NL, VAR, CACHE>(v, n, i0, dv, lo2, hi2, lv, fa,
                                 [&](int l) { return ms_draws4<KIND, VAR>(rng, (uint32_t)l, i0); }, bit, mb, cq, cb,
                                 cv);
}

template <int KIND, int NL, int VAR = 0, bool CACHE = false>
__device__ __forceinline__ void mask_plane(const float *__restrict__ x, uint32_t n, uint32_t i0, const DivNorm &dv,
                                           uint32_t lo2, uint32_t hi2, const LevelsArg &lv, const MsFastArg &fa,
                                           const RngArgs &rng, uint32_t bit, uint4 (&mb)[NL - 1], int32_t cq = 0,
                                           uint32_t cb = 0, uint4 *cv = nullptr)
{
    mask_plane_v<KIND, NL, VAR, CACHE>(load4_nt_tail<0>(x, i0, n), n, i0, dv, lo2, hi2, lv, fa, rng, bit, mb, cq, cb,
                                       cv);
}

// OR the per-element bits of mask_plane into the field accumulators
template <int NL>
__device__ __forceinline__ void mask_or(uint4 (&acc)[NL - 1], const uint4 (&mb)[NL - 1])
{
#pragma unroll
    for (int f = 0; f < NL - 1; ++f) {
        acc[f].x |= mb[f].x;
        acc[f].y |= mb[f].y;
        acc[f].z |= mb[f].z;
        acc[f].w |= mb[f].w;
    }
}

// thermometer bits [m > f] of 4 elements into the field accumulators
template <int NL>
__device__ __forceinline__ void mask_bits(uint4 (&acc)[NL - 1], const uint4 &m, uint32_t sh)
{
#pragma unroll
    for (int f = 0; f < NL - 1; ++f) {
        acc[f].x |= (uint32_t)(m.x > (uint32_t)f) << sh;
        acc[f].y |= (uint32_t)(m.y > (uint32_t)f) << sh;
        acc[f].z |= (uint32_t)(m.z > (uint32_t)f) << sh;
        acc[f].w |= (uint32_t)(m.w > (uint32_t)f) << sh;
    }
}

template <int KIND, int NL, int VAR = 0>
__device__ __forceinline__ uint4 draws_at(const RngArgs &rng, uint32_t i0, uint4 m)
{
    uint4 r = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (uint32_t l = 0; l < (uint32_t)NL; ++l) {
        if (m.x != l && m.y != l && m.z != l && m.w != l)
            continue;
        const uint4 d = ms_draws4<KIND, VAR>(rng, l, i0);
        r.x = m.x == l ? d.x : r.x;
        r.y = m.y == l ? d.y : r.y;
        r.z = m.z == l ? d.z : r.z;
        r.w = m.w == l ? d.w : r.w;
    }
    return r;
}

template <int NL>
__device__ __forceinline__ float pick_level(const float (&a)[GC_MAX_LEVELS], uint32_t m)
{
    float v = a[0];
#pragma unroll
    for (int l = 1; l < NL; ++l)
        v = m == (uint32_t)l ? a[l] : v;
    return v;
}

// lane value q + qmax of one fast-path element at scale S (q clamped to +-qmax)
__device__ __forceinline__ uint32_t ms_lane(float x, float Ls, uint32_t r, int32_t qmax)
{
    return lane_of_t(x, ms_t(Ls, r), qmax);
}

// lane values of 4 elements at levels m, with their draws r at those levels
template <int NL, int VAR = 0>
__device__ __forceinline__ uint4 select_lanes(const float4 &v, const uint4 &m, const uint4 &r, uint32_t n, uint32_t i0,
                                              const DivNorm &dv, uint32_t lo2, const LevelsArg &lv,
                                              const MsFastArg &fa, int32_t qmax)
{
    RangeLo rg;
    rg.add4(v);
    uint4 ln;
    const gc_f2 q01 = quot2_signed(v.x, v.y, dv), q23 = quot2_signed(v.z, v.w, dv);
    if ((VAR & MSV_WIDE) == 0 && ((VAR & MSV_NOSLOW) || (dv.fast && !rg.tiny(lo2) && q_in_unit(q01, q23)))) {
        const gc_f2 S01 = {pick_level<NL>(fa.S24, m.x), pick_level<NL>(fa.S24, m.y)};
        const gc_f2 S23 = {pick_level<NL>(fa.S24, m.z), pick_level<NL>(fa.S24, m.w)};
        const gc_f2 a = q01 * S01, b = q23 * S23;
        ln.x = ms_lane(v.x, a.x, r.x, qmax);
        ln.y = ms_lane(v.y, a.y, r.y, qmax);
        ln.z = ms_lane(v.z, b.x, r.z, qmax);
        ln.w = ms_lane(v.w, b.y, r.w, qmax);
    } else {
        const float4 ql = quot4_exact(v, dv);
        const int32_t q0 = sgn_of(v.x) * xi_from_q(ql.x, pick_level<NL>(lv.s, m.x), r.x);
        const int32_t q1 = sgn_of(v.y) * xi_from_q(ql.y, pick_level<NL>(lv.s, m.y), r.y);
        const int32_t q2 = sgn_of(v.z) * xi_from_q(ql.z, pick_level<NL>(lv.s, m.z), r.z);
        const int32_t q3 = sgn_of(v.w) * xi_from_q(ql.w, pick_level<NL>(lv.s, m.w), r.w);
        ln.x = (uint32_t)(min(max(q0, -qmax), qmax) + qmax);
        ln.y = (uint32_t)(min(max(q1, -qmax), qmax) + qmax);
        ln.z = (uint32_t)(min(max(q2, -qmax), qmax) + qmax);
        ln.w = (uint32_t)(min(max(q3, -qmax), qmax) + qmax);
    }
    if (i0 + 4 > n) {
        ln.y = i0 + 1 < n ? ln.y : 0u;
        ln.z = i0 + 2 < n ? ln.z : 0u;
        ln.w = i0 + 3 < n ? ln.w : 0u;
    }
    return ln;
}

// lane values of 4 elements at their common levels (0 past n)
template <int KIND, int NL, int VAR = 0>
__device__ __forceinline__ uint4 select_plane(const float *__restrict__ x, uint32_t n, uint32_t i0,
                                              const MaskArg &mk, const FastDiv &fd, const DivNorm &dv, uint32_t lo2,
                                              uint32_t hi2, const LevelsArg &lv, const MsFastArg &fa,
                                              const RngArgs &rng, int32_t qmax)
{
    const float4 v = load4_nt_tail<0>(x, i0, n);
    const uint4 m = mask_levels4_fast<NL>(mk, fd, i0);
    const uint4 r = draws_at<KIND, NL, VAR>(rng, i0, m);  // the selected level's draw, either path
    return select_lanes<NL, VAR>(v, m, r, n, i0, dv, lo2, lv, fa, qmax);
}

// decoded floats of 4 elements (compressors.py:819-826 order 0; 668-680 order 1) * alpha
template <int ORDER, int NL, bool NTS = true>
__device__ __forceinline__ void decode_plane(const uint4 &wd, uint32_t sh, uint32_t msk, int32_t sub, const uint4 &m,
                                             float norm, const LevelsArg &lv, const MsFastArg &fa,
                                             const float (&c)[GC_MAX_LEVELS], bool mk0, float alpha,
                                             float *__restrict__ out, uint32_t i0, uint32_t n)
{
    float4 o;
    float *op = &o.x;
    const uint32_t *wp = &wd.x;
    const uint32_t *mp = &m.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int32_t Q = (int32_t)((wp[e] >> sh) & msk) - sub;
        float d;
        if constexpr (ORDER == 1) {
            d = pick_level<NL>(c, mp[e]) * (float)Q;
        } else {
            const float a = (float)Q * norm;
            const float s = pick_level<NL>(lv.s, mp[e]);
            if (mk0) {
                const float y = pick_level<NL>(fa.y, mp[e]);
                const float q0 = a * y;
                d = fmaf(fmaf(-s, q0, a), y, q0);
            } else {
                d = a / s;
            }
        }
        op[e] = d * alpha;
    }
    if (i0 + 4 <= n) {
        if constexpr (NTS)
            st_nt4(out + i0, o);
        else
            *reinterpret_cast<float4 *>(out + i0) = o;
    } else {
        for (int e = 0; e < 4; ++e)
            if (i0 + e < n)
                out[i0 + e] = pickf(o, e);
    }
}

constexpr uint32_t kMsQuadsPerBlock = 64;  // word quads per block (one per lane; 4 waves split the planes)

// ---------------------------------------------------------------------------
// mask encode: thermometer fields of the resolution level (compressors.py:799-807)
// ---------------------------------------------------------------------------
// CBY = 0: mask only; 1 / 2: also the q cache cells (CBY bytes per element)
// GC_MS_WPE (measurement builds only: hipcc -DGC_MS_WPE=N of tools/lab_ms.hip): pin the
// Philox-bound kernels' occupancy with amdgpu_waves_per_eu
#ifdef GC_MS_WPE
#define GC_MS_OCC __attribute__((amdgpu_waves_per_eu(GC_MS_WPE, GC_MS_WPE)))
#else
#define GC_MS_OCC
#endif

template <int LM, int KIND, int NL, int VAR = 0, int CBY = 0>
__global__ GC_MS_OCC __launch_bounds__(kBlock) void k_ms_mask_fast(const float *__restrict__ x, uint32_t n,
                                                         const float *__restrict__ normp, LevelsArg lv, MsFastArg fa,
                                                         RngArgs rng, uint32_t M, uint32_t w, uint32_t fields,
                                                         uint32_t *__restrict__ mask_words, void *__restrict__ cache = nullptr,
                                                         int32_t cq = 0, uint32_t cb = 0)
{
    static_assert(CBY == 0 || (VAR & MSV_PERTHREAD) == 0, "the q cache is written by the wave-split kernel only");
    const float norm = *normp;
    const DivNorm dv = make_div(norm);
    const uint32_t lo2 = 2u * dv.lo1, hi2 = 2u * __float_as_uint(norm);
    const uint32_t quads = M >> 2;
    if constexpr ((VAR & MSV_PERTHREAD) != 0) {
        for (uint32_t t = blockIdx.x * kBlock + threadIdx.x; t < quads; t += gridDim.x * kBlock) {
            uint4 acc[NL - 1] = {};
#pragma unroll
            for (int j = 0; j < LM; ++j) {
                const uint32_t i0 = (uint32_t)j * M + 4u * t;
                if (i0 >= n)
                    break;
                uint4 mb[NL - 1];
                mask_plane<KIND, NL, VAR>(x, n, i0, dv, lo2, hi2, lv, fa, rng, 1u << ((uint32_t)j * w), mb);
                mask_or<NL>(acc, mb);
            }
#pragma unroll
            for (int f = 0; f < NL - 1; ++f)
                st_nt4u(mask_words + (uint64_t)f * M + 4u * t, acc[f]);
        }
        return;
    }
    constexpr int PW = (LM + 3) / 4;  // planes per wave
    __shared__ uint4 part[3][kMsQuadsPerBlock];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    for (uint32_t tb = blockIdx.x * kMsQuadsPerBlock; tb < quads; tb += gridDim.x * kMsQuadsPerBlock) {
        const uint32_t t = tb + lane;
        uint4 acc[NL - 1] = {};
        if (t < quads) {
#pragma unroll
            for (int j = 0; j < PW; ++j) {
                const uint32_t p = wave + 4u * j;
                if (p >= (uint32_t)LM)
                    break;
                const uint32_t i0 = p * M + 4u * t;
                if (i0 >= n)
                    break;
                if constexpr (CBY != 0) {
                    uint4 cv, mb[NL - 1];
                    mask_plane<KIND, NL, VAR, true>(x, n, i0, dv, lo2, hi2, lv, fa, rng, 1u << (p * w), mb, cq, cb, &cv);
                    cache_store<CBY>(cache, i0, n, cv);
                    mask_or<NL>(acc, mb);
                } else {
                    uint4 mb[NL - 1];
                    mask_plane<KIND, NL, VAR>(x, n, i0, dv, lo2, hi2, lv, fa, rng, 1u << (p * w), mb);
                    mask_or<NL>(acc, mb);
                }
            }
        }
#pragma unroll
        for (int f = 0; f < NL - 1; ++f) {
            if (wave)
                part[wave - 1][lane] = acc[f];
            __syncthreads();
            if (wave == 0 && t < quads) {
                const uint4 a = part[0][lane], b = part[1][lane], c = part[2][lane];
                st_nt4u(mask_words + (uint64_t)f * M + 4u * t,
                        make_uint4(acc[f].x | a.x | b.x | c.x, acc[f].y | a.y | b.y | c.y,
                                   acc[f].z | a.z | b.z | c.z, acc[f].w | a.w | b.w | c.w));
            }
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------------------
// select encode: q at each element's common level, packed (compressors.py:809-817)
// ---------------------------------------------------------------------------
template <int LQ, int KIND, int NL, int VAR = 0>
__global__ __launch_bounds__(kBlock) void k_ms_select_fast(const float *__restrict__ x, uint32_t n,
                                                           const float *__restrict__ normp, LevelsArg lv,
                                                           MsFastArg fa, RngArgs rng, MaskArg mk, FastDiv fd,
                                                           uint32_t Mq, uint32_t wq, int32_t qmax,
                                                           uint32_t *__restrict__ words)
{
    const float norm = *normp;
    const DivNorm dv = make_div(norm);
    const uint32_t lo2 = 2u * dv.lo1, hi2 = 2u * __float_as_uint(norm);
    const uint32_t quads = Mq >> 2;
    if constexpr ((VAR & MSV_PERTHREAD) != 0) {
        for (uint32_t t = blockIdx.x * kBlock + threadIdx.x; t < quads; t += gridDim.x * kBlock) {
            uint4 acc = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (int k = 0; k < LQ; ++k) {
                const uint32_t i0 = (uint32_t)k * Mq + 4u * t;
                if (i0 >= n)
                    break;
                const uint4 ln = select_plane<KIND, NL, VAR>(x, n, i0, mk, fd, dv, lo2, hi2, lv, fa, rng, qmax);
                const uint32_t sh = (uint32_t)k * wq;
                acc.x += ln.x << sh;
                acc.y += ln.y << sh;
                acc.z += ln.z << sh;
                acc.w += ln.w << sh;
            }
            st_nt4u(words + 4u * t, acc);
        }
        return;
    }
    constexpr int PW = (LQ + 3) / 4;
    __shared__ uint4 part[3][kMsQuadsPerBlock];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    for (uint32_t tb = blockIdx.x * kMsQuadsPerBlock; tb < quads; tb += gridDim.x * kMsQuadsPerBlock) {
        const uint32_t t = tb + lane;
        uint4 acc = make_uint4(0u, 0u, 0u, 0u);
        if (t < quads) {
#pragma unroll
            for (int j = 0; j < PW; ++j) {
                const uint32_t p = wave + 4u * j;
                if (p >= (uint32_t)LQ)
                    break;
                const uint32_t i0 = p * Mq + 4u * t;
                if (i0 >= n)
                    break;
                const uint4 ln = select_plane<KIND, NL, VAR>(x, n, i0, mk, fd, dv, lo2, hi2, lv, fa, rng, qmax);
                const uint32_t sh = p * wq;
                acc.x += ln.x << sh;
                acc.y += ln.y << sh;
                acc.z += ln.z << sh;
                acc.w += ln.w << sh;
            }
        }
        if (wave)
            part[wave - 1][lane] = acc;
        __syncthreads();
        if (wave == 0 && t < quads) {
            const uint4 a = part[0][lane], b = part[1][lane], c = part[2][lane];
            st_nt4u(words + 4u * t, make_uint4(acc.x + a.x + b.x + c.x, acc.y + a.y + b.y + c.y,
                                               acc.z + a.z + b.z + c.z, acc.w + a.w + b.w + c.w));
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// select from the q cache (compressors.py:809-817 compress(mask): q[m==i] =
// cache[i][m==i]): per element one cell and the common level, no x, no draws
// ---------------------------------------------------------------------------
template <int LQ, int NL, int CBY>
__global__ __launch_bounds__(kBlock) void k_ms_select_cache(const void *__restrict__ cache, uint32_t n, MaskArg mk,
                                                            FastDiv fd, uint32_t Mq, uint32_t wq, uint32_t cb,
                                                            uint32_t *__restrict__ words)
{
    const uint32_t cm = (1u << cb) - 1u;
    const uint32_t quads = Mq >> 2;
    constexpr int PW = (LQ + 3) / 4;
    __shared__ uint4 part[3][kMsQuadsPerBlock];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    for (uint32_t tb = blockIdx.x * kMsQuadsPerBlock; tb < quads; tb += gridDim.x * kMsQuadsPerBlock) {
        const uint32_t t = tb + lane;
        uint4 acc = make_uint4(0u, 0u, 0u, 0u);
        if (t < quads) {
            // every plane's cells and mask words are loaded before any is used
            // (short, latency-bound planes: no load -> use -> load chains)
            uint2 c[PW];
            uint4 mw[PW][NL - 1];
            uint32_t shm[PW];
#pragma unroll
            for (int j = 0; j < PW; ++j) {
                const uint32_t p = wave + 4u * j;
                const uint32_t i0 = p * Mq + 4u * t;
                c[j] = make_uint2(0u, 0u);
                shm[j] = 0;
#pragma unroll
                for (int f = 0; f < NL - 1; ++f)
                    mw[j][f] = make_uint4(0u, 0u, 0u, 0u);
                if (p < (uint32_t)LQ && i0 < n) {
                    c[j] = cache_load<CBY>(cache, i0, n);
                    const uint32_t plane = fdiv(i0, fd);
                    const uint32_t pos = i0 - plane * fd.d;
                    shm[j] = plane * mk.w;
#pragma unroll
                    for (int f = 0; f < NL - 1; ++f)
                        mw[j][f] = *reinterpret_cast<const uint4 *>(mk.words + (uint64_t)f * mk.M + pos);
                }
            }
            const uint32_t msk = (1u << mk.w) - 1u;
#pragma unroll
            for (int j = 0; j < PW; ++j) {
                const uint4 cj = cache_cells<CBY>(c[j]);
                uint4 m = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
                for (int f = 0; f < NL - 1; ++f) {  // common level = #fields whose W-sum == W (mask_levels4_fast)
                    m.x += ((mw[j][f].x >> shm[j]) & msk) == mk.world;
                    m.y += ((mw[j][f].y >> shm[j]) & msk) == mk.world;
                    m.z += ((mw[j][f].z >> shm[j]) & msk) == mk.world;
                    m.w += ((mw[j][f].w >> shm[j]) & msk) == mk.world;
                }
                const uint32_t p = wave + 4u * j;  // planes past LQ / n contribute c = 0
                const uint32_t sh = p < (uint32_t)LQ ? p * wq : 0u;
                acc.x += ((cj.x >> (m.x * cb)) & cm) << sh;
                acc.y += ((cj.y >> (m.y * cb)) & cm) << sh;
                acc.z += ((cj.z >> (m.z * cb)) & cm) << sh;
                acc.w += ((cj.w >> (m.w * cb)) & cm) << sh;
            }
        }
        if (wave)
            part[wave - 1][lane] = acc;
        __syncthreads();
        if (wave == 0 && t < quads) {
            const uint4 a = part[0][lane], b = part[1][lane], c = part[2][lane];
            st_nt4u(words + 4u * t, make_uint4(acc.x + a.x + b.x + c.x, acc.y + a.y + b.y + c.y,
                                               acc.z + a.z + b.z + c.z, acc.w + a.w + b.w + c.w));
        }
        __syncthreads();
    }
}

// the same with two adjacent word quads per lane (8 elements of a plane: one
// 8- / 16-byte cell load, twice the bytes in flight per wave; Mq % 8 == 0)
template <int LQ, int NL, int CBY, bool NTS = true>
__global__ __launch_bounds__(kBlock) void k_ms_select_cache_o2(const void *__restrict__ cache, uint32_t n, MaskArg mk,
                                                               FastDiv fd, uint32_t Mq, uint32_t wq, uint32_t cb,
                                                               uint32_t *__restrict__ words)
{
    const uint32_t cm = (1u << cb) - 1u;
    const uint32_t octs = Mq >> 3;
    constexpr int PW = (LQ + 3) / 4;
    __shared__ uint4 part[3][2][kMsQuadsPerBlock];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    typedef typename CacheCell<CBY>::T T;
    for (uint32_t tb = blockIdx.x * kMsQuadsPerBlock; tb < octs; tb += gridDim.x * kMsQuadsPerBlock) {
        const uint32_t t = tb + lane;
        uint4 acc[2] = {};
        if (t < octs) {
            // every plane's cells and mask words are loaded before any is used
            uint2 c[PW][2];
            uint4 mw[PW][2][NL - 1];
            uint32_t shm[PW][2];
#pragma unroll
            for (int j = 0; j < PW; ++j) {
                const uint32_t p = wave + 4u * j;
                const uint32_t i0 = p * Mq + 8u * t;
#pragma unroll
                for (int hq = 0; hq < 2; ++hq) {
                    c[j][hq] = make_uint2(0u, 0u);
                    shm[j][hq] = 0;
#pragma unroll
                    for (int f = 0; f < NL - 1; ++f)
                        mw[j][hq][f] = make_uint4(0u, 0u, 0u, 0u);
                }
                if (p < (uint32_t)LQ && i0 < n) {
                    if (i0 + 8 <= n) {  // 8 cells in one load (i0 % 8 == 0: 8 CBY-byte aligned)
                        const T *cp = reinterpret_cast<const T *>(cache) + i0;
                        if constexpr (CBY == 1) {
                            const uint2 u = *reinterpret_cast<const uint2 *>(cp);
                            c[j][0] = make_uint2(u.x, 0u);
                            c[j][1] = make_uint2(u.y, 0u);
                        } else {
                            const uint4 u = *reinterpret_cast<const uint4 *>(cp);
                            c[j][0] = make_uint2(u.x, u.y);
                            c[j][1] = make_uint2(u.z, u.w);
                        }
                    } else {
                        c[j][0] = cache_load<CBY>(cache, i0, n);
                        if (i0 + 4 < n)
                            c[j][1] = cache_load<CBY>(cache, i0 + 4, n);
                    }
#pragma unroll
                    for (int hq = 0; hq < 2; ++hq) {
                        const uint32_t iq = i0 + 4u * hq;
                        if (hq == 1 && iq >= n)
                            break;
                        const uint32_t plane = fdiv(iq, fd);
                        const uint32_t pos = iq - plane * fd.d;
                        shm[j][hq] = plane * mk.w;
#pragma unroll
                        for (int f = 0; f < NL - 1; ++f)
                            mw[j][hq][f] = *reinterpret_cast<const uint4 *>(mk.words + (uint64_t)f * mk.M + pos);
                    }
                }
            }
            const uint32_t msk = (1u << mk.w) - 1u;
#pragma unroll
            for (int j = 0; j < PW; ++j) {
                const uint32_t p = wave + 4u * j;  // planes past LQ / n contribute c = 0
                const uint32_t sh = p < (uint32_t)LQ ? p * wq : 0u;
#pragma unroll
                for (int hq = 0; hq < 2; ++hq) {
                    const uint4 cj = cache_cells<CBY>(c[j][hq]);
                    uint4 m = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
                    for (int f = 0; f < NL - 1; ++f) {
                        m.x += ((mw[j][hq][f].x >> shm[j][hq]) & msk) == mk.world;
                        m.y += ((mw[j][hq][f].y >> shm[j][hq]) & msk) == mk.world;
                        m.z += ((mw[j][hq][f].z >> shm[j][hq]) & msk) == mk.world;
                        m.w += ((mw[j][hq][f].w >> shm[j][hq]) & msk) == mk.world;
                    }
                    acc[hq].x += ((cj.x >> (m.x * cb)) & cm) << sh;
                    acc[hq].y += ((cj.y >> (m.y * cb)) & cm) << sh;
                    acc[hq].z += ((cj.z >> (m.z * cb)) & cm) << sh;
                    acc[hq].w += ((cj.w >> (m.w * cb)) & cm) << sh;
                }
            }
        }
        if (wave) {
            part[wave - 1][0][lane] = acc[0];
            part[wave - 1][1][lane] = acc[1];
        }
        __syncthreads();
        if (wave == 0 && t < octs) {
#pragma unroll
            for (int hq = 0; hq < 2; ++hq) {
                const uint4 a = part[0][hq][lane], b = part[1][hq][lane], c = part[2][hq][lane];
                st4u<NTS>(words + 8u * t + 4u * hq, make_uint4(acc[hq].x + a.x + b.x + c.x, acc[hq].y + a.y + b.y + c.y,
                                                               acc[hq].z + a.z + b.z + c.z, acc[hq].w + a.w + b.w + c.w));
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// W = 1: mask + select in ONE pass (compressors.py:778-817 with the MIN
// all-reduce of reducer.py:1680 over a single rank, the identity: the common
// level is the rank's own).  Per 4 elements: the levels 1..NL-1 decide the
// mask, the chosen level's rounding is kept, and level 0's draw block is
// computed only when an element stays at level 0 — the same draws,
// arithmetic and decisions as mask_plane + select_plane, so both streams are
// bit-identical to the two-pass encode.
//
// Work split: the coupled W = 1 layouts (gc_ms_mask_layout) make mask plane
// P = h + r k the q lane k of q words h Mm + pos, so a block of r waves owns
// 64 mask word quads, and wave h owns q stream h: it walks the Lq planes
// P = h + r k of its quad column and assembles its q words in registers — no
// LDS traffic for the q lanes; only the mask words (one bit per plane) are
// OR-ed across the r waves.  The plane index is wave-uniform (scalar).
// ---------------------------------------------------------------------------
// fast path of 4 elements: the thermometer bits (field f = [m > f], as bitP
// or 0) and -q at the chosen level m.  T at level l is ms_t (T >> 24 = -xi);
// levels above 0 may exceed 7 bits: their T saturates (v_cvt_flr_i32_f32
// clamps) once |Ls| > 2^31, i.e. xi >= 128 > maxv, which is exactly "not this
// level"; a level is only ever chosen with xi <= maxv <= 127, so the chosen
// T >> 24 is a sign-extended byte.  -q = (T >> 24) * sign(x) (0 for +-0,
// whose T is >= 0 anyway).
template <int NL, int VAR, typename DR>
__device__ __forceinline__ void fused_quad_fast(const float4 &v, const gc_f2 &q01, const gc_f2 &q23,
                                                const MsFastArg &fa, const DR &dr, uint32_t bitP,
                                                uint4 (&mb)[NL - 1], int4 &nq)
{
    uint4 r0e;
    if constexpr ((VAR & MSV_EAGER0) != 0)
        r0e = dr(0);  // independent of the upper levels': the chains interleave
    int4 T;
    bool k0 = false, k1 = false, k2 = false, k3 = false;  // some level >= 1 qualifies
#pragma unroll
    for (int l = NL - 1; l >= 1; --l) {  // the highest qualifying level wins
        const uint4 r = dr(l);
        const gc_f2 S = {fa.S24[l], fa.S24[l]};
        const gc_f2 a = q01 * S, b = q23 * S;
        const int32_t u0 = ms_t_v(a.x, r.x), u1 = ms_t_v(a.y, r.y), u2 = ms_t_v(b.x, r.z), u3 = ms_t_v(b.y, r.w);
        const bool c0 = u0 >= fa.thr, c1 = u1 >= fa.thr, c2 = u2 >= fa.thr, c3 = u3 >= fa.thr;
        if (l == NL - 1) {
            T = make_int4(u0, u1, u2, u3);
        } else {
            T.x = k0 ? T.x : u0;
            T.y = k1 ? T.y : u1;
            T.z = k2 ? T.z : u2;
            T.w = k3 ? T.w : u3;
        }
        k0 = k0 || c0;
        k1 = k1 || c1;
        k2 = k2 || c2;
        k3 = k3 || c3;
        // field f = l - 1: [m >= l] = some level >= l qualifies
        mb[l - 1] = make_uint4(k0 ? bitP : 0u, k1 ? bitP : 0u, k2 ? bitP : 0u, k3 ? bitP : 0u);
    }
    if ((VAR & MSV_EAGER0) != 0 || !(k0 && k1 && k2 && k3)) {  // level 0's draws only when an element stays there
        uint4 r;
        if constexpr ((VAR & MSV_EAGER0) != 0)
            r = r0e;
        else
            r = dr(0);
        const gc_f2 S = {fa.S24[0], fa.S24[0]};
        const gc_f2 a = q01 * S, b = q23 * S;
        const int32_t w0 = ms_t_v(a.x, r.x), w1 = ms_t_v(a.y, r.y), w2 = ms_t_v(b.x, r.z), w3 = ms_t_v(b.y, r.w);
        T.x = k0 ? T.x : w0;
        T.y = k1 ? T.y : w1;
        T.z = k2 ? T.z : w2;
        T.w = k3 ? T.w : w3;
    }
    nq.x = __mul24(T.x >> 24, med3_i32(__float_as_int(v.x), -1, 1));
    nq.y = __mul24(T.y >> 24, med3_i32(__float_as_int(v.y), -1, 1));
    nq.z = __mul24(T.z >> 24, med3_i32(__float_as_int(v.z), -1, 1));
    nq.w = __mul24(T.w >> 24, med3_i32(__float_as_int(v.w), -1, 1));
}

// generic path of 4 elements (range-check failures, norms outside the
// Markstein range, MSV_WIDE): the same bits and -q from the per-element rounding
template <int NL, int VAR, typename DR>
__device__ __forceinline__ void fused_quad_slow(const float4 &v, const DivNorm &dv, const LevelsArg &lv,
                                                const DR &dr, uint32_t bitP, uint4 (&mb)[NL - 1], int4 &nq,
                                                int32_t qmax)
{
    const float4 ql = quot4_exact(v, dv);
    uint4 m = make_uint4(0u, 0u, 0u, 0u);
    int4 q = make_int4(0, 0, 0, 0);
#pragma unroll
    for (int l = 1; l < NL; ++l) {
        const uint4 r = dr(l);
        const float s = lv.s[l];
        const int32_t x0 = xi_from_q(ql.x, s, r.x), x1 = xi_from_q(ql.y, s, r.y);
        const int32_t x2 = xi_from_q(ql.z, s, r.z), x3 = xi_from_q(ql.w, s, r.w);
        if (x0 <= lv.maxv) { m.x = l; q.x = sgn_of(v.x) * x0; }
        if (x1 <= lv.maxv) { m.y = l; q.y = sgn_of(v.y) * x1; }
        if (x2 <= lv.maxv) { m.z = l; q.z = sgn_of(v.z) * x2; }
        if (x3 <= lv.maxv) { m.w = l; q.w = sgn_of(v.w) * x3; }
    }
    if (m.x == 0u || m.y == 0u || m.z == 0u || m.w == 0u) {
        const uint4 r = dr(0);
        const float s = lv.s[0];
        q.x = m.x == 0u ? sgn_of(v.x) * xi_from_q(ql.x, s, r.x) : q.x;
        q.y = m.y == 0u ? sgn_of(v.y) * xi_from_q(ql.y, s, r.y) : q.y;
        q.z = m.z == 0u ? sgn_of(v.z) * xi_from_q(ql.z, s, r.z) : q.z;
        q.w = m.w == 0u ? sgn_of(v.w) * xi_from_q(ql.w, s, r.w) : q.w;
    }
#pragma unroll
    for (int f = 0; f < NL - 1; ++f)
        mb[f] = make_uint4(m.x > (uint32_t)f ? bitP : 0u, m.y > (uint32_t)f ? bitP : 0u,
                           m.z > (uint32_t)f ? bitP : 0u, m.w > (uint32_t)f ? bitP : 0u);
    // |x| > norm (a caller's norm below max |x|, or inf) saturates at +-qmax
    // like the two-pass select's lane_of_q; an unclamped q would carry into
    // the word's other lanes
    nq = make_int4(-med3_i32(q.x, -qmax, qmax), -med3_i32(q.y, -qmax, qmax), -med3_i32(q.z, -qmax, qmax),
                   -med3_i32(q.w, -qmax, qmax));
}

constexpr uint32_t kMsFusedMaxR = 8;  // q words per mask word at W = 1: 32 / (q lanes per word) <= 8

// one plane of the fused encode: the thermometer bits into the mask fields,
// -q * 2^(k wq) into the wave's q word accumulator (word = C - acc, modular:
// lane = qmax + q).  Elements past n have x = 0 (no lane) and no mask bit.
template <int NL>
__device__ __forceinline__ void fused_accumulate(uint32_t n, uint32_t i0, uint32_t sh, uint4 (&mb)[NL - 1],
                                                 const int4 &nq, uint4 (&macc)[NL - 1], uint4 &acc)
{
    if (i0 + 4 > n) {
#pragma unroll
        for (int f = 0; f < NL - 1; ++f) {
            mb[f].x = i0 < n ? mb[f].x : 0u;
            mb[f].y = i0 + 1 < n ? mb[f].y : 0u;
            mb[f].z = i0 + 2 < n ? mb[f].z : 0u;
            mb[f].w = i0 + 3 < n ? mb[f].w : 0u;
        }
    }
#pragma unroll
    for (int f = 0; f < NL - 1; ++f) {
        macc[f].x |= mb[f].x;
        macc[f].y |= mb[f].y;
        macc[f].z |= mb[f].z;
        macc[f].w |= mb[f].w;
    }
    acc.x += (uint32_t)nq.x << sh;
    acc.y += (uint32_t)nq.y << sh;
    acc.z += (uint32_t)nq.z << sh;
    acc.w += (uint32_t)nq.w << sh;
}

template <int NL, int VAR, typename DR>
__device__ __forceinline__ void fused_plane_d(const float4 &v, uint32_t n, uint32_t i0, const DivNorm &dv,
                                              uint32_t lo2, const LevelsArg &lv, const MsFastArg &fa, const DR &dr,
                                              uint32_t bitP, uint32_t sh, uint4 (&macc)[NL - 1], uint4 &acc,
                                              int32_t qmax)
{
    RangeLo rg;
    rg.add4(v);
    uint4 mb[NL - 1];
    int4 nq;
    const gc_f2 q01 = quot2_signed(v.x, v.y, dv), q23 = quot2_signed(v.z, v.w, dv);
    if ((VAR & MSV_WIDE) == 0 && ((VAR & MSV_NOSLOW) || (dv.fast && !rg.tiny(lo2) && q_in_unit(q01, q23))))
        fused_quad_fast<NL, VAR>(v, q01, q23, fa, dr, bitP, mb, nq);
    else
        fused_quad_slow<NL, VAR>(v, dv, lv, dr, bitP, mb, nq, qmax);
    fused_accumulate<NL>(n, i0, sh, mb, nq, macc, acc);
}

template <int KIND, int NL, int VAR>
__device__ __forceinline__ void fused_plane_r(const float4 &v, uint32_t n, uint32_t i0, const DivNorm &dv,
                                              uint32_t lo2, uint32_t hi2, const LevelsArg &lv, const MsFastArg &fa,
                                              const RngArgs &rng, uint32_t bitP, uint32_t sh,
                                              uint4 (&macc)[NL - 1], uint4 &acc, int32_t qmax)
{
    fused_plane_d<NL, VAR>(v, n, i0, dv, lo2, lv, fa,
                           [&](int l) { return ms_draws4<KIND, VAR>(rng, (uint32_t)l, i0); }, bitP, sh, macc, acc,
                           qmax);
}

__device__ __forceinline__ float4 load4_guard(const float *__restrict__ x, uint32_t i0, uint32_t n)
{
    return i0 < n ? load4_nt_tail<0>(x, i0, n) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

// blockDim = 64 r (r <= kMsFusedMaxR waves); wave h walks planes h + r k, k < Lq.
// U planes' loads are issued together before their math (U = 1: one plane at
// a time): a wave's chain of dependent plane loads is what bounds the kernel
// (at 7 waves per SIMD and one 1 KB load in flight per wave, Little's law
// gives about the 3.2 TB/s it reaches), so U > 1 keeps U KB in flight per wave.
template <int KIND, int NL, int VAR = 0, int U = 1>
__global__ GC_MS_OCC __launch_bounds__(64 * kMsFusedMaxR) void k_ms_fused_w1(const float *__restrict__ x, uint32_t n,
                                                                 const float *__restrict__ normp, LevelsArg lv,
                                                                 MsFastArg fa, RngArgs rng, uint32_t Mm, uint32_t r,
                                                                 uint32_t Lq, uint32_t wq, int32_t qmax, uint32_t Cw,
                                                                 uint32_t pend, uint32_t *__restrict__ mask_words,
                                                                 uint32_t *__restrict__ words)
{
    // host-computed: Cw = sum_k qmax << (k wq) (the lane offsets of a full
    // word), pend = ceil(n / Mm) (mask planes holding any element).  A block
    // walks several tiles (grid-stride), so this prologue is paid per block
    const float norm = *normp;
    const DivNorm dv = make_div(norm);
    const uint32_t lo2 = 2u * dv.lo1, hi2 = 2u * __float_as_uint(norm);
    const uint32_t quads = Mm >> 2;
    const uint32_t h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    // planes k < kfull are full for every lane (their end (P + 1) Mm <=
    // (pend - 1) Mm < n: plain 16-byte loads, no per-lane guard); planes
    // k < kend hold elements (P < pend)
    const uint32_t kend = h < pend ? min(Lq, (pend - h + r - 1) / r) : 0u;
    const uint32_t kfull = h + 1 < pend ? min(kend, (pend - 1 - h + r - 1) / r) : 0u;
    __shared__ uint4 part[kMsFusedMaxR - 1][NL - 1][kMsQuadsPerBlock];
    for (uint32_t tb = blockIdx.x * kMsQuadsPerBlock; tb < quads; tb += gridDim.x * kMsQuadsPerBlock) {
        const uint32_t t = tb + lane;
        uint4 macc[NL - 1] = {};
        uint4 acc = make_uint4(0u, 0u, 0u, 0u);
        if (t < quads) {
            uint32_t i0 = h * Mm + 4u * t;
            const uint32_t step = r * Mm;
            uint32_t k = 0;
            if constexpr (U > 1) {
#pragma unroll 1
                for (; k + U <= kfull; k += U) {
                    float4 xv[U];
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        xv[u] = ld_nt(reinterpret_cast<const float4 *>(x + i0 + u * step));
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        fused_plane_r<KIND, NL, VAR>(xv[u], n, i0 + u * step, dv, lo2, hi2, lv, fa, rng,
                                                     1u << (h + r * (k + u)), (k + u) * wq, macc, acc, qmax);
                    i0 += U * step;
                }
            }
#pragma unroll 1
            for (; k < kend; ++k) {
                const float4 v = k < kfull ? ld_nt(reinterpret_cast<const float4 *>(x + i0)) : load4_guard(x, i0, n);
                fused_plane_r<KIND, NL, VAR>(v, n, i0, dv, lo2, hi2, lv, fa, rng, 1u << (h + r * k), k * wq, macc, acc,
                                             qmax);
                i0 += step;
            }
        }
        // q words of stream h: quad t at j0 = h Mm + 4t, lane k = element j0 + e + k Mq
        if (t < quads) {
            const uint64_t j0 = (uint64_t)h * Mm + 4u * t, Mq = (uint64_t)r * Mm;
            uint4 C = make_uint4(Cw, Cw, Cw, Cw);
            if (j0 + 3 + (uint64_t)(Lq - 1) * Mq >= n) {  // lanes of elements past n stay 0
                C = make_uint4(0u, 0u, 0u, 0u);
                for (uint32_t k = 0; k < Lq; ++k) {
                    const uint64_t e = j0 + (uint64_t)k * Mq;
                    const uint32_t c = (uint32_t)qmax << (k * wq);
                    C.x += e < n ? c : 0u;
                    C.y += e + 1 < n ? c : 0u;
                    C.z += e + 2 < n ? c : 0u;
                    C.w += e + 3 < n ? c : 0u;
                }
            }
            st_nt4u(words + j0, make_uint4(C.x - acc.x, C.y - acc.y, C.z - acc.z, C.w - acc.w));
        }
        // mask words: OR of the r waves' plane bits
        if (h)
#pragma unroll
            for (int f = 0; f < NL - 1; ++f)
                part[h - 1][f][lane] = macc[f];
        __syncthreads();
        if (h == 0 && t < quads) {
#pragma unroll
            for (int f = 0; f < NL - 1; ++f) {
                uint4 o = macc[f];
                for (uint32_t q = 0; q + 1 < r; ++q) {
                    const uint4 a = part[q][f][lane];
                    o = make_uint4(o.x | a.x, o.y | a.y, o.z | a.z, o.w | a.w);
                }
                st_nt4u(mask_words + (uint64_t)f * Mm + 4u * t, o);
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Octet kernels: 2 levels with the dense Philox stream (draws4<2>, gc_device.h).
// A lane owns 2 adjacent word quads of a plane, i.e. the 8 elements of one
// draw group (plane sizes that are multiples of 8 words: the host checks), so
// one ms2_octet (3 Philox blocks) gives both levels' draws of all 8, against
// 2 blocks per quad (4 per octet) of the per-quad kernels above.  The mask
// without the q cache needs level 1 only (ms2_octet_level, 2 blocks per octet,
// no worse than per quad).  Same outputs as the per-quad kernels with KIND 2,
// bit for bit: the per-element arithmetic is the same code (mask_plane_d,
// fused_plane_d, select_lanes), only the draws are shared.
// ---------------------------------------------------------------------------
// the octet at element i0 (i0 % 8 == 0): 0 past n
__device__ __forceinline__ void load8_nt(const float *__restrict__ x, uint32_t i0, uint32_t n, float4 &v0, float4 &v1)
{
    if (i0 + 8 <= n) {
        v0 = ld_nt(reinterpret_cast<const float4 *>(x + i0));
        v1 = ld_nt(reinterpret_cast<const float4 *>(x + i0 + 4));
        return;
    }
    v0 = load4_nt_tail<0>(x, i0, n);
    v1 = i0 + 4 < n ? load4_nt_tail<0>(x, i0 + 4, n) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

// mask encode (k_ms_mask_fast with NL = 2): the block owns 64 octets, its 4
// waves the planes p = wave + 4 j
template <int LM, int VAR = 0, int CBY = 0>
__global__ GC_MS_OCC __launch_bounds__(kBlock) void k_ms_mask_fast_o2(const float *__restrict__ x, uint32_t n,
                                                            const float *__restrict__ normp, LevelsArg lv,
                                                            MsFastArg fa, RngArgs rng, uint32_t M, uint32_t w,
                                                            uint32_t *__restrict__ mask_words,
                                                            void *__restrict__ cache = nullptr, int32_t cq = 0,
                                                            uint32_t cb = 0)
{
    const float norm = *normp;
    const DivNorm dv = make_div(norm);
    const uint32_t lo2 = 2u * dv.lo1, hi2 = 2u * __float_as_uint(norm);
    const uint32_t octs = M >> 3;
    constexpr int PW = (LM + 3) / 4;
    __shared__ uint4 part[3][2][kMsQuadsPerBlock];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    for (uint32_t tb = blockIdx.x * kMsQuadsPerBlock; tb < octs; tb += gridDim.x * kMsQuadsPerBlock) {
        const uint32_t t = tb + lane;
        uint4 acc[2] = {};
        // utail = false: the wave's 64 octets of this plane are all below n
        // (wave-uniform), so no per-lane tail tests (MSV_UFLAG)
        auto plane = [&](uint32_t p, uint32_t i0, const float4 (&v)[2], const uint4 (&d)[2][2], bool utail) {
#pragma unroll
            for (int hq = 0; hq < 2; ++hq) {
                const uint32_t iq = i0 + 4u * hq;
                if (hq == 1 && utail && iq >= n)
                    break;
                uint4 mb[1];
                if constexpr (CBY != 0) {
                    uint4 cv;
                    mask_plane_d<2, VAR, true>(v[hq], n, iq, dv, lo2, hi2, lv, fa, [&](int l) { return d[l][hq]; },
                                               1u << (p * w), mb, cq, cb, &cv, utail);
                    cache_store<CBY>(cache, iq, n, cv, utail);
                } else {
                    mask_plane_d<2, VAR, false>(v[hq], n, iq, dv, lo2, hi2, lv, fa, [&](int l) { return d[1][hq]; },
                                                1u << (p * w), mb, 0, 0, nullptr, utail);
                }
                acc[hq].x |= mb[0].x;
                acc[hq].y |= mb[0].y;
                acc[hq].z |= mb[0].z;
                acc[hq].w |= mb[0].w;
            }
        };
        const bool tile_full = tb + kMsQuadsPerBlock <= octs;
#pragma unroll
        for (int j = 0; j < ((VAR & MSV_ROLL) ? 1 : PW); ++j) {
#pragma unroll 1
        for (int j1 = 0; j1 < ((VAR & MSV_ROLL) ? PW : 1); ++j1) {
            const uint32_t p = wave + 4u * (j + j1);
            const uint32_t pb = p * M + 8u * tb;  // the wave's first octet (uniform)
            if (p >= (uint32_t)LM || pb >= n)
                break;
            const uint32_t i0 = pb + 8u * lane;
            if (t >= octs || i0 >= n)
                continue;
            // the tail tests behind a wave-uniform flag (MSV_UFLAG), else per lane
            const bool tl = (VAR & MSV_UFLAG) == 0 || !(tile_full && pb + 8u * kMsQuadsPerBlock <= n);
            float4 v[2];
            if (tl) {
                load8_nt(x, i0, n, v[0], v[1]);
            } else {
                v[0] = ld_nt(reinterpret_cast<const float4 *>(x + i0));
                v[1] = ld_nt(reinterpret_cast<const float4 *>(x + i0 + 4));
            }
            uint4 d[2][2];
            if constexpr (CBY != 0)
                ms2_octet(rng, i0 >> 3, d);
            else
                ms2_octet_level(rng, i0 >> 3, 1, d[1]);
            plane(p, i0, v, d, tl);
        }
        }
        if (wave) {
            part[wave - 1][0][lane] = acc[0];
            part[wave - 1][1][lane] = acc[1];
        }
        __syncthreads();
        if (wave == 0 && t < octs) {
#pragma unroll
            for (int hq = 0; hq < 2; ++hq) {
                const uint4 a = part[0][hq][lane], b = part[1][hq][lane], c = part[2][hq][lane];
                st4u<(VAR & MSV_PLAINST) == 0>(mask_words + 8u * t + 4u * hq,
                                               make_uint4(acc[hq].x | a.x | b.x | c.x, acc[hq].y | a.y | b.y | c.y,
                                                          acc[hq].z | a.z | b.z | c.z, acc[hq].w | a.w | b.w | c.w));
            }
        }
        __syncthreads();
    }
}

// select encode (k_ms_select_fast with NL = 2)
template <int LQ, int VAR = 0>
__global__ __launch_bounds__(kBlock) void k_ms_select_fast_o2(const float *__restrict__ x, uint32_t n,
                                                              const float *__restrict__ normp, LevelsArg lv,
                                                              MsFastArg fa, RngArgs rng, MaskArg mk, FastDiv fd,
                                                              uint32_t Mq, uint32_t wq, int32_t qmax,
                                                              uint32_t *__restrict__ words)
{
    const float norm = *normp;
    const DivNorm dv = make_div(norm);
    const uint32_t lo2 = 2u * dv.lo1;
    const uint32_t octs = Mq >> 3;
    constexpr int PW = (LQ + 3) / 4;
    __shared__ uint4 part[3][2][kMsQuadsPerBlock];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    for (uint32_t tb = blockIdx.x * kMsQuadsPerBlock; tb < octs; tb += gridDim.x * kMsQuadsPerBlock) {
        const uint32_t t = tb + lane;
        uint4 acc[2] = {};
        if (t < octs) {
#pragma unroll
            for (int j = 0; j < PW; ++j) {
                const uint32_t p = wave + 4u * j;
                if (p >= (uint32_t)LQ)
                    break;
                const uint32_t i0 = p * Mq + 8u * t;
                if (i0 >= n)
                    break;
                float4 v[2];
                load8_nt(x, i0, n, v[0], v[1]);
                uint4 m[2];
                m[0] = mask_levels4_fast<2>(mk, fd, i0);
                m[1] = i0 + 4 < n ? mask_levels4_fast<2>(mk, fd, i0 + 4) : make_uint4(0u, 0u, 0u, 0u);
                uint4 d[2][2];
                ms2_octet(rng, i0 >> 3, d);
                const uint32_t sh = p * wq;
#pragma unroll
                for (int hq = 0; hq < 2; ++hq) {
                    const uint32_t iq = i0 + 4u * hq;
                    if (hq == 1 && iq >= n)
                        break;
                    const uint4 &mm = m[hq];
                    const uint4 r = make_uint4(mm.x ? d[1][hq].x : d[0][hq].x, mm.y ? d[1][hq].y : d[0][hq].y,
                                               mm.z ? d[1][hq].z : d[0][hq].z, mm.w ? d[1][hq].w : d[0][hq].w);
                    const uint4 ln = select_lanes<2, VAR>(v[hq], mm, r, n, iq, dv, lo2, lv, fa, qmax);
                    acc[hq].x += ln.x << sh;
                    acc[hq].y += ln.y << sh;
                    acc[hq].z += ln.z << sh;
                    acc[hq].w += ln.w << sh;
                }
            }
        }
        if (wave) {
            part[wave - 1][0][lane] = acc[0];
            part[wave - 1][1][lane] = acc[1];
        }
        __syncthreads();
        if (wave == 0 && t < octs) {
#pragma unroll
            for (int hq = 0; hq < 2; ++hq) {
                const uint4 a = part[0][hq][lane], b = part[1][hq][lane], c = part[2][hq][lane];
                st4u<(VAR & MSV_PLAINST) == 0>(words + 8u * t + 4u * hq,
                                               make_uint4(acc[hq].x + a.x + b.x + c.x, acc[hq].y + a.y + b.y + c.y,
                                                          acc[hq].z + a.z + b.z + c.z, acc[hq].w + a.w + b.w + c.w));
            }
        }
        __syncthreads();
    }
}

// W = 1 one-pass encode (k_ms_fused_w1 with NL = 2): lanes = octets of the
// mask stream's quads, wave h = q stream h as there
template <int VAR = 0>
__global__ GC_MS_OCC __launch_bounds__(64 * kMsFusedMaxR) void k_ms_fused_w1_o2(
    const float *__restrict__ x, uint32_t n, const float *__restrict__ normp, LevelsArg lv, MsFastArg fa, RngArgs rng,
    uint32_t Mm, uint32_t r, uint32_t Lq, uint32_t wq, int32_t qmax, uint32_t Cw, uint32_t pend,
    uint32_t *__restrict__ mask_words, uint32_t *__restrict__ words)
{
    const float norm = *normp;
    const DivNorm dv = make_div(norm);
    const uint32_t lo2 = 2u * dv.lo1;
    const uint32_t octs = Mm >> 3;
    const uint32_t h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t kend = h < pend ? min(Lq, (pend - h + r - 1) / r) : 0u;
    const uint32_t kfull = h + 1 < pend ? min(kend, (pend - 1 - h + r - 1) / r) : 0u;
    __shared__ uint4 part[kMsFusedMaxR - 1][2][kMsQuadsPerBlock];
    for (uint32_t tb = blockIdx.x * kMsQuadsPerBlock; tb < octs; tb += gridDim.x * kMsQuadsPerBlock) {
        const uint32_t t = tb + lane;
        uint4 macc[2][1] = {};
        uint4 acc[2] = {};
        if (t < octs) {
            uint32_t i0 = h * Mm + 8u * t;
            const uint32_t step = r * Mm;
            auto load = [&](uint32_t k, uint32_t i, float4 (&v)[2]) {
                if (k < kfull) {
                    v[0] = ld_nt(reinterpret_cast<const float4 *>(x + i));
                    v[1] = ld_nt(reinterpret_cast<const float4 *>(x + i + 4));
                } else {
                    v[0] = load4_guard(x, i, n);
                    v[1] = load4_guard(x, i + 4, n);
                }
            };
            float4 vn[2];
            if constexpr ((VAR & MSV_PREFETCH) != 0) {
                if (kend > 0)
                    load(0, i0, vn);
            }
#pragma unroll 1
            for (uint32_t k = 0; k < kend; ++k) {
                float4 v[2];
                if constexpr ((VAR & MSV_PREFETCH) != 0) {
                    v[0] = vn[0];
                    v[1] = vn[1];
                    if (k + 1 < kend)
                        load(k + 1, i0 + step, vn);
                } else {
                    load(k, i0, v);
                }
                uint4 d[2][2];
                ms2_octet(rng, i0 >> 3, d);
                const uint32_t bitP = 1u << (h + r * k), sh = k * wq;
#pragma unroll
                for (int hq = 0; hq < 2; ++hq)
                    fused_plane_d<2, VAR>(v[hq], n, i0 + 4u * hq, dv, lo2, lv, fa, [&](int l) { return d[l][hq]; },
                                          bitP, sh, macc[hq], acc[hq], qmax);
                i0 += step;
            }
        }
        if (t < octs) {
            const uint64_t Mq = (uint64_t)r * Mm;
#pragma unroll
            for (int hq = 0; hq < 2; ++hq) {
                const uint64_t j0 = (uint64_t)h * Mm + 8u * t + 4u * hq;
                uint4 C = make_uint4(Cw, Cw, Cw, Cw);
                if (j0 + 3 + (uint64_t)(Lq - 1) * Mq >= n) {  // lanes of elements past n stay 0
                    C = make_uint4(0u, 0u, 0u, 0u);
                    for (uint32_t k = 0; k < Lq; ++k) {
                        const uint64_t e = j0 + (uint64_t)k * Mq;
                        const uint32_t c = (uint32_t)qmax << (k * wq);
                        C.x += e < n ? c : 0u;
                        C.y += e + 1 < n ? c : 0u;
                        C.z += e + 2 < n ? c : 0u;
                        C.w += e + 3 < n ? c : 0u;
                    }
                }
                st4u<(VAR & MSV_PLAINST) == 0>(words + j0, make_uint4(C.x - acc[hq].x, C.y - acc[hq].y,
                                                                     C.z - acc[hq].z, C.w - acc[hq].w));
            }
        }
        if (h) {
            part[h - 1][0][lane] = macc[0][0];
            part[h - 1][1][lane] = macc[1][0];
        }
        __syncthreads();
        if (h == 0 && t < octs) {
#pragma unroll
            for (int hq = 0; hq < 2; ++hq) {
                uint4 o = macc[hq][0];
                for (uint32_t q = 0; q + 1 < r; ++q) {
                    const uint4 a = part[q][hq][lane];
                    o = make_uint4(o.x | a.x, o.y | a.y, o.z | a.z, o.w | a.w);
                }
                st4u<(VAR & MSV_PLAINST) == 0>(mask_words + 8u * t + 4u * hq, o);
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// decode (compressors.py:819-826 order 0; 668-680 order 1) + alpha
// ---------------------------------------------------------------------------
template <int LQ, int ORDER, int NL, int VAR = 0>
__global__ __launch_bounds__(kBlock) void k_ms_decode_fast(const uint32_t *__restrict__ words, MaskArg mk, FastDiv fd,
                                                           uint32_t n, const float *__restrict__ normp, LevelsArg lv,
                                                           MsFastArg fa, uint32_t Mq, uint32_t wq, int32_t sub,
                                                           float alpha, float *__restrict__ out)
{
    const float norm = *normp;
    // order 1: c_l = RN(norm / s_l); order 0: Markstein by s_l when Q*norm stays normal
    float c[GC_MAX_LEVELS] = {};
#pragma unroll
    for (int l = 0; l < NL; ++l)
        c[l] = ORDER == 1 ? norm / lv.s[l] : 0.0f;
    const bool mk0 = norm >= 0x1p-100f && norm <= 0x1p100f;
    const uint32_t msk = (1u << wq) - 1u;
    const uint32_t quads = Mq >> 2;
    if constexpr ((VAR & MSV_PERTHREAD) != 0) {
        for (uint32_t t = blockIdx.x * kBlock + threadIdx.x; t < quads; t += gridDim.x * kBlock) {
            const uint4 wd = *reinterpret_cast<const uint4 *>(words + 4u * t);
#pragma unroll
            for (int k = 0; k < LQ; ++k) {
                const uint32_t i0 = (uint32_t)k * Mq + 4u * t;
                if (i0 >= n)
                    break;
                decode_plane<ORDER, NL>(wd, (uint32_t)k * wq, msk, sub, mask_levels4_fast<NL>(mk, fd, i0), norm, lv, fa, c,
                                    mk0, alpha, out, i0, n);
            }
        }
        return;
    }
    constexpr int PW = (LQ + 3) / 4;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    for (uint32_t tb = blockIdx.x * kMsQuadsPerBlock; tb < quads; tb += gridDim.x * kMsQuadsPerBlock) {
        const uint32_t t = tb + lane;
        if (t >= quads)
            continue;
        const uint4 wd = *reinterpret_cast<const uint4 *>(words + 4u * t);
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            const uint32_t p = wave + 4u * j;
            if (p >= (uint32_t)LQ)
                break;
            const uint32_t i0 = p * Mq + 4u * t;
            if (i0 >= n)
                break;
            decode_plane<ORDER, NL, (VAR & MSV_PLAINST) == 0>(
                wd, p * wq, msk, sub, mask_levels4_fast<NL>(mk, fd, i0), norm, lv, fa, c,
                mk0, alpha, out, i0, n);
        }
    }
}

}  // namespace gc
