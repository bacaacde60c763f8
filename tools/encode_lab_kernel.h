// encode_lab_kernel.h — MEASUREMENT ONLY (tools/encode_lab.hip, tools/lab2.hip):
// the QSGD encode kernel with the ablation and schedule switches of rounds
// 1-5 (ENC_*), as gclab::k_qsgd_encode<L, KIND, MODE, ABL, MINW>.  The
// product kernel (gradient-compression_amd/csrc/qsgd_encode.h) is this with
// ABL = ENC_INT | ENC_NT | ENC_NTS; the other switches were measured and not
// kept.  Never linked into libgcodec.
#pragma once

#include "qsgd_encode.h"

namespace gclab {
using namespace gc;

enum : int {
    ENC_ABL_NORNG = 1,  // measurement only: draws = element index (no Philox)
    ENC_ABL_NODIV = 2,  // measurement only: ql = |x| * (1/norm) (not exact)
    ENC_PHX0 = 4,       // Philox instruction mix 0 (same outputs)
    ENC_PHX2 = 8,       // Philox instruction mix 2 (same outputs)
    ENC_MED3 = 16,      // clamp with v_max + v_min instead of v_med3_f32
    ENC_ABL_L2 = 32,    // measurement only: loads from a 16 KB window (compute floor)
    ENC_REV = 64,       // walk the full tiles from the top down (Infinity-Cache reuse after absmax)
    ENC_GRP2 = 128,     // schedule the planes in pairs (fewer live Philox chains -> fewer VGPRs)
    ENC_GRP3 = 256,     // schedule the planes in triples
    ENC_SEQ = 512,      // one plane at a time: per-plane range check, sched barrier between planes
    ENC_PF = 1024,      // register prefetch: the next tile's L loads are issued before this tile's math
    ENC_DIV2 = 2048,    // the compiler's two-correction quotient (div_fast2) instead of Markstein's
    ENC_NT = 4096,      // nontemporal loads of x
    ENC_INT = 8192,     // integer stochastic rounding on full tiles (same outputs; b <= 8)
    ENC_NTS = 16384,    // nontemporal stores of the packed words
};

template <int ABL>
__device__ __forceinline__ void store_words_abl(uint32_t *p, const uint4 &v)
{
    if constexpr ((ABL & ENC_NTS) != 0) {
        typedef uint32_t u4v __attribute__((ext_vector_type(4)));
        const u4v r = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(r, reinterpret_cast<u4v *>(p));
    } else {
        *reinterpret_cast<uint4 *>(p) = v;
    }
}

template <int KIND, int ABL>
__device__ __forceinline__ uint4 draws4_abl(const RngArgs &rng, uint32_t level, uint64_t i0);

// one full tile (L planes x 4 words) on the integer path.  Lanes k < H
// accumulate at shift k*w, lanes k >= H at (k-H)*w, so every 24-bit
// multiplier is +-2^sh with sh <= 15; word = C -+ (lo + (hi << H*w)).
template <int L, int KIND, int ABL, bool WIDE>
__device__ __forceinline__ uint4 enc_tile_int_abl(const float4 (&xv)[L], uint32_t t4, uint32_t M32, const DivNorm &dv,
                                              float S24, uint32_t w, uint32_t Cw, const RngArgs &rng)
{
    constexpr int H = L / 2;
    int32_t lo[4] = {0, 0, 0, 0}, hi[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < L; ++k) {
        const gc_f2 l01 = ls2(xv[k].x, xv[k].y, dv, S24);
        const gc_f2 l23 = ls2(xv[k].z, xv[k].w, dv, S24);
        const uint4 r = draws4_abl<KIND, ABL>(rng, 0, k * M32 + t4);
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

// lane value of one element (ql = |x| / norm).  A NaN quotient (0/0, NaN
// input) gives xi = 0 (fmaxf(NaN, 0) = 0); an infinite one saturates at s.
template <int ABL = 0>
__device__ __forceinline__ uint32_t enc_lane_abl(float x, float ql, float s, int32_t qmax, uint32_t r)
{
    // v_med3_f32(l, 0, s): clamps to [0, s]; a NaN l yields 0 (checked against
    // the oracle by tests/test_gpu_parity.py::test_encode_non_finite_and_tiny_inputs)
    const float l = (ABL & ENC_MED3) ? fminf(fmaxf(ql * s, 0.0f), s) : __builtin_amdgcn_fmed3f(ql * s, 0.0f, s);
    const uint32_t fl = (uint32_t)(int32_t)l;
    const float p = __builtin_amdgcn_fractf(l);
    const float u = (float)(r & 0xFFFFFFu) * 0x1p-24f;
    const uint32_t xi = fl + (u < p ? 1u : 0u);
    // qmax + sign(x)*xi without a multiply: sg = 0 or ~0 from the sign bit
    // (-0.0 and signed NaN give xi = 0 anyway): (xi ^ sg) - sg + qmax
    const uint32_t sg = (uint32_t)(__float_as_int(x) >> 31);
    return (xi ^ sg) + ((uint32_t)qmax - sg);
}

template <int ABL>
__device__ __forceinline__ float4 quot4_fast_abl(const float4 &v, const DivNorm &d)
{
    float4 q;
    if constexpr ((ABL & ENC_ABL_NODIV) != 0) {
        q.x = fabsf(v.x) * d.r;
        q.y = fabsf(v.y) * d.r;
        q.z = fabsf(v.z) * d.r;
        q.w = fabsf(v.w) * d.r;
    } else if constexpr ((ABL & ENC_DIV2) != 0) {
        q.x = div_fast2(fabsf(v.x), d);
        q.y = div_fast2(fabsf(v.y), d);
        q.z = div_fast2(fabsf(v.z), d);
        q.w = div_fast2(fabsf(v.w), d);
    } else {
        q.x = div_fast(fabsf(v.x), d);
        q.y = div_fast(fabsf(v.y), d);
        q.z = div_fast(fabsf(v.z), d);
        q.w = div_fast(fabsf(v.w), d);
    }
    return q;
}

template <int KIND, int ABL>
__device__ __forceinline__ uint4 draws4_abl(const RngArgs &rng, uint32_t level, uint64_t i0);

// One full tile from split-plane draws (KIND 4 / 5, gc_device.h).  With c =
// ceil(|Ls|) = fl*2^24 + F the bit is [m < F], m = the 24-bit draw.  Knowing
// only m's top HB bits hm (low bits zero), [hm < F] is already right unless
// F - 1 and m share their top HB bits (then hm <= F - 1 < hm + 2^(24-HB) and
// the low bits decide): those elements flag their quad, and only flagged
// quads load the LO plane (8 / 4 bytes).  A flag where F = 0 is harmless (the
// loaded bits give the exact answer either way).  HB = 8 flags ~1 draw in
// 256, HB = 16 ~1 in 65,536.  Otherwise enc_tile_int's arithmetic.
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

template <int L, int KIND, bool WIDE>
__device__ __forceinline__ uint4 enc_tile_int_split(const float4 (&xv)[L], uint32_t t4, uint32_t M32, const DivNorm &dv,
                                                    float S24, uint32_t w, uint32_t Cw, const RngArgs &rng)
{
    constexpr uint32_t HB = KIND == 4 ? 8u : 16u, LB = 24u - HB;
    constexpr uint32_t HM = ((1u << HB) - 1u) << LB;
    constexpr int H = L / 2;
    const uint8_t *hp = reinterpret_cast<const uint8_t *>(rng.stream);
    const uint8_t *lp = hp + split_hpad(rng.n, HB);
    // the HI words as loaded (one / two per plane); a plane's draws are unpacked where used
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
    // per plane: c (WIDE) or -c (narrow) per element; a quad whose low bits
    // decide loads the LO plane at once (rare: the wave waits only then)
    int32_t lo[4] = {0, 0, 0, 0}, hi[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < L; ++k) {
        const gc_f2 l01 = ls2(xv[k].x, xv[k].y, dv, S24);
        const gc_f2 l23 = ls2(xv[k].z, xv[k].w, dv, S24);
        const float ls[4] = {l01.x, l01.y, l23.x, l23.y};
        uint32_t rd[4];
        if constexpr (HB == 8) {
            rd[0] = (hw[k][0] << 16) & HM;
            rd[1] = (hw[k][0] << 8) & HM;
            rd[2] = hw[k][0] & HM;
            rd[3] = (hw[k][0] >> 8) & HM;
        } else {
            rd[0] = (hw[k][0] << 8) & HM;
            rd[1] = (hw[k][0] >> 8) & HM;
            rd[2] = (hw[k][HB / 8 - 1] << 8) & HM;
            rd[3] = (hw[k][HB / 8 - 1] >> 8) & HM;
        }
        int32_t cc[4];
        bool any = false;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            uint32_t cm1;
            if constexpr (WIDE) {
                cc[e] = (int32_t)(uint32_t)__builtin_ceilf(fabsf(ls[e]));
                cm1 = (uint32_t)cc[e] - 1u;
            } else {
                cc[e] = cvt_flr_neg_abs(ls[e]);
                cm1 = ~(uint32_t)cc[e];
            }
            any |= ((cm1 ^ rd[e]) & HM) == 0u;
        }
        if (__builtin_expect(any, 0)) {
            const uint32_t i0 = k * M32 + t4;
            if constexpr (HB == 8) {
                const uint2 v = *reinterpret_cast<const uint2 *>(lp + 2u * i0);
                rd[0] |= v.x & 0xFFFFu;
                rd[1] |= v.x >> 16;
                rd[2] |= v.y & 0xFFFFu;
                rd[3] |= v.y >> 16;
            } else {
                const uint32_t v = *reinterpret_cast<const uint32_t *>(lp + i0);
                rd[0] |= v & 0xFFu;
                rd[1] |= (v >> 8) & 0xFFu;
                rd[2] |= (v >> 16) & 0xFFu;
                rd[3] |= v >> 24;
            }
        }
        const uint32_t sh = (uint32_t)(k < H ? k : k - H) * w;
        const int32_t bl = -(1 << sh), bh = 1 << sh;
        int32_t *a = k < H ? lo : hi;
        const float xs[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int32_t sg = med3_i32(__float_as_int(xs[e]), bl, bh);
            if constexpr (WIDE) {  // xi = (c + (~m & 0xFFFFFF)) >> 24 = fl + [m < F]
                const uint32_t t = (uint32_t)add_low24(~rd[e], cc[e]);
                a[e] += __mul24((int32_t)(t >> 24), sg);
            } else {  // (m - c) >> 24 = -xi (m < 2^24 here)
                const int32_t t = (int32_t)rd[e] + cc[e];
                a[e] += __mul24(t >> 24, sg);
            }
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

// one full tile (L planes x 4 words) on the integer path.  Lanes k < H
// accumulate at shift k*w, lanes k >= H at (k-H)*w, so every 24-bit
// multiplier is +-2^sh with sh <= 15; word = C -+ (lo + (hi << H*w)).
template <int L, int KIND, int ABL, bool WIDE>
__device__ __forceinline__ uint4 enc_tile_int(const float4 (&xv)[L], uint32_t t4, uint32_t M32, const DivNorm &dv,
                                              float S24, uint32_t w, uint32_t Cw, const RngArgs &rng)
{
    if constexpr (KIND == 4 || KIND == 5)
        return enc_tile_int_split<L, KIND, WIDE>(xv, t4, M32, dv, S24, w, Cw, rng);
    constexpr int H = L / 2;
    int32_t lo[4] = {0, 0, 0, 0}, hi[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < L; ++k) {
        const gc_f2 l01 = ls2(xv[k].x, xv[k].y, dv, S24);
        const gc_f2 l23 = ls2(xv[k].z, xv[k].w, dv, S24);
        const uint4 r = draws4_abl<KIND, ABL>(rng, 0, k * M32 + t4);
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

// fast-path tile check for ENC_INT: every |x| <= norm (inf / NaN excluded by
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
template <int ABL = 0>
__device__ __forceinline__ uint32_t enc_lane(float x, float ql, float s, int32_t qmax, uint32_t r)
{
    // v_med3_f32(l, 0, s): clamps to [0, s]; a NaN l yields 0 (checked against
    // the oracle by tests/test_gpu_parity.py::test_encode_non_finite_and_tiny_inputs)
    const float l = (ABL & ENC_MED3) ? fminf(fmaxf(ql * s, 0.0f), s) : __builtin_amdgcn_fmed3f(ql * s, 0.0f, s);
    const uint32_t fl = (uint32_t)(int32_t)l;
    const float p = __builtin_amdgcn_fractf(l);
    const float u = (float)(r & 0xFFFFFFu) * 0x1p-24f;
    const uint32_t xi = fl + (u < p ? 1u : 0u);
    // qmax + sign(x)*xi without a multiply: sg = 0 or ~0 from the sign bit
    // (-0.0 and signed NaN give xi = 0 anyway): (xi ^ sg) - sg + qmax
    const uint32_t sg = (uint32_t)(__float_as_int(x) >> 31);
    return (xi ^ sg) + ((uint32_t)qmax - sg);
}

template <int ABL>
__device__ __forceinline__ float4 quot4_fast(const float4 &v, const DivNorm &d)
{
    float4 q;
    if constexpr ((ABL & ENC_ABL_NODIV) != 0) {
        q.x = fabsf(v.x) * d.r;
        q.y = fabsf(v.y) * d.r;
        q.z = fabsf(v.z) * d.r;
        q.w = fabsf(v.w) * d.r;
    } else if constexpr ((ABL & ENC_DIV2) != 0) {
        q.x = div_fast2(fabsf(v.x), d);
        q.y = div_fast2(fabsf(v.y), d);
        q.z = div_fast2(fabsf(v.z), d);
        q.w = div_fast2(fabsf(v.w), d);
    } else {
        q.x = div_fast(fabsf(v.x), d);
        q.y = div_fast(fabsf(v.y), d);
        q.z = div_fast(fabsf(v.z), d);
        q.w = div_fast(fabsf(v.w), d);
    }
    return q;
}

template <int KIND, int ABL>
__device__ __forceinline__ uint4 draws4_abl(const RngArgs &rng, uint32_t level, uint64_t i0)
{
    if constexpr ((ABL & ENC_ABL_NORNG) != 0) {
        const uint32_t b = (uint32_t)i0 * 2654435761u;
        return make_uint4(b, b + 1u, b + 2u, b + 3u);
    } else if constexpr ((ABL & ENC_PHX0) != 0) {
        return draws4<KIND, 0>(rng, level, i0);
    } else if constexpr ((ABL & ENC_PHX2) != 0) {
        return draws4<KIND, 2>(rng, level, i0);
    } else {
        return draws4<KIND>(rng, level, i0);
    }
}

// Full tiles: every one of the L planes of words 4t..4t+3 is in range, so
// no per-element bounds, 32-bit element indices, L float4 loads in flight.
// Tail quads, gathers, unaligned x and the non-fast-division case go through
// the generic body.
template <int L, int KIND, int MODE, int ABL, int MINW = 1>
__global__ __launch_bounds__(kBlock, MINW) void k_qsgd_encode(const float *__restrict__ x, const int64_t *__restrict__ idx,
                                                        uint64_t n, const float *__restrict__ normp, float s,
                                                        int32_t qmax, uint32_t w, uint64_t M, RngArgs rng,
                                                        uint32_t *__restrict__ words)
{
    const float norm = *normp;
    const DivNorm dv = make_div(norm);
    const bool fast = dv.fast || (ABL & ENC_ABL_NODIV) != 0;
    const uint64_t quads = M >> 2;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;

    // quads whose last plane is full: (L-1)*M + 4t + 3 < n
    const uint64_t last = (uint64_t)(L - 1) * M;
    const uint64_t full = (MODE == 0 && fast && n >= last + 4 && n < (1ull << 32)) ? (n - last) >> 2 : 0;
    const uint32_t M32 = (uint32_t)M;
    // ENC_INT constants (uniform): b <= 7 (s * 2^24 < 2^31) takes the signed
    // floor form, b = 8 the unsigned ceil form
    const bool intok = s <= 255.0f, narrow = s <= 127.0f;
    const float S24 = s * 16777216.0f;
    const uint32_t lo2 = 2u * dv.lo1, hi2 = 2u * __float_as_uint(norm);
    uint32_t Cw = 0;
    for (int k = 0; k < L; ++k)
        Cw += (uint32_t)qmax << (k * w);
    if constexpr ((ABL & ENC_PF) != 0) {
        float4 nx[L];
        if (t < full) {
#pragma unroll
            for (int k = 0; k < L; ++k)
                nx[k] = *reinterpret_cast<const float4 *>(x + (k * M32 + (uint32_t)t * 4u));
        }
        for (; t < full; t += stride) {
            const uint32_t t4 = (uint32_t)t * 4u;
            float4 xv[L];
#pragma unroll
            for (int k = 0; k < L; ++k)
                xv[k] = nx[k];
            if (t + stride < full) {
                const uint32_t n4 = (uint32_t)(t + stride) * 4u;
#pragma unroll
                for (int k = 0; k < L; ++k)
                    nx[k] = *reinterpret_cast<const float4 *>(x + (k * M32 + n4));
            }
            float4 q[L];
            Range rg;
#pragma unroll
            for (int k = 0; k < L; ++k) {
                q[k] = quot4_fast_abl<ABL>(xv[k], dv);
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
                const uint4 r = draws4_abl<KIND, ABL>(rng, 0, k * M32 + t4);
                const uint32_t sh = (uint32_t)k * w;
                acc.x |= enc_lane_abl<ABL>(xv[k].x, q[k].x, s, qmax, r.x) << sh;
                acc.y |= enc_lane_abl<ABL>(xv[k].y, q[k].y, s, qmax, r.y) << sh;
                acc.z |= enc_lane_abl<ABL>(xv[k].z, q[k].z, s, qmax, r.z) << sh;
                acc.w |= enc_lane_abl<ABL>(xv[k].w, q[k].w, s, qmax, r.w) << sh;
            }
            *reinterpret_cast<uint4 *>(words + t4) = acc;
        }
    }
    for (; t < full; t += stride) {
        const uint32_t t4 = (uint32_t)((ABL & ENC_REV) ? (full - 1 - t) : t) * 4u;
        float4 xv[L];
#pragma unroll
        for (int k = 0; k < L; ++k) {
            const float4 *p = reinterpret_cast<const float4 *>(x + ((ABL & ENC_ABL_L2) ? ((k * M32 + t4) & 4095u)
                                                                                      : (k * M32 + t4)));
            if constexpr ((ABL & ENC_NT) != 0) {
                typedef float f4v __attribute__((ext_vector_type(4)));
                const f4v r = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(p));
                xv[k] = make_float4(r.x, r.y, r.z, r.w);
            } else {
                xv[k] = *p;
            }
        }
        if constexpr ((ABL & ENC_INT) != 0) {
            if (intok) {
                RangeI rg;
#pragma unroll
                for (int k = 0; k < L; ++k)
                    rg.add4(xv[k]);
                if (__builtin_expect(!rg.slow(lo2, hi2), 1)) {
                    const uint4 acc = narrow ? enc_tile_int_abl<L, KIND, ABL, false>(xv, t4, M32, dv, S24, w, Cw, rng)
                                             : enc_tile_int_abl<L, KIND, ABL, true>(xv, t4, M32, dv, S24, w, Cw, rng);
                    store_words_abl<ABL>(words + t4, acc);
                    continue;
                }
            }
        }
        if constexpr ((ABL & ENC_SEQ) != 0) {
            uint4 acc = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (int k = 0; k < L; ++k) {
                if (k)
                    __builtin_amdgcn_sched_barrier(0);
                const uint32_t i0 = k * M32 + t4;
                const uint4 r = draws4_abl<KIND, ABL>(rng, 0, i0);
                Range rg;
                rg.add4(xv[k]);
                const float4 q = __builtin_expect(rg.slow(dv), 0) ? quot4_ieee(xv[k], norm) : quot4_fast_abl<ABL>(xv[k], dv);
                const uint32_t sh = (uint32_t)k * w;
                acc.x |= enc_lane_abl<ABL>(xv[k].x, q.x, s, qmax, r.x) << sh;
                acc.y |= enc_lane_abl<ABL>(xv[k].y, q.y, s, qmax, r.y) << sh;
                acc.z |= enc_lane_abl<ABL>(xv[k].z, q.z, s, qmax, r.z) << sh;
                acc.w |= enc_lane_abl<ABL>(xv[k].w, q.w, s, qmax, r.w) << sh;
            }
            *reinterpret_cast<uint4 *>(words + t4) = acc;
            continue;
        }
        float4 q[L];
        Range rg;
#pragma unroll
        for (int k = 0; k < L; ++k) {
            q[k] = quot4_fast_abl<ABL>(xv[k], dv);
            rg.add4(xv[k]);
        }
        if ((ABL & ENC_ABL_NODIV) == 0 && __builtin_expect(rg.slow(dv), 0)) {
#pragma unroll
            for (int k = 0; k < L; ++k)
                q[k] = quot4_ieee(xv[k], norm);
        }
        uint4 acc = make_uint4(0u, 0u, 0u, 0u);
        constexpr int G = (ABL & ENC_GRP2) ? 2 : ((ABL & ENC_GRP3) ? 3 : L);
#pragma unroll
        for (int k = 0; k < L; ++k) {
            if (k && (k % G) == 0)
                __builtin_amdgcn_sched_barrier(0);
            const uint32_t i0 = k * M32 + t4;
            const uint4 r = draws4_abl<KIND, ABL>(rng, 0, i0);
            const uint32_t sh = (uint32_t)k * w;
            acc.x |= enc_lane_abl<ABL>(xv[k].x, q[k].x, s, qmax, r.x) << sh;
            acc.y |= enc_lane_abl<ABL>(xv[k].y, q[k].y, s, qmax, r.y) << sh;
            acc.z |= enc_lane_abl<ABL>(xv[k].z, q[k].z, s, qmax, r.z) << sh;
            acc.w |= enc_lane_abl<ABL>(xv[k].w, q[k].w, s, qmax, r.w) << sh;
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
                        const uint4 r = draws4_abl<KIND, ABL>(rng, 0, i0);
                        Range rg;
                        rg.add4(v[j]);
                        const float4 q = fast && ((ABL & ENC_ABL_NODIV) != 0 || !rg.slow(dv))
                                             ? quot4_fast_abl<ABL>(v[j], dv)
                                             : quot4_ieee(v[j], norm);
                        const uint32_t sh = (uint32_t)k * w;
                        acc.x |= enc_lane_abl<ABL>(v[j].x, q.x, s, qmax, r.x) << sh;
                        acc.y |= (i0 + 1 < n ? enc_lane_abl<ABL>(v[j].y, q.y, s, qmax, r.y) : 0u) << sh;
                        acc.z |= (i0 + 2 < n ? enc_lane_abl<ABL>(v[j].z, q.z, s, qmax, r.z) : 0u) << sh;
                        acc.w |= (i0 + 3 < n ? enc_lane_abl<ABL>(v[j].w, q.w, s, qmax, r.w) : 0u) << sh;
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
                const uint4 r = draws4_abl<KIND, ABL>(rng, 0, i0);
                float4 q;
                Range rg;
                rg.add4(v);
                if (fast && ((ABL & ENC_ABL_NODIV) != 0 || !rg.slow(dv)))
                    q = quot4_fast_abl<ABL>(v, dv);
                else
                    q = quot4_ieee(v, norm);
                const uint32_t sh = (uint32_t)k * w;
                acc.x |= enc_lane_abl<ABL>(v.x, q.x, s, qmax, r.x) << sh;
                acc.y |= (i0 + 1 < n ? enc_lane_abl<ABL>(v.y, q.y, s, qmax, r.y) : 0u) << sh;
                acc.z |= (i0 + 2 < n ? enc_lane_abl<ABL>(v.z, q.z, s, qmax, r.z) : 0u) << sh;
                acc.w |= (i0 + 3 < n ? enc_lane_abl<ABL>(v.w, q.w, s, qmax, r.w) : 0u) << sh;
            }
        }
        *reinterpret_cast<uint4 *>(words + 4 * t) = acc;
    }
}

}  // namespace gclab
