// qsgd_encode.h — the fused QSGD-MaxNorm encode kernel (quantize + stochastic
// round + carry-free planar pack), compressors.py:299-316.
//
// Shared by qsgd.hip (the product instantiation, ABL = 0) and
// tools/encode_lab.hip (ablation variants for measurement only).
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
                q[k] = quot4_fast<ABL>(xv[k], dv);
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
                acc.x |= enc_lane<ABL>(xv[k].x, q[k].x, s, qmax, r.x) << sh;
                acc.y |= enc_lane<ABL>(xv[k].y, q[k].y, s, qmax, r.y) << sh;
                acc.z |= enc_lane<ABL>(xv[k].z, q[k].z, s, qmax, r.z) << sh;
                acc.w |= enc_lane<ABL>(xv[k].w, q[k].w, s, qmax, r.w) << sh;
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
                const float4 q = __builtin_expect(rg.slow(dv), 0) ? quot4_ieee(xv[k], norm) : quot4_fast<ABL>(xv[k], dv);
                const uint32_t sh = (uint32_t)k * w;
                acc.x |= enc_lane<ABL>(xv[k].x, q.x, s, qmax, r.x) << sh;
                acc.y |= enc_lane<ABL>(xv[k].y, q.y, s, qmax, r.y) << sh;
                acc.z |= enc_lane<ABL>(xv[k].z, q.z, s, qmax, r.z) << sh;
                acc.w |= enc_lane<ABL>(xv[k].w, q.w, s, qmax, r.w) << sh;
            }
            *reinterpret_cast<uint4 *>(words + t4) = acc;
            continue;
        }
        float4 q[L];
        Range rg;
#pragma unroll
        for (int k = 0; k < L; ++k) {
            q[k] = quot4_fast<ABL>(xv[k], dv);
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
            acc.x |= enc_lane<ABL>(xv[k].x, q[k].x, s, qmax, r.x) << sh;
            acc.y |= enc_lane<ABL>(xv[k].y, q[k].y, s, qmax, r.y) << sh;
            acc.z |= enc_lane<ABL>(xv[k].z, q[k].z, s, qmax, r.z) << sh;
            acc.w |= enc_lane<ABL>(xv[k].w, q[k].w, s, qmax, r.w) << sh;
        }
        *reinterpret_cast<uint4 *>(words + t4) = acc;
    }
    // generic body: tail quads (partial planes), gathers, unaligned x, odd norms
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
                    q = quot4_fast<ABL>(v, dv);
                else
                    q = quot4_ieee(v, norm);
                const uint32_t sh = (uint32_t)k * w;
                acc.x |= enc_lane<ABL>(v.x, q.x, s, qmax, r.x) << sh;
                acc.y |= (i0 + 1 < n ? enc_lane<ABL>(v.y, q.y, s, qmax, r.y) : 0u) << sh;
                acc.z |= (i0 + 2 < n ? enc_lane<ABL>(v.z, q.z, s, qmax, r.z) : 0u) << sh;
                acc.w |= (i0 + 3 < n ? enc_lane<ABL>(v.w, q.w, s, qmax, r.w) : 0u) << sh;
            }
        }
        *reinterpret_cast<uint4 *>(words + 4 * t) = acc;
    }
}

}  // namespace gc
