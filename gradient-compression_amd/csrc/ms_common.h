// ms_common.h — device-side pieces of the multi-scale codec shared by
// multiscale.hip (the generic kernels), ms_fast.h (the dense fast paths) and
// tools/lab_ms.hip: level table, generic per-element level / select code,
// thermometer mask lanes.  compressors.py:754-826, 612-680.
//
// Level loops run over GC_MAX_LEVELS with a count guard, so every lv.s[l] is
// a static index: the table stays in kernel-argument SGPRs instead of being
// copied to scratch for dynamic indexing.
#pragma once

#include "gc_device.h"

namespace gc {

struct LevelsArg {
    uint32_t count;
    int32_t maxv;  // 2^bits[0] - 1 (compressors.py:800)
    float s[GC_MAX_LEVELS];
};

__device__ __forceinline__ float sel_level(const LevelsArg &lv, uint32_t m)
{
    float s = lv.s[0];
#pragma unroll
    for (int l = 1; l < GC_MAX_LEVELS; ++l)
        if ((uint32_t)l < lv.count && m == (uint32_t)l)
            s = lv.s[l];
    return s;
}

template <int MODE>
__device__ __forceinline__ float4 load4m(const float *__restrict__ x, const int64_t *__restrict__ idx, uint64_t i0,
                                         uint64_t n)
{
    if (MODE == 0 && i0 + 4 <= n)
        return *reinterpret_cast<const float4 *>(x + i0);
    float4 v;
    v.x = i0 + 0 < n ? (MODE == 2 ? x[idx[i0 + 0]] : x[i0 + 0]) : 0.0f;
    v.y = i0 + 1 < n ? (MODE == 2 ? x[idx[i0 + 1]] : x[i0 + 1]) : 0.0f;
    v.z = i0 + 2 < n ? (MODE == 2 ? x[idx[i0 + 2]] : x[i0 + 2]) : 0.0f;
    v.w = i0 + 3 < n ? (MODE == 2 ? x[idx[i0 + 3]] : x[i0 + 3]) : 0.0f;
    return v;
}

// resolution level of 4 elements: last level whose |q| <= maxv (level 0 always
// qualifies, so its draws are not needed here; level l uses draw block l)
template <int KIND>
__device__ __forceinline__ uint4 ms_levels4(const float4 &q, const LevelsArg &lv, const RngArgs &rng, uint64_t i0)
{
    uint4 m = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (uint32_t l = 1; l < GC_MAX_LEVELS; ++l) {
        if (l >= lv.count)
            break;
        const uint4 r = draws4<KIND>(rng, l, i0);
        const float s = lv.s[l];
        if (xi_from_q(q.x, s, r.x) <= lv.maxv) m.x = l;
        if (xi_from_q(q.y, s, r.y) <= lv.maxv) m.y = l;
        if (xi_from_q(q.z, s, r.z) <= lv.maxv) m.z = l;
        if (xi_from_q(q.w, s, r.w) <= lv.maxv) m.w = l;
    }
    return m;
}

// q of 4 elements at their own levels m (same draws as the mask pass)
template <int KIND>
__device__ __forceinline__ int4 ms_select4(const float4 &v, const float4 &q, const LevelsArg &lv, const RngArgs &rng,
                                           uint64_t i0, uint4 m)
{
    int4 o = make_int4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t l = 0; l < GC_MAX_LEVELS; ++l) {
        if (l >= lv.count)
            break;
        if (m.x != l && m.y != l && m.z != l && m.w != l)
            continue;
        const uint4 r = draws4<KIND>(rng, l, i0);
        const float s = lv.s[l];
        if (m.x == l) o.x = sgn_of(v.x) * xi_from_q(q.x, s, r.x);
        if (m.y == l) o.y = sgn_of(v.y) * xi_from_q(q.y, s, r.y);
        if (m.z == l) o.z = sgn_of(v.z) * xi_from_q(q.z, s, r.z);
        if (m.w == l) o.w = sgn_of(v.w) * xi_from_q(q.w, s, r.w);
    }
    return o;
}

struct MaskArg {
    const uint32_t *words;
    uint64_t M;       // words per field stream
    uint32_t w;       // lane bits
    uint32_t fields;  // count - 1
    uint32_t world;
};

// common level of elements pos..pos+3 (pos % 4 == 0, same plane) from W-summed fields
__device__ __forceinline__ uint4 mask_levels4(const MaskArg &mk, uint64_t i0)
{
    const uint64_t plane = i0 / mk.M, pos = i0 - plane * mk.M;
    const uint32_t sh = (uint32_t)plane * mk.w;
    const uint32_t msk = (1u << mk.w) - 1u;
    uint4 m = make_uint4(0u, 0u, 0u, 0u);
    for (uint32_t f = 0; f < mk.fields; ++f) {
        const uint4 wd = *reinterpret_cast<const uint4 *>(mk.words + f * mk.M + pos);
        m.x += ((wd.x >> sh) & msk) == mk.world;
        m.y += ((wd.y >> sh) & msk) == mk.world;
        m.z += ((wd.z >> sh) & msk) == mk.world;
        m.w += ((wd.w >> sh) & msk) == mk.world;
    }
    return m;
}

}  // namespace gc
