// multiscale.hip — multi-scale / two-scale QSGD-MaxNorm on gfx950
// (compressors.py:754-826 QSGDMaxNormMultiScaleCompressor, and for two levels
// compressors.py:612-680 QSGDMaxNormTwoScaleCompressor, reducer.py:1454-1715).
//
// The reference materialises an L x n float32 cache of every level's
// quantisation (compress_cache, 778-797), then a resolution mask (799-807), a
// MIN all-reduce of the int8 mask, and a select (809-817).  Here the mask
// kernel quantises every level on the fly and emits the mask as thermometer
// lanes (field k = [m >= k], k = 1..L-1), which a SUM all-reduce turns into
// the MIN over ranks (m = #fields whose sum == W).  The select then either
// recomputes the chosen level with the SAME counter-based draw (x read
// twice), or — gc_ms_*_cached, dense fast path — reads the cache the mask
// kernel wrote as one 1-2 byte cell per element (every level's lane value):
// 43 + 15 us instead of 24 + 36 us at 23.5M floats, the same total: both
// kernels are bound by the Philox draws (profiles/r01s_lab_ms.log); opt-in.
#include <algorithm>
#include <cstdlib>

#include "gc_device.h"
#include "gc_host.h"
#include "segments.h"
#include "ms_common.h"
#include "ms_fast.h"
namespace gc {

template <int LM, int KIND, int MODE>
__global__ __launch_bounds__(kBlock) void k_ms_mask_encode(const float *__restrict__ x, const int64_t *__restrict__ idx,
                                                           uint64_t n, const float *__restrict__ normp, LevelsArg lv,
                                                           RngArgs rng, uint64_t M, uint32_t w, uint32_t fields,
                                                           uint32_t *__restrict__ mask_words)
{
    const float norm = *normp;
    const DivNorm dv = make_div(norm);
    const uint64_t quads = M >> 2;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < quads; t += (uint64_t)gridDim.x * kBlock) {
        uint4 acc[GC_MAX_LEVELS - 1];
#pragma unroll
        for (int f = 0; f < GC_MAX_LEVELS - 1; ++f)
            acc[f] = make_uint4(0u, 0u, 0u, 0u);
        constexpr int C = gather_chunk(LM);
#pragma unroll
        for (int j0 = 0; j0 < LM; j0 += C) {
            float4 g[C];
            if constexpr (MODE == 2)  // GRandK: all index loads, then all value loads
                gather_planes<C>(x, idx, n, M, 4 * t, j0, g);
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int j = j0 + c;
                const uint64_t i0 = (uint64_t)j * M + 4 * t;
                if (j < LM && i0 < n) {
                    const float4 v = MODE == 2 ? g[c] : load4m<MODE>(x, idx, i0, n);
                    const uint4 m = ms_levels4<KIND>(quot4_exact(v, dv), lv, rng, i0);
                    const uint32_t sh = (uint32_t)j * w;
#pragma unroll
                    for (int f = 0; f < GC_MAX_LEVELS - 1; ++f) {
                        if ((uint32_t)f < fields) {
                            acc[f].x |= (uint32_t)(m.x > (uint32_t)f) << sh;
                            acc[f].y |= (uint32_t)(m.y > (uint32_t)f && i0 + 1 < n) << sh;
                            acc[f].z |= (uint32_t)(m.z > (uint32_t)f && i0 + 2 < n) << sh;
                            acc[f].w |= (uint32_t)(m.w > (uint32_t)f && i0 + 3 < n) << sh;
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int f = 0; f < GC_MAX_LEVELS - 1; ++f)
            if ((uint32_t)f < fields)
                *reinterpret_cast<uint4 *>(mask_words + (uint64_t)f * M + 4 * t) = acc[f];
    }
}

template <int LQ, int KIND, int MODE>
__global__ __launch_bounds__(kBlock) void k_ms_select_encode(const float *__restrict__ x,
                                                             const int64_t *__restrict__ idx, uint64_t n,
                                                             const float *__restrict__ normp, LevelsArg lv,
                                                             RngArgs rng, MaskArg mk, uint64_t Mq, uint32_t wq,
                                                             int32_t qmax, uint32_t *__restrict__ words)
{
    const float norm = *normp;
    const DivNorm dv = make_div(norm);
    const uint64_t quads = Mq >> 2;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < quads; t += (uint64_t)gridDim.x * kBlock) {
        uint4 acc = make_uint4(0u, 0u, 0u, 0u);
        constexpr int C = gather_chunk(LQ);
#pragma unroll
        for (int k0 = 0; k0 < LQ; k0 += C) {
            float4 g[C];
            if constexpr (MODE == 2)
                gather_planes<C>(x, idx, n, Mq, 4 * t, k0, g);
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int k = k0 + c;
                const uint64_t i0 = (uint64_t)k * Mq + 4 * t;
                if (k < LQ && i0 < n) {
                    const float4 v = MODE == 2 ? g[c] : load4m<MODE>(x, idx, i0, n);
                    const uint4 m = mask_levels4(mk, i0);
                    const int4 q = ms_select4<KIND>(v, quot4_exact(v, dv), lv, rng, i0, m);
                    const uint32_t sh = (uint32_t)k * wq;
                    acc.x |= (uint32_t)(min(max(q.x, -qmax), qmax) + qmax) << sh;
                    acc.y |= (i0 + 1 < n ? (uint32_t)(min(max(q.y, -qmax), qmax) + qmax) : 0u) << sh;
                    acc.z |= (i0 + 2 < n ? (uint32_t)(min(max(q.z, -qmax), qmax) + qmax) : 0u) << sh;
                    acc.w |= (i0 + 3 < n ? (uint32_t)(min(max(q.w, -qmax), qmax) + qmax) : 0u) << sh;
                }
            }
        }
        *reinterpret_cast<uint4 *>(words + 4 * t) = acc;
    }
}

__device__ __forceinline__ float ms_dq(int32_t Q, float norm, float s, int order, float alpha)
{
    const float d = order ? (norm / s) * (float)Q : ((float)Q * norm) / s;
    return d * alpha;
}

template <int LQ, int MODE>
__global__ __launch_bounds__(kBlock) void k_ms_decode(const uint32_t *__restrict__ words, MaskArg mk,
                                                      const int64_t *__restrict__ idx, uint64_t n,
                                                      const float *__restrict__ normp, LevelsArg lv, uint64_t Mq,
                                                      uint32_t wq, int32_t sub, int order, float alpha,
                                                      float *__restrict__ out, SegArg sg)
{
    const float norm = *normp;
    const uint32_t msk = wq >= 32 ? 0xffffffffu : ((1u << wq) - 1u);
    const uint64_t quads = Mq >> 2;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < quads; t += (uint64_t)gridDim.x * kBlock) {
        const uint4 wd = *reinterpret_cast<const uint4 *>(words + 4 * t);
        constexpr int C = gather_chunk(LQ);
#pragma unroll
        for (int k0 = 0; k0 < LQ; k0 += C) {
          int64_t id[C][4];
          if constexpr (MODE == 2 || MODE == 4)  // GRandK scatter: the chunk's index loads together
              gather_idx<C>(idx, n, Mq, 4 * t, k0, id);
#pragma unroll
          for (int c = 0; c < C; ++c) {
            const int k = k0 + c;
            const uint64_t i0 = (uint64_t)k * Mq + 4 * t;
            if (k < LQ && i0 < n) {
                const uint4 m = mask_levels4(mk, i0);
                const uint32_t sh = (uint32_t)k * wq;
                float4 o;
                o.x = ms_dq((int32_t)((wd.x >> sh) & msk) - sub, norm, sel_level(lv, m.x), order, alpha);
                o.y = ms_dq((int32_t)((wd.y >> sh) & msk) - sub, norm, sel_level(lv, m.y), order, alpha);
                o.z = ms_dq((int32_t)((wd.z >> sh) & msk) - sub, norm, sel_level(lv, m.z), order, alpha);
                o.w = ms_dq((int32_t)((wd.w >> sh) & msk) - sub, norm, sel_level(lv, m.w), order, alpha);
                if (MODE == 3) {
                    seg_store4(sg, i0, n, o);
                } else if (MODE == 4) {  // GRandK scatter into the tensors: the setgrad's 0 + RN(alpha d)
                    for (int e = 0; e < 4; ++e)
                        if (i0 + e < n) {
                            const uint64_t id_e = (uint64_t)id[c][e];
                            const SegPos p = seg_find(sg, id_e);
                            p.r.ptr[id_e - p.r.start] = pickf(o, e) + 0.0f;
                        }
                } else if (MODE == 0 && i0 + 4 <= n) {
                    *reinterpret_cast<float4 *>(out + i0) = o;
                } else {
                    for (int e = 0; e < 4; ++e)
                        if (i0 + e < n)
                            out[MODE == 2 ? id[c][e] : i0 + e] = pickf(o, e);
                }
            }
          }
        }
    }
}

// ---------------------------------------------------------------------------
// unpacked (int8 mask / int8|int32 q) forms — the literal compressor drop-in
// ---------------------------------------------------------------------------
template <int KIND, int MODE>
__global__ __launch_bounds__(kBlock) void k_ms_quantize_mask(const float *__restrict__ x, uint64_t n,
                                                             const float *__restrict__ normp, LevelsArg lv,
                                                             RngArgs rng, int8_t *__restrict__ mask)
{
    const float norm = *normp;
    const DivNorm dv = make_div(norm);
    const uint64_t groups = (n + 3) >> 2;
    for (uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x; g < groups; g += (uint64_t)gridDim.x * kBlock) {
        const uint64_t i0 = g << 2;
        const float4 v = load4m<MODE>(x, nullptr, i0, n);
        const uint4 m = ms_levels4<KIND>(quot4_exact(v, dv), lv, rng, i0);
        for (int e = 0; e < 4; ++e)
            if (i0 + e < n)
                mask[i0 + e] = (int8_t)pick(m, e);
    }
}

template <int KIND, int MODE, typename QT>
__global__ __launch_bounds__(kBlock) void k_ms_select_quantize(const float *__restrict__ x, uint64_t n,
                                                               const float *__restrict__ normp, LevelsArg lv,
                                                               RngArgs rng, const int8_t *__restrict__ mask,
                                                               QT *__restrict__ q)
{
    const float norm = *normp;
    const DivNorm dv = make_div(norm);
    const uint64_t groups = (n + 3) >> 2;
    for (uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x; g < groups; g += (uint64_t)gridDim.x * kBlock) {
        const uint64_t i0 = g << 2;
        const float4 v = load4m<MODE>(x, nullptr, i0, n);
        uint4 m;
        m.x = (uint32_t)mask[i0];
        m.y = i0 + 1 < n ? (uint32_t)mask[i0 + 1] : 0u;
        m.z = i0 + 2 < n ? (uint32_t)mask[i0 + 2] : 0u;
        m.w = i0 + 3 < n ? (uint32_t)mask[i0 + 3] : 0u;
        const int4 qq = ms_select4<KIND>(v, quot4_exact(v, dv), lv, rng, i0, m);
        if (i0 + 0 < n) q[i0 + 0] = (QT)qq.x;
        if (i0 + 1 < n) q[i0 + 1] = (QT)qq.y;
        if (i0 + 2 < n) q[i0 + 2] = (QT)qq.z;
        if (i0 + 3 < n) q[i0 + 3] = (QT)qq.w;
    }
}

template <typename QT>
__global__ __launch_bounds__(kBlock) void k_ms_dequantize(const QT *__restrict__ q, const int8_t *__restrict__ mask,
                                                          uint64_t n, const float *__restrict__ normp, LevelsArg lv,
                                                          int order, float alpha, float *__restrict__ out)
{
    const float norm = *normp;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock)
        out[i] = ms_dq((int32_t)q[i], norm, sel_level(lv, (uint32_t)mask[i]), order, alpha);
}

__global__ __launch_bounds__(kBlock) void k_ms_mask_unpack(MaskArg mk, uint64_t n, int8_t *__restrict__ mask)
{
    const uint32_t msk = (1u << mk.w) - 1u;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        const uint64_t plane = i / mk.M, pos = i - plane * mk.M;
        uint32_t m = 0;
        for (uint32_t f = 0; f < mk.fields; ++f)
            m += ((mk.words[f * mk.M + pos] >> ((uint32_t)plane * mk.w)) & msk) == mk.world;
        mask[i] = (int8_t)m;
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static LevelsArg levels_arg(const gc_levels *lv)
{
    LevelsArg a;
    a.count = lv->count;
    a.maxv = (int32_t)((1u << lv->bits[0]) - 1u);
    for (int i = 0; i < GC_MAX_LEVELS; ++i)
        a.s[i] = i < (int)lv->count ? (float)((1u << lv->bits[i]) - 1u) : 1.0f;
    return a;
}

static int check_rng_ms(const gc_rng *r, const char *what)
{
    GC_REQUIRE(r, "%s: null rng", what);
    GC_REQUIRE(r->kind == GC_RNG_PHILOX || r->kind == GC_RNG_STREAM, "%s: unknown rng kind", what);
    GC_REQUIRE(r->kind != GC_RNG_STREAM || r->stream, "%s: STREAM rng without stream", what);
    return GC_OK;
}

static RngArgs rng_args_ms(const gc_rng *r, uint64_t n)
{
    RngArgs a;
    a.seed = r->seed;
    a.offset = r->offset;
    a.stream = r->stream;
    a.n = n;
    return a;
}

static int check_mask_lanes(const gc_lanes *ml, const gc_levels *lv, uint64_t n, const char *what)
{
    int rc = check_lanes(ml, n, what);
    if (rc)
        return rc;
    GC_REQUIRE(ml->range == 1 && ml->offset == 0, "%s: mask lanes not made by gc_ms_mask_layout", what);
    GC_REQUIRE(lv->count >= 2, "%s: needs >= 2 levels", what);
    return GC_OK;
}

static int check_q_lanes(const gc_lanes *ql, const gc_levels *lv, uint64_t n, const char *what)
{
    int rc = check_lanes(ql, n, what);
    if (rc)
        return rc;
    gc_lanes ref;
    if ((rc = gc_ms_layout(n, lv, ql->world, &ref)))
        return rc;
    GC_REQUIRE(ref.offset == ql->offset && ref.range == ql->range, "%s: q lanes not made by gc_ms_layout", what);
    return GC_OK;
}

static MaskArg mask_arg(const uint32_t *w, const gc_lanes *ml, uint32_t count)
{
    MaskArg m;
    m.words = w;
    m.M = ml->plane_words;
    m.w = ml->bits;
    m.fields = count - 1;
    m.world = ml->world;
    return m;
}


// dense fast path (ms_fast.h): aligned dense x, n < 2^32, the lowest level
// <= 7 bits (its xi reaches s_0 and must fit the signed integer rounding), the
// others <= 24 bits (s * 2^24 exact; their T saturates once xi >= 128, which
// only ever means "not this level": fused_quad_fast)
static bool ms_fast_ok(int mode, uint64_t n, const gc_levels *lv)
{
    return mode == 0 && n < (1ull << 32) && (lv->count == 2 || lv->count == 3) && lv->bits[0] <= 7 &&
           lv->bits[lv->count - 1] <= 24;
}

// a lowest level of 8-24 bits: the same wave-split kernels with generic rounding (MSV_WIDE)
static bool ms_fast_wide_ok(int mode, uint64_t n, const gc_levels *lv)
{
    return mode == 0 && n < (1ull << 32) && (lv->count == 2 || lv->count == 3) && lv->bits[lv->count - 1] <= 24;
}

// dense fast decode (k_ms_decode_fast): no rounding, so no 7-bit limit; the
// order-0 Markstein quotient by s = 2^b - 1 is exhaustively checked for
// b = 1..16 (profiles/r01q_divcheck_levels.log)
static bool ms_fast_decode_ok(int mode, uint64_t n, const gc_levels *lv)
{
    return mode == 0 && n < (1ull << 32) && (lv->count == 2 || lv->count == 3) && lv->bits[lv->count - 1] <= 16;
}

static MsFastArg ms_fast_arg(const gc_levels *lv)
{
    MsFastArg a;
    for (int i = 0; i < GC_MAX_LEVELS; ++i) {
        const float s = i < (int)lv->count ? (float)((1u << lv->bits[i]) - 1u) : 1.0f;
        a.S24[i] = s * 16777216.0f;
        a.y[i] = 1.0f / s;
    }
    a.thr = -(int32_t)((1u << lv->bits[0]) - 1u) * (1 << 24);
    return a;
}

// blocks of the wave-split fast kernels: one per 64 word quads (ms_fast.h)
static unsigned ms_grid(uint64_t quads)
{
    const uint64_t b = (quads + kMsQuadsPerBlock - 1) / kMsQuadsPerBlock;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(b, 65535));
}

// tiles (64 word quads) per block of the wave-split kernels.  One: two or more
// amortise the prologue (the norm's reciprocal and range bounds, 60-75 VALU
// per wave; 43.2 -> 40.5 VALU per element for the one-pass encode at two) but
// halve the waves in flight, and the kernels are slower (one-pass 35.1 /
// 38.7 / 42.6 / 54.6 us at 1 / 2 / 3 / 4 tiles, mask + cache 35.7 / 38.5 /
// 41.5 / 46.4 us; profiles/r03k_lab_ms_t*.log).  GC_MS_FUSED_TILES overrides
// it (measurement only)
static uint64_t ms_tiles_env()
{
    static const uint64_t t = [] {
        const char *e = getenv("GC_MS_FUSED_TILES");
        const long v = e ? atol(e) : 0;
        return (uint64_t)(v >= 1 && v <= 64 ? v : 0);
    }();
    return t;
}

static uint64_t ms_tiles() { return ms_tiles_env() ? ms_tiles_env() : 1; }

// tiles per block of the W = 1 one-pass octet kernel with r waves per block:
// two from r = 5 (the 5-bit q lanes of levels (4, 8): 6 per word), whose
// blocks of five waves run 5 x 6 planes per tile (38.8 -> 35.3 us on the
// ResNet50 bucket, 3 tiles 39.7: profiles/r06y_ms_tiles_ab.json); one below
static uint64_t ms_w1_tiles(uint32_t r) { return ms_tiles_env() ? ms_tiles_env() : (r >= 5 ? 2 : 1); }

// planes per load batch of the one-pass W = 1 encode (k_ms_fused_w1's U) for
// two levels with Philox draws: 2 (33.7-33.9 against 34.9-35.0 us at U = 1 on
// the ResNet50 bucket, 73 against 57 VGPRs; U = 3 the same as 2:
// profiles/r03s_ms_sweep_u*.log).  GC_MS_FUSED_U=1 selects the one-plane loop
// (measurement only)
// the select from the q cache with two word quads per lane (k_ms_select_cache_o2);
// GC_MS_SELECT_CACHE_OCTETS=0 keeps one quad per lane (A/B)
static bool ms_select_cache_octets()
{
    static const bool on = [] {
        const char *e = getenv("GC_MS_SELECT_CACHE_OCTETS");
        return !(e && atol(e) == 0);
    }();
    return on;
}

static int ms_fused_u()
{
    static const int u = [] {
        const char *e = getenv("GC_MS_FUSED_U");
        return e && atol(e) == 1 ? 1 : 2;
    }();
    return u;
}

// q cache geometry (ms_fast.h): cell bytes per element (0 = not supported:
// outside the dense wave-split kernels, or the count fields of cb bits exceed
// 16 bits).  Levels of 8-24 bits (MSV_WIDE) cache too: the cell holds the
// lane (q clamped to +-qmax, qmax = 2^bits[0] - 1), not the level's raw q.
struct CacheGeom {
    uint32_t bytes, cb;
    int32_t qmax;
};

static CacheGeom ms_cache_geom(uint64_t n, const gc_levels *lv)
{
    CacheGeom g{0, 0, 0};
    gc_lanes ql;
    if (!ms_fast_wide_ok(0, n, lv) || gc_ms_layout(n, lv, 1, &ql) != GC_OK)
        return g;
    const uint64_t span = 2ull * ql.offset;  // lane values 0 .. 2 qmax
    uint32_t cb = 0;
    while ((span >> cb) != 0)
        ++cb;
    const uint32_t bits = cb * lv->count;
    g.bytes = bits <= 8 ? 1u : (bits <= 16 ? 2u : 0u);
    g.cb = cb;
    g.qmax = (int32_t)ql.offset;
    return g;
}

#define GC_DISPATCH_L2(L, ...)                                                   \
    switch (L) {                                                                 \
    case 1: { constexpr int LL = 1; __VA_ARGS__; } break;                        \
    case 2: { constexpr int LL = 2; __VA_ARGS__; } break;                        \
    case 3: { constexpr int LL = 3; __VA_ARGS__; } break;                        \
    case 4: { constexpr int LL = 4; __VA_ARGS__; } break;                        \
    case 5: { constexpr int LL = 5; __VA_ARGS__; } break;                        \
    case 6: { constexpr int LL = 6; __VA_ARGS__; } break;                        \
    case 8: { constexpr int LL = 8; __VA_ARGS__; } break;                        \
    case 10: { constexpr int LL = 10; __VA_ARGS__; } break;                      \
    case 16: { constexpr int LL = 16; __VA_ARGS__; } break;                      \
    case 32: { constexpr int LL = 32; __VA_ARGS__; } break;                      \
    default: return fail(GC_EINVAL, "unsupported lanes per word %u", (unsigned)(L)); \
    }

}  // namespace gc

using namespace gc;

extern "C" {

int gc_ms_encode_w1(const float *x, uint64_t n, const float *norm, const gc_levels *levels, const gc_rng *rng,
                    const gc_lanes *mask_lanes, const gc_lanes *q_lanes, uint32_t *mask_words, uint32_t *words,
                    gc_stream_t stream)
{
    int rc;
    if ((rc = check_levels(levels, "gc_ms_encode_w1")) || (rc = check_rng_ms(rng, "gc_ms_encode_w1")) ||
        (rc = check_mask_lanes(mask_lanes, levels, n, "gc_ms_encode_w1")) ||
        (rc = check_q_lanes(q_lanes, levels, n, "gc_ms_encode_w1")))
        return rc;
    GC_REQUIRE(mask_lanes->world == 1 && q_lanes->world == 1, "gc_ms_encode_w1: lanes for W = 1 only");
    GC_REQUIRE(norm && mask_words && words && (n == 0 || x), "gc_ms_encode_w1: null pointer");
    GC_REQUIRE(aligned16(mask_words) && aligned16(words), "gc_ms_encode_w1: streams must be 16-byte aligned");
    const uint32_t r = 32u / q_lanes->per_word;
    GC_REQUIRE(mask_lanes->per_word == 32 && r <= kMsFusedMaxR && q_lanes->plane_words == (uint64_t)r * mask_lanes->plane_words,
               "gc_ms_encode_w1: layouts not coupled (gc_ms_layout / gc_ms_mask_layout at W = 1)");
    const int mode = aligned16(x) ? 0 : 1;
    GC_REQUIRE(ms_fast_wide_ok(mode, n, levels),
               "gc_ms_encode_w1: needs a dense 16-byte aligned x, n < 2^32 and 2 or 3 levels of <= 24 bits");
    if (mask_lanes->plane_words == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const LevelsArg la = levels_arg(levels);
    const RngArgs ra = rng_args_ms(rng, n);
    const MsFastArg fa = ms_fast_arg(levels);
    const uint32_t Mm = (uint32_t)mask_lanes->plane_words;
    const unsigned g = (unsigned)std::max<uint64_t>(1, (ms_grid(Mm >> 2) + ms_tiles() - 1) / ms_tiles());
    const bool wide = !ms_fast_ok(mode, n, levels);
    const int32_t qmax = (int32_t)q_lanes->offset;
    uint32_t Cw = 0;
    for (uint32_t k = 0; k < q_lanes->per_word; ++k)
        Cw += (uint32_t)qmax << (k * q_lanes->bits);
    const uint32_t pend = (uint32_t)((n + Mm - 1) / Mm);
#define GC_FW(KIND_, NL_, ...)                                                                                     \
    hipLaunchKernelGGL((k_ms_fused_w1<KIND_, NL_, __VA_ARGS__>), dim3(g), dim3(64 * r), 0, st, x, (uint32_t)n, norm, la, \
                       fa, ra, Mm, r, q_lanes->per_word, q_lanes->bits, qmax, Cw, pend, mask_words, words)
    if (levels->count == 2) {
        if (rng->kind == GC_RNG_PHILOX && Mm % 8 == 0) {  // the octet kernel: dense draws shared by 8 elements
            const unsigned g8 = (unsigned)std::max<uint64_t>(1, (ms_grid(Mm >> 3) + ms_w1_tiles(r) - 1) / ms_w1_tiles(r));
#define GC_FW8(VAR_)                                                                                                \
    hipLaunchKernelGGL((k_ms_fused_w1_o2<VAR_>), dim3(g8), dim3(64 * r), 0, st, x, (uint32_t)n, norm, la, fa, ra, Mm, r, \
                       q_lanes->per_word, q_lanes->bits, qmax, Cw, pend, mask_words, words)
            // plain stores: the decode that follows at W = 1 reads these words
            // and mask words at once (profiles/r05zh_lab_ms.log)
            if (wide) { GC_FW8(MSV_WIDE | MSV_PREFETCH | MSV_PLAINST); } else { GC_FW8(MSV_PREFETCH | MSV_PLAINST); }
#undef GC_FW8
        } else if (rng->kind == GC_RNG_PHILOX) {
            if (wide) { GC_FW(2, 2, MSV_WIDE); }
            else if (ms_fused_u() == 2) { GC_FW(2, 2, MSV_EAGER0, 2); }
            else { GC_FW(2, 2, MSV_EAGER0); }
        }
        else { if (wide) { GC_FW(1, 2, MSV_WIDE); } else { GC_FW(1, 2, 0); } }
    } else {
        if (rng->kind == GC_RNG_PHILOX) { if (wide) { GC_FW(0, 3, MSV_WIDE); } else { GC_FW(0, 3, MSV_EAGER0); } }
        else { if (wide) { GC_FW(1, 3, MSV_WIDE); } else { GC_FW(1, 3, 0); } }
    }
#undef GC_FW
    return launch_status("gc_ms_encode_w1");
}

int gc_ms_mask_encode(const float *x, const int64_t *idx, uint64_t n, const float *norm, const gc_levels *levels,
                      const gc_rng *rng, const gc_lanes *mask_lanes, uint32_t *mask_words, gc_stream_t stream)
{
    int rc;
    if ((rc = check_levels(levels, "gc_ms_mask_encode")) || (rc = check_rng_ms(rng, "gc_ms_mask_encode")) ||
        (rc = check_mask_lanes(mask_lanes, levels, n, "gc_ms_mask_encode")))
        return rc;
    GC_REQUIRE(norm && mask_words && (n == 0 || x), "gc_ms_mask_encode: null pointer");
    GC_REQUIRE(aligned16(mask_words), "gc_ms_mask_encode: mask_words must be 16-byte aligned");
    if (mask_lanes->plane_words == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const LevelsArg la = levels_arg(levels);
    const RngArgs ra = rng_args_ms(rng, n);
    const int mode = idx ? 2 : (aligned16(x) ? 0 : 1);
    const unsigned grid = grid_for(mask_lanes->plane_words >> 2);
    const uint64_t M = mask_lanes->plane_words;
    const uint32_t w = mask_lanes->bits, fields = levels->count - 1;
#define GC_ME(KIND_, MODE_)                                                                                       \
    GC_DISPATCH_L2(mask_lanes->per_word, hipLaunchKernelGGL((k_ms_mask_encode<LL, KIND_, MODE_>), dim3(grid),    \
                                                            dim3(kBlock), 0, st, x, idx, n, norm, la, ra, M, w,  \
                                                            fields, mask_words))
    if (ms_fast_wide_ok(mode, n, levels)) {
        const MsFastArg fa = ms_fast_arg(levels);
        const unsigned g = (unsigned)std::max<uint64_t>(1, (ms_grid(M >> 2) + ms_tiles() - 1) / ms_tiles());
        const bool wide = !ms_fast_ok(mode, n, levels);
#define GC_MF(KIND_, NL_)                                                                                         \
    if (wide)                                                                                                     \
        GC_DISPATCH_L2(mask_lanes->per_word,                                                                      \
                       hipLaunchKernelGGL((k_ms_mask_fast<LL, KIND_, NL_, MSV_WIDE>), dim3(g), dim3(kBlock), 0, st, \
                                          x, (uint32_t)n, norm, la, fa, ra, (uint32_t)M, w, fields, mask_words,   \
                                          (void *)nullptr, 0, 0u))                                                \
    else                                                                                                          \
    GC_DISPATCH_L2(mask_lanes->per_word, hipLaunchKernelGGL((k_ms_mask_fast<LL, KIND_, NL_>), dim3(g), dim3(kBlock), 0, \
                                                            st, x, (uint32_t)n, norm, la, fa, ra, (uint32_t)M, w,  \
                                                            fields, mask_words, (void *)nullptr, 0, 0u))
        if (levels->count == 2 && rng->kind == GC_RNG_PHILOX && M % 8 == 0) {
            const unsigned g8 = (unsigned)std::max<uint64_t>(1, (ms_grid(M >> 3) + ms_tiles() - 1) / ms_tiles());
#define GC_MF8(VAR_)                                                                                               \
    GC_DISPATCH_L2(mask_lanes->per_word, hipLaunchKernelGGL((k_ms_mask_fast_o2<LL, VAR_>), dim3(g8), dim3(kBlock), 0, \
                                                            st, x, (uint32_t)n, norm, la, fa, ra, (uint32_t)M, w,      \
                                                            mask_words, (void *)nullptr, 0, 0u))
            if (wide) { GC_MF8(MSV_WIDE | MSV_ROLL | MSV_PLAINST); } else { GC_MF8(MSV_ROLL | MSV_UFLAG | MSV_PLAINST); }
#undef GC_MF8
        } else if (levels->count == 2) {
            if (rng->kind == GC_RNG_PHILOX) { GC_MF(2, 2); } else { GC_MF(1, 2); }
        } else {
            if (rng->kind == GC_RNG_PHILOX) { GC_MF(0, 3); } else { GC_MF(1, 3); }
        }
#undef GC_MF
    } else if (rng->kind == GC_RNG_PHILOX && levels->count == 2) {
        if (mode == 0) { GC_ME(2, 0); } else if (mode == 1) { GC_ME(2, 1); } else { GC_ME(2, 2); }
    } else if (rng->kind == GC_RNG_PHILOX) {
        if (mode == 0) { GC_ME(0, 0); } else if (mode == 1) { GC_ME(0, 1); } else { GC_ME(0, 2); }
    } else {
        if (mode == 0) { GC_ME(1, 0); } else if (mode == 1) { GC_ME(1, 1); } else { GC_ME(1, 2); }
    }
#undef GC_ME
    return launch_status("gc_ms_mask_encode");
}

int gc_ms_select_encode(const float *x, const int64_t *idx, uint64_t n, const float *norm, const gc_levels *levels,
                        const gc_rng *rng, const uint32_t *mask_words, const gc_lanes *mask_lanes,
                        const gc_lanes *q_lanes, uint32_t *words, gc_stream_t stream)
{
    int rc;
    if ((rc = check_levels(levels, "gc_ms_select_encode")) || (rc = check_rng_ms(rng, "gc_ms_select_encode")) ||
        (rc = check_mask_lanes(mask_lanes, levels, n, "gc_ms_select_encode")) ||
        (rc = check_q_lanes(q_lanes, levels, n, "gc_ms_select_encode")))
        return rc;
    GC_REQUIRE(norm && mask_words && words && (n == 0 || x), "gc_ms_select_encode: null pointer");
    GC_REQUIRE(aligned16(words) && aligned16(mask_words), "gc_ms_select_encode: words must be 16-byte aligned");
    if (q_lanes->plane_words == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const LevelsArg la = levels_arg(levels);
    const RngArgs ra = rng_args_ms(rng, n);
    const MaskArg mk = mask_arg(mask_words, mask_lanes, levels->count);
    const int mode = idx ? 2 : (aligned16(x) ? 0 : 1);
    const unsigned grid = grid_for(q_lanes->plane_words >> 2);
    const uint64_t Mq = q_lanes->plane_words;
    const uint32_t wq = q_lanes->bits;
    const int32_t qmax = (int32_t)q_lanes->offset;
#define GC_SE(KIND_, MODE_)                                                                                        \
    GC_DISPATCH_L2(q_lanes->per_word, hipLaunchKernelGGL((k_ms_select_encode<LL, KIND_, MODE_>), dim3(grid),       \
                                                         dim3(kBlock), 0, st, x, idx, n, norm, la, ra, mk, Mq, wq, \
                                                         qmax, words))
    if (ms_fast_wide_ok(mode, n, levels) && mask_lanes->plane_words >= 2 && mask_lanes->plane_words < (1ull << 32)) {
        const MsFastArg fa = ms_fast_arg(levels);
        const FastDiv fd = make_fastdiv((uint32_t)mask_lanes->plane_words);
        const unsigned g = (unsigned)std::max<uint64_t>(1, (ms_grid(Mq >> 2) + ms_tiles() - 1) / ms_tiles());
        const bool wide = !ms_fast_ok(mode, n, levels);
#define GC_SF(KIND_, NL_)                                                                                             \
    if (wide)                                                                                                         \
        GC_DISPATCH_L2(q_lanes->per_word,                                                                             \
                       hipLaunchKernelGGL((k_ms_select_fast<LL, KIND_, NL_, MSV_WIDE>), dim3(g), dim3(kBlock), 0, st,   \
                                          x, (uint32_t)n, norm, la, fa, ra, mk, fd, (uint32_t)Mq, wq, qmax, words))  \
    else                                                                                                              \
    GC_DISPATCH_L2(q_lanes->per_word, hipLaunchKernelGGL((k_ms_select_fast<LL, KIND_, NL_>), dim3(g), dim3(kBlock), 0,   \
                                                         st, x, (uint32_t)n, norm, la, fa, ra, mk, fd, (uint32_t)Mq, \
                                                         wq, qmax, words))
        if (levels->count == 2 && rng->kind == GC_RNG_PHILOX && Mq % 8 == 0) {
            const unsigned g8 = (unsigned)std::max<uint64_t>(1, (ms_grid(Mq >> 3) + ms_tiles() - 1) / ms_tiles());
#define GC_SF8(VAR_)                                                                                                \
    GC_DISPATCH_L2(q_lanes->per_word, hipLaunchKernelGGL((k_ms_select_fast_o2<LL, VAR_>), dim3(g8), dim3(kBlock), 0, st, \
                                                         x, (uint32_t)n, norm, la, fa, ra, mk, fd, (uint32_t)Mq, wq,  \
                                                         qmax, words))
            if (wide) { GC_SF8(MSV_WIDE | MSV_ROLL | MSV_PLAINST); } else { GC_SF8(MSV_ROLL | MSV_PLAINST); }
#undef GC_SF8
        } else if (levels->count == 2) {
            if (rng->kind == GC_RNG_PHILOX) { GC_SF(2, 2); } else { GC_SF(1, 2); }
        } else {
            if (rng->kind == GC_RNG_PHILOX) { GC_SF(0, 3); } else { GC_SF(1, 3); }
        }
#undef GC_SF
    } else if (rng->kind == GC_RNG_PHILOX && levels->count == 2) {
        if (mode == 0) { GC_SE(2, 0); } else if (mode == 1) { GC_SE(2, 1); } else { GC_SE(2, 2); }
    } else if (rng->kind == GC_RNG_PHILOX) {
        if (mode == 0) { GC_SE(0, 0); } else if (mode == 1) { GC_SE(0, 1); } else { GC_SE(0, 2); }
    } else {
        if (mode == 0) { GC_SE(1, 0); } else if (mode == 1) { GC_SE(1, 1); } else { GC_SE(1, 2); }
    }
#undef GC_SE
    return launch_status("gc_ms_select_encode");
}

int gc_ms_cache_bytes(uint64_t n, const gc_levels *levels, uint32_t *bytes_per_element)
{
    int rc = check_levels(levels, "gc_ms_cache_bytes");
    if (rc)
        return rc;
    GC_REQUIRE(bytes_per_element, "gc_ms_cache_bytes: null output");
    *bytes_per_element = levels->count >= 2 ? ms_cache_geom(n, levels).bytes : 0u;
    return GC_OK;
}

int gc_ms_mask_encode_cached(const float *x, uint64_t n, const float *norm, const gc_levels *levels,
                             const gc_rng *rng, const gc_lanes *mask_lanes, uint32_t *mask_words, void *cache,
                             gc_stream_t stream)
{
    const char *what = "gc_ms_mask_encode_cached";
    int rc;
    if ((rc = check_levels(levels, what)) || (rc = check_rng_ms(rng, what)) ||
        (rc = check_mask_lanes(mask_lanes, levels, n, what)))
        return rc;
    const CacheGeom cg = ms_cache_geom(n, levels);
    GC_REQUIRE(cg.bytes, "%s: no q cache for these levels / n (gc_ms_cache_bytes == 0)", what);
    GC_REQUIRE(norm && mask_words && (n == 0 || (x && cache)), "%s: null pointer", what);
    GC_REQUIRE(aligned16(mask_words) && (n == 0 || (aligned16(x) && aligned16(cache))),
               "%s: x, mask_words and cache must be 16-byte aligned", what);
    if (mask_lanes->plane_words == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const LevelsArg la = levels_arg(levels);
    const RngArgs ra = rng_args_ms(rng, n);
    const MsFastArg fa = ms_fast_arg(levels);
    const uint32_t M = (uint32_t)mask_lanes->plane_words, w = mask_lanes->bits, fields = levels->count - 1;
    const unsigned g = (unsigned)std::max<uint64_t>(1, (ms_grid(M >> 2) + ms_tiles() - 1) / ms_tiles());
    const bool wide = !ms_fast_ok(0, n, levels);
#define GC_MFC(KIND_, NL_, VAR_, CBY_)                                                                                \
    GC_DISPATCH_L2(mask_lanes->per_word,                                                                             \
                   hipLaunchKernelGGL((k_ms_mask_fast<LL, KIND_, NL_, VAR_, CBY_>), dim3(g), dim3(kBlock), 0, st, x,  \
                                      (uint32_t)n, norm, la, fa, ra, M, w, fields, mask_words, cache, cg.qmax, cg.cb))
#define GC_MFC_V(KIND_, NL_, CBY_) \
    if (wide) { GC_MFC(KIND_, NL_, MSV_WIDE, CBY_); } else { GC_MFC(KIND_, NL_, 0, CBY_); }
#define GC_MFC_K(NL_, CBY_) \
    if (rng->kind == GC_RNG_PHILOX) { GC_MFC_V(NL_ == 2 ? 2 : 0, NL_, CBY_); } else { GC_MFC_V(1, NL_, CBY_); }
#define GC_MFC8(VAR_, CBY_)                                                                                           \
    GC_DISPATCH_L2(mask_lanes->per_word,                                                                             \
                   hipLaunchKernelGGL((k_ms_mask_fast_o2<LL, VAR_, CBY_>), dim3(g8), dim3(kBlock), 0, st, x, (uint32_t)n, \
                                      norm, la, fa, ra, M, w, mask_words, cache, cg.qmax, cg.cb))
    if (levels->count == 2 && rng->kind == GC_RNG_PHILOX && M % 8 == 0) {  // octets: dense draws, 3 blocks per 8
        const unsigned g8 = (unsigned)std::max<uint64_t>(1, (ms_grid(M >> 3) + ms_tiles() - 1) / ms_tiles());
        if (cg.bytes == 1) {
            if (wide) { GC_MFC8(MSV_WIDE | MSV_ROLL | MSV_PLAINST, 1); } else { GC_MFC8(MSV_ROLL | MSV_UFLAG | MSV_PLAINST, 1); }
        } else {
            if (wide) { GC_MFC8(MSV_WIDE | MSV_ROLL | MSV_PLAINST, 2); } else { GC_MFC8(MSV_ROLL | MSV_UFLAG | MSV_PLAINST, 2); }
        }
    } else if (levels->count == 2) {
        if (cg.bytes == 1) { GC_MFC_K(2, 1) } else { GC_MFC_K(2, 2) }
    } else {
        if (cg.bytes == 1) { GC_MFC_K(3, 1) } else { GC_MFC_K(3, 2) }
    }
#undef GC_MFC8
#undef GC_MFC_K
#undef GC_MFC_V
#undef GC_MFC
    return launch_status(what);
}

int gc_ms_select_cached(const void *cache, uint64_t n, const gc_levels *levels, const uint32_t *mask_words,
                        const gc_lanes *mask_lanes, const gc_lanes *q_lanes, uint32_t *words, gc_stream_t stream)
{
    const char *what = "gc_ms_select_cached";
    int rc;
    if ((rc = check_levels(levels, what)) || (rc = check_mask_lanes(mask_lanes, levels, n, what)) ||
        (rc = check_q_lanes(q_lanes, levels, n, what)))
        return rc;
    const CacheGeom cg = ms_cache_geom(n, levels);
    GC_REQUIRE(cg.bytes, "%s: no q cache for these levels / n (gc_ms_cache_bytes == 0)", what);
    GC_REQUIRE(mask_words && words && (n == 0 || cache), "%s: null pointer", what);
    GC_REQUIRE(aligned16(words) && aligned16(mask_words) && (n == 0 || aligned16(cache)),
               "%s: words, mask_words and cache must be 16-byte aligned", what);
    if (q_lanes->plane_words == 0)
        return GC_OK;
    GC_REQUIRE(mask_lanes->plane_words >= 2 && mask_lanes->plane_words < (1ull << 32), "%s: mask stream size", what);
    hipStream_t st = as_stream(stream);
    const MaskArg mk = mask_arg(mask_words, mask_lanes, levels->count);
    const FastDiv fd = make_fastdiv((uint32_t)mask_lanes->plane_words);
    const uint32_t Mq = (uint32_t)q_lanes->plane_words;
    const unsigned g = (unsigned)std::max<uint64_t>(1, (ms_grid(Mq >> 2) + ms_tiles() - 1) / ms_tiles());
#define GC_SC(NL_, CBY_)                                                                                            \
    GC_DISPATCH_L2(q_lanes->per_word, hipLaunchKernelGGL((k_ms_select_cache<LL, NL_, CBY_>), dim3(g), dim3(kBlock), 0, \
                                                         st, cache, (uint32_t)n, mk, fd, Mq, q_lanes->bits, cg.cb,    \
                                                         words))
#define GC_SC8(NL_, CBY_)                                                                                           \
    GC_DISPATCH_L2(q_lanes->per_word, hipLaunchKernelGGL((k_ms_select_cache_o2<LL, NL_, CBY_, false>), dim3(g8), dim3(kBlock), \
                                                         0, st, cache, (uint32_t)n, mk, fd, Mq, q_lanes->bits, cg.cb, \
                                                         words))
    if (Mq % 8 == 0 && ms_select_cache_octets()) {  // two quads per lane
        const unsigned g8 = (unsigned)std::max<uint64_t>(1, (ms_grid(Mq >> 3) + ms_tiles() - 1) / ms_tiles());
        if (levels->count == 2) {
            if (cg.bytes == 1) { GC_SC8(2, 1); } else { GC_SC8(2, 2); }
        } else {
            if (cg.bytes == 1) { GC_SC8(3, 1); } else { GC_SC8(3, 2); }
        }
    } else if (levels->count == 2) {
        if (cg.bytes == 1) { GC_SC(2, 1); } else { GC_SC(2, 2); }
    } else {
        if (cg.bytes == 1) { GC_SC(3, 1); } else { GC_SC(3, 2); }
    }
#undef GC_SC8
#undef GC_SC
    return launch_status(what);
}

static int ms_decode(const char *what, const uint32_t *words, const uint32_t *mask_words, const int64_t *idx,
                     uint64_t n, const float *norm, const gc_levels *levels, const gc_lanes *mask_lanes,
                     const gc_lanes *q_lanes, int order, float alpha, float *out, const gc_segments *segs,
                     gc_stream_t stream)
{
    int rc;
    if ((rc = check_levels(levels, what)) || (rc = check_mask_lanes(mask_lanes, levels, n, what)) ||
        (rc = check_q_lanes(q_lanes, levels, n, what)))
        return rc;
    GC_REQUIRE(mask_lanes->world == q_lanes->world, "%s: mask and q lanes sized for different worlds", what);
    GC_REQUIRE(norm && mask_words && words && (n == 0 || out || segs), "%s: null pointer", what);
    GC_REQUIRE(order == 0 || order == 1, "%s: order must be 0 (multi-scale) or 1 (two-scale)", what);
    GC_REQUIRE(aligned16(words) && aligned16(mask_words), "%s: words must be 16-byte aligned", what);
    SegArg sg{};
    if (segs && (rc = seg_arg(segs, idx ? segs->n : n, &sg, what)))  // with idx: n = K of the table's elements
        return rc;
    if (q_lanes->plane_words == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const LevelsArg la = levels_arg(levels);
    const MaskArg mk = mask_arg(mask_words, mask_lanes, levels->count);
    const int mode = segs ? (idx ? 4 : 3) : idx ? 2 : (aligned16(out) ? 0 : 1);
    const unsigned grid = grid_for(q_lanes->plane_words >> 2);
    const int32_t sub = (int32_t)(q_lanes->world * q_lanes->offset);
#define GC_MD(MODE_)                                                                                               \
    GC_DISPATCH_L2(q_lanes->per_word, hipLaunchKernelGGL((k_ms_decode<LL, MODE_>), dim3(grid), dim3(kBlock), 0, st, \
                                                         words, mk, idx, n, norm, la, q_lanes->plane_words,        \
                                                         q_lanes->bits, sub, order, alpha, out, sg))
    if (ms_fast_decode_ok(mode, n, levels) && mask_lanes->plane_words >= 2 && mask_lanes->plane_words < (1ull << 32)) {
        const MsFastArg fa = ms_fast_arg(levels);
        const FastDiv fd = make_fastdiv((uint32_t)mask_lanes->plane_words);
        // one thread per word quad walking all its planes (MSV_PERTHREAD): each
        // quad's words are read once, not by every wave of the block; the
        // words a decode reads were usually written just before it (by the
        // encode at W = 1, by the SUM otherwise), and re-reading fresh lines
        // from four waves cost more than the split saves (the whole W = 1
        // step 71.6 -> 68.7 us with the one-pass kernel's plain stores,
        // profiles/r05zh_lab_ms.log; the decode alone 18.6 against 19.0 us)
        const unsigned g = (unsigned)std::min<uint64_t>(((q_lanes->plane_words >> 2) + kBlock - 1) / kBlock, 65535);
#define GC_DF(ORD_, NL_)                                                                                               \
    GC_DISPATCH_L2(q_lanes->per_word, hipLaunchKernelGGL((k_ms_decode_fast<LL, ORD_, NL_, MSV_PERTHREAD>), dim3(g),    \
                                                         dim3(kBlock), 0, st, \
                                                         words, mk, fd, (uint32_t)n, norm, la, fa,                  \
                                                         (uint32_t)q_lanes->plane_words, q_lanes->bits, sub, alpha, out))
        if (levels->count == 2) {
            if (order == 0) { GC_DF(0, 2); } else { GC_DF(1, 2); }
        } else {
            if (order == 0) { GC_DF(0, 3); } else { GC_DF(1, 3); }
        }
#undef GC_DF
    } else if (mode == 0) { GC_MD(0); } else if (mode == 1) { GC_MD(1); } else if (mode == 2) { GC_MD(2); }
    else if (mode == 3) { GC_MD(3); } else { GC_MD(4); }
#undef GC_MD
    return launch_status(what);
}

int gc_ms_decode(const uint32_t *words, const uint32_t *mask_words, const int64_t *idx, uint64_t n, const float *norm,
                 const gc_levels *levels, const gc_lanes *mask_lanes, const gc_lanes *q_lanes, int order, float alpha,
                 float *out, gc_stream_t stream)
{
    return ms_decode("gc_ms_decode", words, mask_words, idx, n, norm, levels, mask_lanes, q_lanes, order, alpha, out,
                     nullptr, stream);
}

int gc_ms_decode_segments(const uint32_t *words, const uint32_t *mask_words, uint64_t n, const float *norm,
                          const gc_levels *levels, const gc_lanes *mask_lanes, const gc_lanes *q_lanes, int order,
                          float alpha, const gc_segments *segs, gc_stream_t stream)
{
    GC_REQUIRE(segs, "gc_ms_decode_segments: null segments");
    return ms_decode("gc_ms_decode_segments", words, mask_words, nullptr, n, norm, levels, mask_lanes, q_lanes, order,
                     alpha, nullptr, segs, stream);
}

int gc_ms_decode_scatter_segments(const uint32_t *words, const uint32_t *mask_words, const int64_t *idx, uint64_t k,
                                  const float *norm, const gc_levels *levels, const gc_lanes *mask_lanes,
                                  const gc_lanes *q_lanes, int order, float alpha, const gc_segments *segs,
                                  gc_stream_t stream)
{
    GC_REQUIRE(segs && (k == 0 || idx), "gc_ms_decode_scatter_segments: null segments / idx");
    return ms_decode("gc_ms_decode_scatter_segments", words, mask_words, idx, k, norm, levels, mask_lanes, q_lanes,
                     order, alpha, nullptr, segs, stream);
}

int gc_ms_mask_unpack(const uint32_t *mask_words, const gc_lanes *mask_lanes, uint32_t levels_count, int8_t *mask,
                      gc_stream_t stream)
{
    GC_REQUIRE(mask_lanes && mask_words, "gc_ms_mask_unpack: null pointer");
    int rc = check_lanes(mask_lanes, mask_lanes->n, "gc_ms_mask_unpack");
    if (rc)
        return rc;
    GC_REQUIRE(levels_count >= 2 && levels_count <= GC_MAX_LEVELS, "gc_ms_mask_unpack: bad level count");
    GC_REQUIRE(mask_lanes->n == 0 || mask, "gc_ms_mask_unpack: null mask");
    if (mask_lanes->n == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_ms_mask_unpack, dim3(grid_for(mask_lanes->n)), dim3(kBlock), 0, st,
                       mask_arg(mask_words, mask_lanes, levels_count), mask_lanes->n, mask);
    return launch_status("gc_ms_mask_unpack");
}

int gc_ms_quantize_mask(const float *x, uint64_t n, const float *norm, const gc_levels *levels, const gc_rng *rng,
                        int8_t *mask, gc_stream_t stream)
{
    int rc;
    if ((rc = check_levels(levels, "gc_ms_quantize_mask")) || (rc = check_rng_ms(rng, "gc_ms_quantize_mask")))
        return rc;
    GC_REQUIRE(n == 0 || (x && norm && mask), "gc_ms_quantize_mask: null pointer");
    if (n == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const LevelsArg la = levels_arg(levels);
    const RngArgs ra = rng_args_ms(rng, n);
    const unsigned grid = grid_for((n + 3) >> 2);
    const bool vec = aligned16(x);
    if (rng->kind == GC_RNG_PHILOX && levels->count == 2) {
        if (vec) hipLaunchKernelGGL((k_ms_quantize_mask<2, 0>), dim3(grid), dim3(kBlock), 0, st, x, n, norm, la, ra, mask);
        else hipLaunchKernelGGL((k_ms_quantize_mask<2, 1>), dim3(grid), dim3(kBlock), 0, st, x, n, norm, la, ra, mask);
    } else if (rng->kind == GC_RNG_PHILOX) {
        if (vec) hipLaunchKernelGGL((k_ms_quantize_mask<0, 0>), dim3(grid), dim3(kBlock), 0, st, x, n, norm, la, ra, mask);
        else hipLaunchKernelGGL((k_ms_quantize_mask<0, 1>), dim3(grid), dim3(kBlock), 0, st, x, n, norm, la, ra, mask);
    } else {
        if (vec) hipLaunchKernelGGL((k_ms_quantize_mask<1, 0>), dim3(grid), dim3(kBlock), 0, st, x, n, norm, la, ra, mask);
        else hipLaunchKernelGGL((k_ms_quantize_mask<1, 1>), dim3(grid), dim3(kBlock), 0, st, x, n, norm, la, ra, mask);
    }
    return launch_status("gc_ms_quantize_mask");
}

int gc_ms_select_quantize(const float *x, uint64_t n, const float *norm, const gc_levels *levels, const gc_rng *rng,
                          const int8_t *mask, void *q, uint32_t q_dtype, gc_stream_t stream)
{
    int rc;
    if ((rc = check_levels(levels, "gc_ms_select_quantize")) || (rc = check_rng_ms(rng, "gc_ms_select_quantize")))
        return rc;
    GC_REQUIRE(q_dtype == GC_I8 || q_dtype == GC_I32, "gc_ms_select_quantize: q_dtype must be GC_I8 or GC_I32");
    GC_REQUIRE(n == 0 || (x && norm && mask && q), "gc_ms_select_quantize: null pointer");
    if (n == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const LevelsArg la = levels_arg(levels);
    const RngArgs ra = rng_args_ms(rng, n);
    const unsigned grid = grid_for((n + 3) >> 2);
    const bool vec = aligned16(x);
#define GC_SQ(KIND_, MODE_, QT_)                                                                                \
    hipLaunchKernelGGL((k_ms_select_quantize<KIND_, MODE_, QT_>), dim3(grid), dim3(kBlock), 0, st, x, n, norm, la, \
                       ra, mask, reinterpret_cast<QT_ *>(q))
    if (rng->kind == GC_RNG_PHILOX && levels->count == 2) {
        if (q_dtype == GC_I8) { if (vec) GC_SQ(2, 0, int8_t); else GC_SQ(2, 1, int8_t); }
        else { if (vec) GC_SQ(2, 0, int32_t); else GC_SQ(2, 1, int32_t); }
    } else if (rng->kind == GC_RNG_PHILOX) {
        if (q_dtype == GC_I8) { if (vec) GC_SQ(0, 0, int8_t); else GC_SQ(0, 1, int8_t); }
        else { if (vec) GC_SQ(0, 0, int32_t); else GC_SQ(0, 1, int32_t); }
    } else {
        if (q_dtype == GC_I8) { if (vec) GC_SQ(1, 0, int8_t); else GC_SQ(1, 1, int8_t); }
        else { if (vec) GC_SQ(1, 0, int32_t); else GC_SQ(1, 1, int32_t); }
    }
#undef GC_SQ
    return launch_status("gc_ms_select_quantize");
}

int gc_ms_dequantize(const void *q, uint32_t q_dtype, const int8_t *mask, uint64_t n, const float *norm,
                     const gc_levels *levels, int order, float alpha, float *out, gc_stream_t stream)
{
    int rc;
    if ((rc = check_levels(levels, "gc_ms_dequantize")))
        return rc;
    GC_REQUIRE(q_dtype == GC_I8 || q_dtype == GC_I32, "gc_ms_dequantize: q_dtype must be GC_I8 or GC_I32");
    GC_REQUIRE(order == 0 || order == 1, "gc_ms_dequantize: order must be 0 or 1");
    GC_REQUIRE(n == 0 || (q && mask && norm && out), "gc_ms_dequantize: null pointer");
    if (n == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const LevelsArg la = levels_arg(levels);
    if (q_dtype == GC_I8)
        hipLaunchKernelGGL((k_ms_dequantize<int8_t>), dim3(grid_for(n)), dim3(kBlock), 0, st,
                           reinterpret_cast<const int8_t *>(q), mask, n, norm, la, order, alpha, out);
    else
        hipLaunchKernelGGL((k_ms_dequantize<int32_t>), dim3(grid_for(n)), dim3(kBlock), 0, st,
                           reinterpret_cast<const int32_t *>(q), mask, n, norm, la, order, alpha, out);
    return launch_status("gc_ms_dequantize");
}

}  // extern "C"
