// segments.hip — the reference's TensorBuffer + setgrad (reducer.py:46-68,
// 543-549) as streaming kernels over a gc_segments table:
//   k_seg_flatten_absmax  tensors -> flat bucket, fused with the max-norm scan
//                         (reducer.py:512-516: TensorBuffer(grad_in) then
//                         buffer.abs().max(), one pass instead of two)
//   k_seg_scatter         flat bucket -> tensors, times alpha (the setgrad
//                         loop: out[:] = 0; out.add_(grad, alpha=1/W))
// The fused decode -> tensors is k_qsgd_decode / k_ms_decode MODE 3.
//
// Work split: a block owns a range of kRange consecutive flat elements per
// iteration and walks the (block-uniform) pieces of it that fall in one
// tensor each; inside a piece, if tensor and flat side are co-aligned mod 16 B,
// threads move float4s (4 independent loads in flight per thread), else
// dwords — every wave access is contiguous either way.
#include "gc_device.h"
#include "gc_host.h"
#include "segments.h"

#include <algorithm>

namespace gc {

constexpr uint64_t kRange = 16384;  // flat elements per block iteration (16 per thread)

struct OpFlatten {  // tensor -> flat, max |x| bits
    uint32_t m = 0;
    __device__ __forceinline__ float operator()(float x)
    {
        m = max(m, absbits(x));
        return x;
    }
};

// flat -> tensor.  The reference's setgrad is `out[:] = 0; out.add_(g, alpha)`
// = 0 + RN(alpha * g): the +0 turns -0 into +0 (a local -0 gradient kept by
// GRandK comes out as +0 there, so it must here); no FMA (-ffp-contract=off).
struct OpScale {
    float alpha;
    __device__ __forceinline__ float operator()(float x) { return x * alpha + 0.0f; }
};

__device__ __forceinline__ float4 op4(OpFlatten &op, float4 v)
{
    op.m = max(op.m, absbits4(v));
    return v;
}
__device__ __forceinline__ float4 op4(OpScale &op, float4 v)
{
    return make_float4(op(v.x), op(v.y), op(v.z), op(v.w));
}

// cnt elements src[0..cnt) -> dst[0..cnt) (dst may be null when !STORE)
template <bool STORE, class OP>
__device__ __forceinline__ void seg_piece(const float *src, float *dst, uint64_t cnt, OP &op)
{
    const uint64_t tid = threadIdx.x, B = blockDim.x;
    const uintptr_t sa = reinterpret_cast<uintptr_t>(src) & 15u;
    const uintptr_t da = STORE ? (reinterpret_cast<uintptr_t>(dst) & 15u) : sa;
    uint64_t vb = cnt, ve = cnt;  // vector body [vb, ve)
    if (sa == da) {
        vb = std::min<uint64_t>(((16u - sa) & 15u) >> 2, cnt);
        ve = vb + ((cnt - vb) & ~3ull);
    }
    // vector body
    uint64_t i = vb + 4 * tid;
    for (; i + 12 * B < ve; i += 16 * B) {
        const float4 a = *reinterpret_cast<const float4 *>(src + i);
        const float4 b = *reinterpret_cast<const float4 *>(src + i + 4 * B);
        const float4 c = *reinterpret_cast<const float4 *>(src + i + 8 * B);
        const float4 d = *reinterpret_cast<const float4 *>(src + i + 12 * B);
        const float4 ra = op4(op, a), rb = op4(op, b), rc = op4(op, c), rd = op4(op, d);
        if (STORE) {
            *reinterpret_cast<float4 *>(dst + i) = ra;
            *reinterpret_cast<float4 *>(dst + i + 4 * B) = rb;
            *reinterpret_cast<float4 *>(dst + i + 8 * B) = rc;
            *reinterpret_cast<float4 *>(dst + i + 12 * B) = rd;
        }
    }
    for (; i < ve; i += 4 * B) {
        const float4 r = op4(op, *reinterpret_cast<const float4 *>(src + i));
        if (STORE)
            *reinterpret_cast<float4 *>(dst + i) = r;
    }
    // scalar head [0, vb) and tail [ve, cnt) (or everything when not co-aligned)
    for (uint64_t j = tid; j < vb; j += B) {
        const float r = op(src[j]);
        if (STORE)
            dst[j] = r;
    }
    for (uint64_t j = ve + tid; j < cnt; j += B) {
        const float r = op(src[j]);
        if (STORE)
            dst[j] = r;
    }
}

// the block's flat range [r0, r1): piece by piece (block-uniform walk)
template <bool TO_FLAT, bool STORE, class OP>
__device__ __forceinline__ void seg_range(const SegArg &sg, uint64_t r0, uint64_t r1, float *flat, OP &op)
{
    SegPos p = seg_find(sg, r0);
    for (;;) {
        const uint64_t lo = std::max(r0, p.r.start), hi = std::min(r1, p.r.end);
        float *t = p.r.ptr + (lo - p.r.start);
        float *f = STORE || !TO_FLAT ? flat + lo : nullptr;
        if (TO_FLAT)
            seg_piece<STORE>(t, f, hi - lo, op);
        else
            seg_piece<true>(f, t, hi - lo, op);
        if (hi >= r1)
            break;
        p.r = seg_rec(sg, ++p.s);
    }
}

template <bool WS, bool STORE>
__global__ __launch_bounds__(kAbsmaxThreads) void k_seg_flatten_absmax(SegArg sg, uint64_t n, float *__restrict__ flat,
                                                                       uint32_t *__restrict__ out,
                                                                       uint32_t *__restrict__ ws)
{
    OpFlatten op;
    const uint64_t ranges = (n + kRange - 1) / kRange;
    for (uint64_t c = blockIdx.x; c < ranges; c += gridDim.x) {
        const uint64_t r0 = c * kRange;
        seg_range<true, STORE>(sg, r0, std::min(r0 + kRange, n), flat, op);
    }
    absmax_finish<WS>(op.m, out, ws);
}

__global__ __launch_bounds__(kAbsmaxThreads) void k_seg_scatter(SegArg sg, uint64_t n, const float *__restrict__ flat,
                                                                float alpha)
{
    OpScale op{alpha};
    const uint64_t ranges = (n + kRange - 1) / kRange;
    for (uint64_t c = blockIdx.x; c < ranges; c += gridDim.x) {
        const uint64_t r0 = c * kRange;
        seg_range<false, true>(sg, r0, std::min(r0 + kRange, n), const_cast<float *>(flat), op);
    }
}

// src tensors -> dst tensors of the same sizes, times alpha: the GRandK setgrad
// (reducer.py:759-761: every coordinate, the selected ones overwritten after)
__global__ __launch_bounds__(kAbsmaxThreads) void k_seg_copy(SegArg src, SegArg dst, uint64_t n, float alpha)
{
    OpScale op{alpha};
    const uint64_t ranges = (n + kRange - 1) / kRange;
    for (uint64_t c = blockIdx.x; c < ranges; c += gridDim.x) {
        const uint64_t r0 = c * kRange, r1 = std::min(r0 + kRange, n);
        SegPos p = seg_find(src, r0);
        for (;;) {  // the tables share every segment boundary: record s of dst matches record s of src
            const SegRec d = seg_rec(dst, p.s);
            const uint64_t lo = std::max(r0, p.r.start), hi = std::min(r1, p.r.end);
            seg_piece<true>(p.r.ptr + (lo - p.r.start), d.ptr + (lo - d.start), hi - lo, op);
            if (hi >= r1)
                break;
            p.r = seg_rec(src, ++p.s);
        }
    }
}

int seg_arg(const gc_segments *segs, uint64_t n, SegArg *out, const char *what)
{
    GC_REQUIRE(segs, "%s: null segments", what);
    GC_REQUIRE(segs->n == n, "%s: segments hold %llu elements, bucket has %llu", what,
               (unsigned long long)segs->n, (unsigned long long)n);
    GC_REQUIRE(segs->chunk_shift >= 4 && segs->chunk_shift <= 30, "%s: chunk_shift %u outside 4..30", what,
               segs->chunk_shift);
    GC_REQUIRE(n == 0 || (segs->count > 0 && segs->seg && segs->chunk_seg), "%s: empty segment table", what);
    out->seg = reinterpret_cast<const SegRec *>(segs->seg);
    out->chunk_seg = segs->chunk_seg;
    out->count = segs->count;
    out->shift = segs->chunk_shift;
    return GC_OK;
}

}  // namespace gc

using namespace gc;

static_assert(sizeof(gc_seg) == sizeof(SegRec), "gc_seg / SegRec layout");

extern "C" {

uint32_t gc_segments_sizes_hash(const uint64_t *sizes, uint64_t count)
{
    uint32_t h = 2166136261u;
    auto mix = [&h](uint64_t v) {
        for (int i = 0; i < 8; ++i, v >>= 8) {
            h ^= (uint32_t)(v & 0xffu);
            h *= 16777619u;
        }
    };
    mix(count);
    for (uint64_t i = 0; sizes && i < count; ++i)
        mix(sizes[i]);
    return h ? h : 1u;
}

uint64_t gc_segments_chunks(uint64_t n, uint32_t chunk_shift)
{
    if (chunk_shift < 4 || chunk_shift > 30)
        return 0;
    return n == 0 ? 0 : ((n - 1) >> chunk_shift) + 1;
}

int gc_segments_plan(const uint64_t *sizes, float *const *ptrs, uint64_t count, uint32_t chunk_shift, gc_seg *seg,
                     uint32_t *chunk_seg, uint64_t chunk_capacity, uint64_t *n_out)
{
    GC_REQUIRE(chunk_shift >= 4 && chunk_shift <= 30, "gc_segments_plan: chunk_shift %u outside 4..30", chunk_shift);
    GC_REQUIRE(count == 0 || (sizes && ptrs && seg), "gc_segments_plan: null pointer");
    GC_REQUIRE(count < (1ull << 32), "gc_segments_plan: more than 2^32 tensors");
    uint64_t n = 0;
    for (uint64_t s = 0; s < count; ++s) {
        GC_REQUIRE(sizes[s] == 0 || ptrs[s], "gc_segments_plan: tensor %llu has no data pointer",
                   (unsigned long long)s);
        GC_REQUIRE(n + sizes[s] >= n, "gc_segments_plan: size overflow");
        seg[s].start = n;
        n += sizes[s];
        seg[s].end = n;
        seg[s].ptr = ptrs[s];
        seg[s].reserved = 0;
    }
    const uint64_t chunks = gc_segments_chunks(n, chunk_shift);
    GC_REQUIRE(chunks <= chunk_capacity && (chunks == 0 || chunk_seg), "gc_segments_plan: chunk table needs %llu entries",
               (unsigned long long)chunks);
    // chunk c -> the segment holding element c << shift (the first non-empty one)
    uint64_t s = 0;
    for (uint64_t c = 0; c < chunks; ++c) {
        const uint64_t e = c << chunk_shift;
        while (seg[s].end <= e)
            ++s;
        chunk_seg[c] = (uint32_t)s;
    }
    if (n_out)
        *n_out = n;
    return GC_OK;
}

int gc_segments_flatten_absmax(const gc_segments *segs, float *flat, float *norm, void *workspace, gc_stream_t stream)
{
    SegArg sg{};
    int rc;
    GC_REQUIRE(segs, "gc_segments_flatten_absmax: null segments");
    if ((rc = seg_arg(segs, segs->n, &sg, "gc_segments_flatten_absmax")))
        return rc;
    GC_REQUIRE(norm, "gc_segments_flatten_absmax: null norm");
    GC_REQUIRE(!flat || (reinterpret_cast<uintptr_t>(flat) & 3u) == 0, "gc_segments_flatten_absmax: flat misaligned");
    const uint64_t n = segs->n;
    hipStream_t st = as_stream(stream);
    uint32_t *o = reinterpret_cast<uint32_t *>(norm);
    uint32_t *ws = reinterpret_cast<uint32_t *>(workspace);
    if (n == 0 || !ws) {
        if (hipMemsetAsync(norm, 0, sizeof(float), st) != hipSuccess)
            return launch_status("gc_segments_flatten_absmax memset");
        if (n == 0)
            return GC_OK;
    }
    const unsigned grid = (unsigned)std::min<uint64_t>((n + kRange - 1) / kRange, 256);  // one per CU
#define GC_SF(WS_, ST_) \
    hipLaunchKernelGGL((k_seg_flatten_absmax<WS_, ST_>), dim3(grid), dim3(kAbsmaxThreads), 0, st, sg, n, flat, o, ws)
    if (ws) {
        if (flat) GC_SF(true, true); else GC_SF(true, false);
    } else {
        if (flat) GC_SF(false, true); else GC_SF(false, false);
    }
#undef GC_SF
    return launch_status("gc_segments_flatten_absmax");
}

int gc_segments_copy(const gc_segments *src, const gc_segments *dst, float alpha, gc_stream_t stream)
{
    SegArg a{}, b{};
    int rc;
    GC_REQUIRE(src && dst, "gc_segments_copy: null segments");
    if ((rc = seg_arg(src, src->n, &a, "gc_segments_copy")) || (rc = seg_arg(dst, src->n, &b, "gc_segments_copy")))
        return rc;
    GC_REQUIRE(src->count == dst->count, "gc_segments_copy: %llu vs %llu tensors", (unsigned long long)src->count,
               (unsigned long long)dst->count);
    GC_REQUIRE(src->sizes_hash == 0 || dst->sizes_hash == 0 || src->sizes_hash == dst->sizes_hash,
               "gc_segments_copy: the two tensor lists have different sizes (hash %08x vs %08x)", src->sizes_hash,
               dst->sizes_hash);
    const uint64_t n = src->n;
    if (n == 0)
        return GC_OK;
    const unsigned grid = (unsigned)std::min<uint64_t>((n + kRange - 1) / kRange, 2048);
    hipLaunchKernelGGL(k_seg_copy, dim3(grid), dim3(kAbsmaxThreads), 0, as_stream(stream), a, b, n, alpha);
    return launch_status("gc_segments_copy");
}

int gc_segments_scatter(const float *flat, float alpha, const gc_segments *segs, gc_stream_t stream)
{
    SegArg sg{};
    int rc;
    GC_REQUIRE(segs, "gc_segments_scatter: null segments");
    if ((rc = seg_arg(segs, segs->n, &sg, "gc_segments_scatter")))
        return rc;
    const uint64_t n = segs->n;
    if (n == 0)
        return GC_OK;
    GC_REQUIRE(flat && (reinterpret_cast<uintptr_t>(flat) & 3u) == 0, "gc_segments_scatter: null or misaligned flat");
    const unsigned grid = (unsigned)std::min<uint64_t>((n + kRange - 1) / kRange, 2048);
    hipLaunchKernelGGL(k_seg_scatter, dim3(grid), dim3(kAbsmaxThreads), 0, as_stream(stream), sg, n, flat, alpha);
    return launch_status("gc_segments_scatter");
}

}  // extern "C"
