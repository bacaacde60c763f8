// qsgd.hip — QSGD-MaxNorm hot path on gfx950:
//   k_absmax        max-norm scan            (reducer.py:516 buffer.abs().max())
//   k_qsgd_encode   quantize + stochastic round + carry-free lane pack
//                   (compressors.py:299-316 fused with the packing step)
//   k_qsgd_decode   unpack W-summed lanes + dequantize + 1/W
//                   (compressors.py:318-321, reducer.py:544-549)
//   k_qsgd_quantize / k_qsgd_dequantize   unpacked int8/int32 drop-ins
//   k_lane_pack4 / k_lane_unpack          packing of already-quantized ints
//
// Memory-bound streaming kernels.  Planar lane layout: word j of the packed
// stream holds elements j + k*M (k < L), so a thread that owns words
// 4t..4t+3 reads L fully coalesced float4s (one per plane) and writes one
// uint4: 16 B/lane on every HBM access, no LDS and no cross-lane shuffles.
// The element group i0..i0+3 of each float4 is also one Philox block.
#include "gc_device.h"
#include "gc_host.h"
#include "qsgd_encode.h"
#include "absmax.h"
#include "segments.h"

#include <algorithm>

namespace gc {

// max-norm: k_absmax (absmax.h).  Product grid: kAbsmaxGrid blocks of
// kAbsmaxThreads (two per CU: 32 waves x 4 float4 loads in flight = 128 KB
// per CU).  On the ResNet50 bucket: 256 / 512 / 1024 blocks 16.4 / 15.7 /
// 17.9 us, with the two-level tickets (one level, 256 blocks: 17.1 us;
// profiles/r05m_lab_ms.log)
#ifndef GC_ABSMAX_GRID
#define GC_ABSMAX_GRID 512
#endif
constexpr unsigned kAbsmaxGrid = GC_ABSMAX_GRID;
static_assert(kAbsmaxGrid <= kAbsmaxMaxBlocks, "absmax partials");
constexpr unsigned kEncodeGrid = 12288;  // blocks of the dense encode (see launch_encode)
constexpr unsigned kDecodeGrid = 16384;  // blocks of the dense decode (see qsgd_decode)


// ---------------------------------------------------------------------------
// encode: see qsgd_encode.h (lane(k) of word j = qmax + q(x[kM + j]))
// ---------------------------------------------------------------------------
template <int MODE>
__device__ __forceinline__ float4 load4(const float *__restrict__ x, const int64_t *__restrict__ idx, uint64_t i0,
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

// ---------------------------------------------------------------------------
// decode: out = RN(RN(c * (lane - W*qoff)) * alpha), c = RN(norm / s)
// ---------------------------------------------------------------------------
template <int MODE>  // 0: float4 dense, 1: scalar dense, 2: scatter through idx, 3: into the tensors of a gc_segments
__device__ __forceinline__ void store4(float *__restrict__ out, const int64_t *__restrict__ idx, uint64_t i0,
                                       uint64_t n, float4 v, const SegArg &sg)
{
    if constexpr (MODE == 3) {
        seg_store4(sg, i0, n, v);
        return;
    }
    if (MODE == 0 && i0 + 4 <= n) {
        st_nt4(out + i0, v);
        return;
    }
    if (i0 + 0 < n)
        out[MODE == 2 ? idx[i0 + 0] : i0 + 0] = v.x;
    if (i0 + 1 < n)
        out[MODE == 2 ? idx[i0 + 1] : i0 + 1] = v.y;
    if (i0 + 2 < n)
        out[MODE == 2 ? idx[i0 + 2] : i0 + 2] = v.z;
    if (i0 + 3 < n)
        out[MODE == 2 ? idx[i0 + 3] : i0 + 3] = v.w;
}

__device__ __forceinline__ float dq(uint32_t word, uint32_t sh, uint32_t mask, int32_t sub, float c, float alpha)
{
    const int32_t Q = (int32_t)((word >> sh) & mask) - sub;
    const float d = c * (float)Q;
    return d * alpha;
}

template <int L, int MODE>
__global__ __launch_bounds__(kBlock) void k_qsgd_decode(const uint32_t *__restrict__ words,
                                                        const int64_t *__restrict__ idx, uint64_t n,
                                                        const float *__restrict__ normp, float s, int32_t sub,
                                                        uint32_t w, uint64_t M, float alpha, float *__restrict__ out,
                                                        SegArg sg)
{
    const float c = *normp / s;
    const uint32_t mask = w >= 32 ? 0xffffffffu : ((1u << w) - 1u);
    const uint64_t quads = M >> 2;
    if constexpr (MODE == 2) {
        // GlobalRandK scatter: each chunk's index loads issue together with
        // the word load (gather_idx), then the stores
        constexpr int C = L < 8 ? L : 8;
        for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < quads; t += (uint64_t)gridDim.x * kBlock) {
            const uint4 wd = *reinterpret_cast<const uint4 *>(words + 4 * t);
#pragma unroll
            for (int k0 = 0; k0 < L; k0 += C) {
                int64_t id[C][4];
                gather_idx<C>(idx, n, M, 4 * t, k0, id);
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    const int k = k0 + j;
                    const uint64_t i0 = (uint64_t)k * M + 4 * t;
                    const uint32_t sh = (uint32_t)k * w;
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (k < L && i0 + e < n)
                            out[id[j][e]] = dq(pick(wd, e), sh, mask, sub, c, alpha);
                }
            }
        }
        return;
    }
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < quads; t += (uint64_t)gridDim.x * kBlock) {
        const uint4 wd = *reinterpret_cast<const uint4 *>(words + 4 * t);
#pragma unroll
        for (int k = 0; k < L; ++k) {
            const uint64_t i0 = (uint64_t)k * M + 4 * t;
            if (i0 < n) {
                const uint32_t sh = (uint32_t)k * w;
                float4 o;
                o.x = dq(wd.x, sh, mask, sub, c, alpha);
                o.y = dq(wd.y, sh, mask, sub, c, alpha);
                o.z = dq(wd.z, sh, mask, sub, c, alpha);
                o.w = dq(wd.w, sh, mask, sub, c, alpha);
                store4<MODE>(out, idx, i0, n, o, sg);
            }
        }
    }
}

// GlobalRandK scatter for small K (reducer.py:754 buffer[idx] = dec):
// out[idx[i]] = RN(RN(c * (lane_i - W*s)) * alpha), one element per thread
// SEG: out is the per-parameter tensor list (a gc_segments table): the scatter
// lands in grad_out directly (reducer.py:754 + 759-761 without the flat bucket)
template <bool SEG = false>
__global__ __launch_bounds__(kBlock) void k_decode_scatter1(const uint32_t *__restrict__ words,
                                                           const int64_t *__restrict__ idx, uint32_t n,
                                                           const float *__restrict__ normp, float s, int32_t sub,
                                                           uint32_t w, uint32_t M, float alpha, float *__restrict__ out,
                                                           SegArg sg = SegArg{})
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t plane = i / M, pos = i - plane * M;
    const uint32_t wd = words[pos];
    const int64_t id = idx[i];
    const float c = *normp / s;
    const uint32_t mask = (1u << w) - 1u;
    const int32_t Q = (int32_t)((wd >> (plane * w)) & mask) - sub;
    const float d = c * (float)Q;
    if constexpr (SEG) {  // the setgrad's 0 + RN(alpha * d) (reducer.py:757-761): -0 becomes +0
        const SegPos p = seg_find(sg, (uint64_t)id);
        p.r.ptr[(uint64_t)id - p.r.start] = d * alpha + 0.0f;
    } else {
        out[id] = d * alpha;
    }
}

// ---------------------------------------------------------------------------
// unpacked quantize / dequantize (the literal compress()/decompress() drop-in)
// ---------------------------------------------------------------------------
// SPLIT (the QSGDBP call site, compressors.py:344-353): q = xi (>= 0) and
// sgn = 1 iff x < 0 as two int32 arrays, the greedy packer's two inputs.
// vst: the outputs take one vector store per 4 elements (q, sgn 16-byte /
// int8 q and le 4-byte aligned; host-checked) — per-element stores of 4
// scattered lanes made the split 1.9x slower than its bytes (88 us at the
// ResNet50 size)
template <int KIND, int MODE, typename QT, bool SPLIT = false>
__global__ __launch_bounds__(kBlock) void k_qsgd_quantize(const float *__restrict__ x, uint64_t n,
                                                          const float *__restrict__ normp, float s, uint32_t level,
                                                          RngArgs rng, QT *__restrict__ q, int8_t *__restrict__ le,
                                                          int32_t le_max, uint32_t vst,
                                                          int32_t *__restrict__ sgn = nullptr)
{
    const float norm = *normp;
    const uint64_t groups = (n + 3) >> 2;
    for (uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x; g < groups; g += (uint64_t)gridDim.x * kBlock) {
        const uint64_t i0 = g << 2;
        const float4 v = load4<MODE>(x, nullptr, i0, n);
        const uint4 r = draws4<KIND>(rng, level, i0);
        if (vst && i0 + 4 <= n) {
            int32_t a[4], b[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const QElem qe = q_elem(pickf(v, e), norm, s, pick(r, e));
                a[e] = SPLIT ? qe.xi : qe.sg * qe.xi;
                b[e] = SPLIT ? (pickf(v, e) < 0.0f ? 1 : 0) : (qe.xi <= le_max ? 1 : 0);
            }
            if constexpr (sizeof(QT) == 4) {
                *reinterpret_cast<int4 *>(q + i0) = make_int4(a[0], a[1], a[2], a[3]);
            } else {
                *reinterpret_cast<uint32_t *>(q + i0) = (uint32_t)(a[0] & 0xff) | (uint32_t)(a[1] & 0xff) << 8 |
                                                        (uint32_t)(a[2] & 0xff) << 16 | (uint32_t)a[3] << 24;
            }
            if constexpr (SPLIT) {
                *reinterpret_cast<int4 *>(sgn + i0) = make_int4(b[0], b[1], b[2], b[3]);
            } else {
                if (le)
                    *reinterpret_cast<uint32_t *>(le + i0) =
                        (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24;
            }
            continue;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (i0 + e < n) {
                const QElem qe = q_elem(pickf(v, e), norm, s, pick(r, e));
                if constexpr (SPLIT) {
                    q[i0 + e] = (QT)qe.xi;
                    sgn[i0 + e] = pickf(v, e) < 0.0f ? 1 : 0;
                    continue;
                }
                q[i0 + e] = (QT)(qe.sg * qe.xi);
                if (le)
                    le[i0 + e] = (int8_t)(qe.xi <= le_max ? 1 : 0);
            }
        }
    }
}

template <typename QT>
__global__ __launch_bounds__(kBlock) void k_qsgd_dequantize(const QT *__restrict__ q, uint64_t n,
                                                            const float *__restrict__ normp, float s, float alpha,
                                                            float *__restrict__ out)
{
    const float c = *normp / s;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        const float d = c * (float)(int32_t)q[i];
        out[i] = d * alpha;
    }
}

// ---------------------------------------------------------------------------
// lane pack / unpack of integer arrays
// ---------------------------------------------------------------------------
// four consecutive words per thread: one 4-byte (int8) / 16-byte (int32) load
// per plane (plane starts are 4-word aligned, check_lanes)
template <typename QT, bool VEC>
__device__ __forceinline__ int4 load_q4(const QT *__restrict__ q, uint64_t i, uint64_t n)
{
    if (VEC && i + 3 < n) {
        if constexpr (sizeof(QT) == 1) {
            const uint32_t u = *reinterpret_cast<const uint32_t *>(q + i);
            return make_int4((int8_t)u, (int8_t)(u >> 8), (int8_t)(u >> 16), (int8_t)(u >> 24));
        } else {
            return *reinterpret_cast<const int4 *>(q + i);
        }
    }
    return make_int4(i < n ? (int32_t)q[i] : 0, i + 1 < n ? (int32_t)q[i + 1] : 0, i + 2 < n ? (int32_t)q[i + 2] : 0,
                     i + 3 < n ? (int32_t)q[i + 3] : 0);
}

// VEC: q aligned to the vector load (4 B int8, 16 B int32); else scalar loads
template <int L, typename QT, bool VEC>
__global__ __launch_bounds__(kBlock) void k_lane_pack4(const QT *__restrict__ q, uint64_t n, int32_t off, uint32_t w,
                                                       uint64_t M, uint32_t *__restrict__ words)
{
    const uint64_t quads = M >> 2;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < quads; t += (uint64_t)gridDim.x * kBlock) {
        uint4 acc = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int k = 0; k < L; ++k) {
            const uint64_t i = (uint64_t)k * M + 4 * t;
            if (i >= n)
                break;
            const int4 v = load_q4<QT, VEC>(q, i, n);
            const uint32_t sh = (uint32_t)k * w;
            acc.x |= (uint32_t)(v.x + off) << sh;
            acc.y |= i + 1 < n ? (uint32_t)(v.y + off) << sh : 0u;
            acc.z |= i + 2 < n ? (uint32_t)(v.z + off) << sh : 0u;
            acc.w |= i + 3 < n ? (uint32_t)(v.w + off) << sh : 0u;
        }
        *reinterpret_cast<uint4 *>(words + 4 * t) = acc;
    }
}

// int8 q with 16-word-aligned planes (M % 16 == 0, every big bucket): a block
// owns 4096 consecutive words, thread t words 16t .. 16t+15 of them: one
// 16-byte nontemporal load per plane, then the words go through LDS so that
// every store instruction writes 1 KB of consecutive words per wave
template <int L>
__global__ __launch_bounds__(kBlock) void k_lane_pack16(const int8_t *__restrict__ q, uint64_t n, int32_t off,
                                                        uint32_t w, uint64_t M, uint32_t *__restrict__ words)
{
    typedef uint32_t u4v __attribute__((ext_vector_type(4)));
    __shared__ u4v stage[kBlock * 4];
    const uint64_t groups = M >> 4;
    for (uint64_t g0 = (uint64_t)blockIdx.x * kBlock; g0 < groups; g0 += (uint64_t)gridDim.x * kBlock) {
        const uint64_t t = g0 + threadIdx.x;
        if (t < groups) {
            uint32_t acc[16] = {};
#pragma unroll
            for (int k = 0; k < L; ++k) {
                const uint64_t i = (uint64_t)k * M + 16 * t;
                if (i >= n)
                    break;
                const uint32_t sh = (uint32_t)k * w;
                if (i + 15 < n) {
                    const u4v u = __builtin_nontemporal_load(reinterpret_cast<const u4v *>(q + i));
                    const uint32_t v4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                    for (int j = 0; j < 16; ++j)
                        acc[j] |= (uint32_t)((int32_t)(int8_t)(v4[j >> 2] >> (8 * (j & 3))) + off) << sh;
                } else {
                    for (int j = 0; j < 16; ++j)
                        if (i + j < n)
                            acc[j] |= (uint32_t)((int32_t)q[i + j] + off) << sh;
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {  // quad j of thread t at slot 4t + j, rotated by t against bank conflicts
                const u4v r = {acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3]};
                stage[4 * threadIdx.x + ((j + threadIdx.x) & 3)] = r;
            }
        }
        __syncthreads();
        const uint64_t quads = min((uint64_t)kBlock, groups - g0) * 4;  // word quads of this block chunk
        u4v *o = reinterpret_cast<u4v *>(words + 16 * g0);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t s = j * kBlock + threadIdx.x;  // quad s = 4 * owner + its j'
            if (s < quads)
                __builtin_nontemporal_store(stage[4 * (s >> 2) + (((s & 3) + (s >> 2)) & 3)], o + s);
        }
        __syncthreads();
    }
}

template <int L>
__global__ __launch_bounds__(kBlock) void k_lane_unpack(const uint32_t *__restrict__ words, uint64_t n, int32_t sub,
                                                        uint32_t w, uint64_t M, int32_t *__restrict__ q)
{
    const uint32_t mask = w >= 32 ? 0xffffffffu : ((1u << w) - 1u);
    for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < M; j += (uint64_t)gridDim.x * kBlock) {
        const uint32_t wd = words[j];
#pragma unroll
        for (int k = 0; k < L; ++k) {
            const uint64_t i = (uint64_t)k * M + j;
            if (i < n)
                q[i] = (int32_t)((wd >> ((uint32_t)k * w)) & mask) - sub;
        }
    }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
static RngArgs rng_args(const gc_rng *r, uint64_t n)
{
    RngArgs a;
    a.seed = r->seed;
    a.offset = r->offset;
    a.stream = r->stream;
    a.n = n;
    return a;
}

static int check_rng(const gc_rng *r, const char *what, bool stream24 = false)
{
    GC_REQUIRE(r, "%s: null rng", what);
    const bool single = r->kind == GC_RNG_STREAM24 || r->kind == GC_RNG_SPLIT8 || r->kind == GC_RNG_SPLIT16;
    GC_REQUIRE(r->kind == GC_RNG_PHILOX || r->kind == GC_RNG_STREAM || (stream24 && single),
               "%s: unknown rng kind %u", what, r->kind);
    GC_REQUIRE(r->kind == GC_RNG_PHILOX || r->stream, "%s: STREAM rng without a stream pointer", what);
    GC_REQUIRE(r->kind != GC_RNG_STREAM24 || ((uintptr_t)r->stream & 3u) == 0,
               "%s: STREAM24 draws must be 4-byte aligned", what);
    GC_REQUIRE((r->kind != GC_RNG_SPLIT8 && r->kind != GC_RNG_SPLIT16) || ((uintptr_t)r->stream & 15u) == 0,
               "%s: split-plane draws must be 16-byte aligned", what);
    return GC_OK;
}

#define GC_DISPATCH_L(L, ...)                                                    \
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

template <int L, int KIND, int MODE>
static void launch_encode(const float *x, const int64_t *idx, uint64_t n, const float *norm, float s, int32_t qmax,
                          const gc_lanes *ln, RngArgs ra, uint32_t *words, hipStream_t st)
{
    // Product variant (tools/lab2, profiles/r01m_*, r01n_*): integer stochastic
    // rounding on full tiles, nontemporal loads of x (read once per pass) and
    // nontemporal stores of the words (-5 us per absmax+encode step); a grid of
    // up to 12288 blocks (48 per CU, ~1.4 tiles per thread at 1e8 floats)
    // keeps more of the 6 plane streams in flight than a 2048-block grid-stride.
    const uint64_t quads = ln->plane_words >> 2;
    if constexpr ((KIND == 4 || KIND == 5) && MODE == 0 && L <= 16)  // split-plane draws, dense x (16-byte aligned)
        hipLaunchKernelGGL((k_qsgd_encode_split<L, KIND>), dim3(grid_for(quads, kEncodeGrid)), dim3(kBlock), 0, st,
                           x, n, norm, s, qmax, ln->bits, ln->plane_words, ra, words);
    else
        hipLaunchKernelGGL((k_qsgd_encode<L, KIND, MODE>), dim3(grid_for(quads, kEncodeGrid)), dim3(kBlock), 0, st,
                           x, idx, n, norm, s, qmax, ln->bits, ln->plane_words, ra, words);
}

}  // namespace gc

using namespace gc;

extern "C" {

size_t gc_absmax_workspace_size(void) { return 4 * kAbsmaxWsWords; }

int gc_absmax_f32(const float *x, const int64_t *idx, uint64_t n, float *norm, void *workspace, gc_stream_t stream)
{
    GC_REQUIRE(norm, "gc_absmax_f32: null norm");
    GC_REQUIRE(n == 0 || x, "gc_absmax_f32: null x");
    hipStream_t st = as_stream(stream);
    uint32_t *o = reinterpret_cast<uint32_t *>(norm);
    uint32_t *ws = reinterpret_cast<uint32_t *>(workspace);
    if (n == 0 || !ws) {
        if (hipMemsetAsync(norm, 0, sizeof(float), st) != hipSuccess)
            return launch_status("gc_absmax_f32 memset");
        if (n == 0)
            return GC_OK;
    }
    const int mode = idx ? 2 : (aligned16(x) ? 0 : 1);
    const uint64_t items = mode == 0 ? (n >> 2) : n;
    const unsigned grid = (unsigned)std::min<uint64_t>(std::max<uint64_t>((items + kAbsmaxThreads - 1) / kAbsmaxThreads, 1),
                                                       kAbsmaxGrid);
    // dense reads are nontemporal (x is streamed once per pass: 61 vs 67 us at
    // 1e8 floats, profiles/r01m_lab2_*.log)
#define GC_AM(MODE_, WS_) \
    hipLaunchKernelGGL((k_absmax<MODE_, WS_, kAbsmaxThreads, 4, MODE_ == 0>), dim3(grid), dim3(kAbsmaxThreads), 0, st, \
                       x, idx, n, o, ws)
    if (ws) {
        if (mode == 0) GC_AM(0, true); else if (mode == 1) GC_AM(1, true); else GC_AM(2, true);
    } else {
        if (mode == 0) GC_AM(0, false); else if (mode == 1) GC_AM(1, false); else GC_AM(2, false);
    }
#undef GC_AM
    return launch_status("gc_absmax_f32");
}

int gc_qsgd_encode(const float *x, const int64_t *idx, uint64_t n, const float *norm, uint32_t bits,
                   const gc_lanes *lanes, const gc_rng *rng, uint32_t *words, gc_stream_t stream)
{
    int rc;
    if ((rc = check_bits(bits, "gc_qsgd_encode")) || (rc = check_lanes(lanes, n, "gc_qsgd_encode")) ||
        (rc = check_rng(rng, "gc_qsgd_encode", true)))
        return rc;
    const uint32_t s = (1u << bits) - 1u;
    GC_REQUIRE(lanes->offset == s && lanes->range == 2ull * s, "gc_qsgd_encode: lanes not made by gc_qsgd_layout");
    GC_REQUIRE(norm && words, "gc_qsgd_encode: null norm/words");
    GC_REQUIRE(n == 0 || x, "gc_qsgd_encode: null x");
    GC_REQUIRE(aligned16(words), "gc_qsgd_encode: words must be 16-byte aligned");
    if (lanes->plane_words == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const RngArgs ra = rng_args(rng, n);
    const int mode = idx ? 2 : (aligned16(x) ? 0 : 1);
    const float sf = (float)s;
    const int32_t qmax = (int32_t)s;
    if (rng->kind == GC_RNG_SPLIT8 || rng->kind == GC_RNG_SPLIT16) {
        const bool h8 = rng->kind == GC_RNG_SPLIT8;
        if (mode == 0) {
            if (h8)
                GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 4, 0>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)))
            else
                GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 5, 0>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)))
        } else if (mode == 1) {
            if (h8)
                GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 4, 1>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)))
            else
                GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 5, 1>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)))
        } else {
            if (h8)
                GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 4, 2>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)))
            else
                GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 5, 2>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)))
        }
    } else if (rng->kind == GC_RNG_STREAM24) {
        if (mode == 0) {
            GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 3, 0>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)));
        } else if (mode == 1) {
            GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 3, 1>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)));
        } else {
            GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 3, 2>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)));
        }
    } else if (rng->kind == GC_RNG_PHILOX) {
        if (mode == 0) {
            GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 0, 0>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)));
        } else if (mode == 1) {
            GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 0, 1>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)));
        } else {
            GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 0, 2>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)));
        }
    } else {
        if (mode == 0) {
            GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 1, 0>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)));
        } else if (mode == 1) {
            GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 1, 1>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)));
        } else {
            GC_DISPATCH_L(lanes->per_word, (launch_encode<LL, 1, 2>(x, idx, n, norm, sf, qmax, lanes, ra, words, st)));
        }
    }
    return launch_status("gc_qsgd_encode");
}

static int qsgd_decode(const char *what, const uint32_t *words, const int64_t *idx, uint64_t n, const float *norm,
                       uint32_t bits, const gc_lanes *lanes, float alpha, float *out, const gc_segments *segs,
                       gc_stream_t stream)
{
    int rc;
    if ((rc = check_bits(bits, what)) || (rc = check_lanes(lanes, n, what)))
        return rc;
    const uint32_t s = (1u << bits) - 1u;
    GC_REQUIRE(lanes->offset == s && lanes->range == 2ull * s, "%s: lanes not made by gc_qsgd_layout", what);
    GC_REQUIRE(norm && words && (n == 0 || out || segs), "%s: null pointer", what);
    GC_REQUIRE(aligned16(words), "%s: words must be 16-byte aligned", what);
    SegArg sg{};
    if (segs && (rc = seg_arg(segs, n, &sg, what)))
        return rc;
    if (lanes->plane_words == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const int mode = segs ? 3 : idx ? 2 : (aligned16(out) ? 0 : 1);
    const int32_t sub = (int32_t)(lanes->world * s);
    // dense / per-tensor decode: one word quad per thread (16384 blocks at 1e8
    // floats) with nontemporal stores, 69 vs 92 us (profiles/r01n_lab2_nt.log)
    const unsigned grid = grid_for(lanes->plane_words >> 2, (mode == 0 || mode == 3) ? kDecodeGrid : 0);
    const float sf = (float)s;
#define GC_DEC(MODE_)                                                                                         \
    GC_DISPATCH_L(lanes->per_word, hipLaunchKernelGGL((k_qsgd_decode<LL, MODE_>), dim3(grid), dim3(kBlock), 0, \
                                                      st, words, idx, n, norm, sf, sub, lanes->bits,          \
                                                      lanes->plane_words, alpha, out, sg))
    if (mode == 0) {
        GC_DEC(0);
    } else if (mode == 1) {
        GC_DEC(1);
    } else if (mode == 2) {
        if (n < (1ull << 32) && lanes->bits < 32 && lanes->plane_words < (1ull << 32)) {
            // one element per thread: the word and the index load in one round trip
            hipLaunchKernelGGL(k_decode_scatter1<false>, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                               words, idx, (uint32_t)n, norm, sf, sub, lanes->bits, (uint32_t)lanes->plane_words,
                               alpha, out);
        } else {
            GC_DEC(2);
        }
    } else {
        GC_DEC(3);
    }
#undef GC_DEC
    return launch_status(what);
}

int gc_qsgd_decode(const uint32_t *words, const int64_t *idx, uint64_t n, const float *norm, uint32_t bits,
                   const gc_lanes *lanes, float alpha, float *out, gc_stream_t stream)
{
    return qsgd_decode("gc_qsgd_decode", words, idx, n, norm, bits, lanes, alpha, out, nullptr, stream);
}

int gc_qsgd_decode_segments(const uint32_t *words, uint64_t n, const float *norm, uint32_t bits,
                            const gc_lanes *lanes, float alpha, const gc_segments *segs, gc_stream_t stream)
{
    GC_REQUIRE(segs, "gc_qsgd_decode_segments: null segments");
    return qsgd_decode("gc_qsgd_decode_segments", words, nullptr, n, norm, bits, lanes, alpha, nullptr, segs, stream);
}

int gc_qsgd_decode_scatter_segments(const uint32_t *words, const int64_t *idx, uint64_t k, const float *norm,
                                    uint32_t bits, const gc_lanes *lanes, float alpha, const gc_segments *segs,
                                    gc_stream_t stream)
{
    const char *what = "gc_qsgd_decode_scatter_segments";
    int rc;
    if ((rc = check_bits(bits, what)) || (rc = check_lanes(lanes, k, what)))
        return rc;
    const uint32_t s = (1u << bits) - 1u;
    GC_REQUIRE(lanes->offset == s && lanes->range == 2ull * s, "%s: lanes not made by gc_qsgd_layout", what);
    GC_REQUIRE(segs && norm && words && (k == 0 || idx), "%s: null pointer", what);
    GC_REQUIRE(k < (1ull << 32) && lanes->bits < 32 && lanes->plane_words < (1ull << 32), "%s: K too large", what);
    SegArg sg{};
    if ((rc = seg_arg(segs, segs->n, &sg, what)))
        return rc;
    if (k == 0)
        return GC_OK;
    hipLaunchKernelGGL(k_decode_scatter1<true>, dim3((unsigned)((k + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       as_stream(stream), words, idx, (uint32_t)k, norm, (float)s, (int32_t)(lanes->world * s),
                       lanes->bits, (uint32_t)lanes->plane_words, alpha, nullptr, sg);
    return launch_status(what);
}

int gc_qsgd_quantize(const float *x, uint64_t n, const float *norm, uint32_t bits, const gc_rng *rng,
                     uint32_t level, void *q, uint32_t q_dtype, gc_stream_t stream)
{
    return gc_qsgd_quantize_le(x, n, norm, bits, rng, level, q, q_dtype, nullptr, 0, stream);
}

int gc_qsgd_quantize_le(const float *x, uint64_t n, const float *norm, uint32_t bits, const gc_rng *rng,
                        uint32_t level, void *q, uint32_t q_dtype, int8_t *le_mask, uint32_t le_bits,
                        gc_stream_t stream)
{
    int rc;
    if ((rc = check_bits(bits, "gc_qsgd_quantize")) || (rc = check_rng(rng, "gc_qsgd_quantize")))
        return rc;
    GC_REQUIRE(q_dtype == GC_I8 || q_dtype == GC_I32, "gc_qsgd_quantize: q_dtype must be GC_I8 or GC_I32");
    GC_REQUIRE(level < 65536, "gc_qsgd_quantize: level too large");
    GC_REQUIRE(!le_mask || (le_bits >= 1 && le_bits <= 24), "gc_qsgd_quantize: bad le_bits");
    GC_REQUIRE(n == 0 || (x && q && norm), "gc_qsgd_quantize: null pointer");
    if (n == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const RngArgs ra = rng_args(rng, n);
    const float sf = (float)((1u << bits) - 1u);
    const int32_t le_max = le_mask ? (int32_t)((1u << le_bits) - 1u) : 0;
    const unsigned grid = grid_for((n + 3) >> 2);
    const bool vec = aligned16(x);
    const uint32_t vst = (q_dtype == GC_I8 ? (reinterpret_cast<uintptr_t>(q) & 3u) == 0 : aligned16(q)) &&
                         (!le_mask || (reinterpret_cast<uintptr_t>(le_mask) & 3u) == 0);
#define GC_Q(KIND_, MODE_, QT_)                                                                                  \
    hipLaunchKernelGGL((k_qsgd_quantize<KIND_, MODE_, QT_>), dim3(grid), dim3(kBlock), 0, st, x, n, norm, sf, level, \
                       ra, reinterpret_cast<QT_ *>(q), le_mask, le_max, vst)
    if (rng->kind == GC_RNG_PHILOX) {
        if (q_dtype == GC_I8) {
            if (vec) GC_Q(0, 0, int8_t); else GC_Q(0, 1, int8_t);
        } else {
            if (vec) GC_Q(0, 0, int32_t); else GC_Q(0, 1, int32_t);
        }
    } else {
        if (q_dtype == GC_I8) {
            if (vec) GC_Q(1, 0, int8_t); else GC_Q(1, 1, int8_t);
        } else {
            if (vec) GC_Q(1, 0, int32_t); else GC_Q(1, 1, int32_t);
        }
    }
#undef GC_Q
    return launch_status("gc_qsgd_quantize");
}

int gc_qsgd_quantize_split(const float *x, uint64_t n, const float *norm, uint32_t bits, const gc_rng *rng,
                           int32_t *xi, int32_t *sign, gc_stream_t stream)
{
    int rc;
    if ((rc = check_bits(bits, "gc_qsgd_quantize_split")) || (rc = check_rng(rng, "gc_qsgd_quantize_split")))
        return rc;
    GC_REQUIRE(n == 0 || (x && xi && sign && norm), "gc_qsgd_quantize_split: null pointer");
    if (n == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const RngArgs ra = rng_args(rng, n);
    const float sf = (float)((1u << bits) - 1u);
    const unsigned grid = grid_for((n + 3) >> 2);
    const bool vec = aligned16(x);
    const uint32_t vst = aligned16(xi) && aligned16(sign);
#define GC_QS(KIND_, MODE_)                                                                                         \
    hipLaunchKernelGGL((k_qsgd_quantize<KIND_, MODE_, int32_t, true>), dim3(grid), dim3(kBlock), 0, st, x, n, norm, \
                       sf, 0u, ra, xi, nullptr, 0, vst, sign)
    if (rng->kind == GC_RNG_PHILOX) {
        if (vec) GC_QS(0, 0); else GC_QS(0, 1);
    } else {
        if (vec) GC_QS(1, 0); else GC_QS(1, 1);
    }
#undef GC_QS
    return launch_status("gc_qsgd_quantize_split");
}

int gc_qsgd_dequantize(const void *q, uint32_t q_dtype, uint64_t n, const float *norm, uint32_t bits, float alpha,
                       float *out, gc_stream_t stream)
{
    int rc;
    if ((rc = check_bits(bits, "gc_qsgd_dequantize")))
        return rc;
    GC_REQUIRE(q_dtype == GC_I8 || q_dtype == GC_I32, "gc_qsgd_dequantize: q_dtype must be GC_I8 or GC_I32");
    GC_REQUIRE(n == 0 || (q && out && norm), "gc_qsgd_dequantize: null pointer");
    if (n == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const float sf = (float)((1u << bits) - 1u);
    if (q_dtype == GC_I8)
        hipLaunchKernelGGL((k_qsgd_dequantize<int8_t>), dim3(grid_for(n)), dim3(kBlock), 0, st,
                           reinterpret_cast<const int8_t *>(q), n, norm, sf, alpha, out);
    else
        hipLaunchKernelGGL((k_qsgd_dequantize<int32_t>), dim3(grid_for(n)), dim3(kBlock), 0, st,
                           reinterpret_cast<const int32_t *>(q), n, norm, sf, alpha, out);
    return launch_status("gc_qsgd_dequantize");
}

int gc_lane_pack(const void *q, uint32_t q_dtype, const gc_lanes *lanes, uint32_t *words, gc_stream_t stream)
{
    int rc;
    GC_REQUIRE(lanes, "gc_lane_pack: null lanes");
    if ((rc = check_lanes(lanes, lanes->n, "gc_lane_pack")))
        return rc;
    GC_REQUIRE(q_dtype == GC_I8 || q_dtype == GC_I32, "gc_lane_pack: q_dtype must be GC_I8 or GC_I32");
    GC_REQUIRE(words && (lanes->n == 0 || q), "gc_lane_pack: null pointer");
    GC_REQUIRE(aligned16(words), "gc_lane_pack: words must be 16-byte aligned (word quads are stored as uint4)");
    if (lanes->plane_words == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const unsigned grid = grid_for(lanes->plane_words / 4);
    const int32_t off = (int32_t)lanes->offset;
    if (q_dtype == GC_I8 && lanes->plane_words % 16 == 0 && (reinterpret_cast<uintptr_t>(q) & 15u) == 0 &&
        (reinterpret_cast<uintptr_t>(words) & 15u) == 0) {
        GC_DISPATCH_L(lanes->per_word,
                      hipLaunchKernelGGL((k_lane_pack16<LL>), dim3(grid_for(lanes->plane_words / 16)), dim3(kBlock), 0,
                                         st, reinterpret_cast<const int8_t *>(q), lanes->n, off, lanes->bits,
                                         lanes->plane_words, words));
    } else if (q_dtype == GC_I8) {
        if ((reinterpret_cast<uintptr_t>(q) & 3u) == 0)
            GC_DISPATCH_L(lanes->per_word,
                          hipLaunchKernelGGL((k_lane_pack4<LL, int8_t, true>), dim3(grid), dim3(kBlock), 0, st,
                                             reinterpret_cast<const int8_t *>(q), lanes->n, off, lanes->bits,
                                             lanes->plane_words, words))
        else
            GC_DISPATCH_L(lanes->per_word,
                          hipLaunchKernelGGL((k_lane_pack4<LL, int8_t, false>), dim3(grid), dim3(kBlock), 0, st,
                                             reinterpret_cast<const int8_t *>(q), lanes->n, off, lanes->bits,
                                             lanes->plane_words, words))
    } else {
        if ((reinterpret_cast<uintptr_t>(q) & 15u) == 0)
            GC_DISPATCH_L(lanes->per_word,
                          hipLaunchKernelGGL((k_lane_pack4<LL, int32_t, true>), dim3(grid), dim3(kBlock), 0, st,
                                             reinterpret_cast<const int32_t *>(q), lanes->n, off, lanes->bits,
                                             lanes->plane_words, words))
        else
            GC_DISPATCH_L(lanes->per_word,
                          hipLaunchKernelGGL((k_lane_pack4<LL, int32_t, false>), dim3(grid), dim3(kBlock), 0, st,
                                             reinterpret_cast<const int32_t *>(q), lanes->n, off, lanes->bits,
                                             lanes->plane_words, words))
    }
    return launch_status("gc_lane_pack");
}

int gc_lane_unpack(const uint32_t *words, const gc_lanes *lanes, int32_t *q, gc_stream_t stream)
{
    int rc;
    GC_REQUIRE(lanes, "gc_lane_unpack: null lanes");
    if ((rc = check_lanes(lanes, lanes->n, "gc_lane_unpack")))
        return rc;
    GC_REQUIRE(words && (lanes->n == 0 || q), "gc_lane_unpack: null pointer");
    if (lanes->plane_words == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    const int32_t sub = (int32_t)(lanes->world * lanes->offset);
    GC_DISPATCH_L(lanes->per_word,
                  hipLaunchKernelGGL((k_lane_unpack<LL>), dim3(grid_for(lanes->plane_words)), dim3(kBlock), 0, st,
                                     words, lanes->n, sub, lanes->bits, lanes->plane_words, q));
    return launch_status("gc_lane_unpack");
}

}  // extern "C"
