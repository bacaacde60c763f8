// randk.hip — small-K GlobalRandK on gfx950 (reducer.py:717-754 with the
// QSGD-MaxNorm codec of compressors.py:419-456; BASELINE config 4: K = 10,000
// of a 14.7M VGG16 bucket).
//
// At this size every kernel is a chain of dependent memory round trips
// (idx -> x[idx] -> reduction -> words), so the kernels are shaped for
// latency, not bandwidth:
//   k_randk_gather    one element per thread over ceil(K/1024) blocks (each
//                     CU issues ~1K random gathers instead of one CU issuing
//                     all of them); the gathered subset is stored contiguously
//                     (xk) with every block's partial max; the block that
//                     draws the last ticket reduces the partials into *norm and,
//                     when FUSED (W = 1: the MAX over one rank is the
//                     identity), quantizes + packs the whole subset itself:
//                     lanes staged in LDS, words stored planar — the gather,
//                     the max-norm and the encode in ONE launch
//   k_decode_scatter1 (qsgd.hip, gc_qsgd_decode with idx) one element per
//                     thread: its word and its index are independent loads
//                     (one round trip), then the scatter
// At W > 1 the encode runs after the MAX all-reduce on the contiguous xk
// (gc_qsgd_encode MODE 0): the subset is gathered once, not twice.
// The hand-off to the last block is absmax.h's (sc1 stores drained before the
// agent-scope ticket, sc1 loads in the last block).
#include "gc_device.h"
#include "gc_host.h"
#include "qsgd_encode.h"
#include "absmax.h"
#include "segments.h"

namespace gc {

constexpr unsigned kRkThreads = 1024;
constexpr uint64_t kRkFusedMax = 16384;  // K of the fused path: uint16 lanes in 32 KB of LDS
constexpr uint32_t kRkFusedMaxBits = 15; // lane values 0 .. 2 (2^b - 1) fit 16 bits
constexpr unsigned kRkMaxBlocks = 256;  // one-level ticket chain (~88 same-address adds per us)

// SEG: x is the reference's TensorBuffer as a gc_segments table (the gather
// reads each index's element straight from its per-parameter tensor: no
// flattened bucket; reducer.py:722-723 gathers from the flattened one)
template <bool FUSED, int KIND, bool SEG = false>
__global__ __launch_bounds__(kRkThreads) void k_randk_gather(const float *__restrict__ x, const int64_t *__restrict__ idx,
                                                            uint32_t k, float *__restrict__ xk, uint32_t *__restrict__ ws,
                                                            float *__restrict__ normp, float s, int32_t qmax, uint32_t w,
                                                            uint32_t L, uint32_t M, RngArgs rng,
                                                            uint32_t *__restrict__ words, SegArg sg = SegArg{})
{
    __shared__ uint32_t part[kRkThreads / 64];
    __shared__ int last;
    const uint32_t i = blockIdx.x * kRkThreads + threadIdx.x;
    uint32_t m = 0;
    if (i < k) {
        float v;
        if constexpr (SEG) {
            const uint64_t e = (uint64_t)idx[i];
            const SegPos p = seg_find(sg, e);
            v = p.r.ptr[e - p.r.start];
        } else {
            v = x[idx[i]];
        }
        if constexpr (FUSED)
            sc1_store(reinterpret_cast<uint32_t *>(xk) + i, __float_as_uint(v));  // read by the last block
        else
            xk[i] = v;
        m = absbits(v);
    }
    if constexpr (FUSED)  // every thread's xk store drained before the barrier that precedes the ticket
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    m = block_max<kRkThreads>(m, part);
    if (threadIdx.x == 0) {
        sc1_store(&ws[kWsPart + blockIdx.x], m);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial out before the ticket
        last = __hip_atomic_fetch_add(&ws[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last)
        return;
    const uint32_t r = block_max_sc1<kRkThreads>(&ws[kWsPart], gridDim.x, part);
    __shared__ float normsh;
    if (threadIdx.x == 0) {
        *reinterpret_cast<uint32_t *>(normp) = r;
        sc1_store(&ws[0], 0u);  // re-arm
        normsh = __uint_as_float(r);
    }
    if constexpr (FUSED) {
        __syncthreads();
        // ---- W = 1: quantize + stochastic round the subset, pack planar words
        __shared__ uint16_t lane[kRkFusedMax];
        const float norm = normsh;
        const DivNorm dv = make_div(norm);
        const uint32_t quads = (k + 3) >> 2;
        for (uint32_t q = threadIdx.x; q < quads; q += kRkThreads) {
            const uint32_t i0 = q << 2;
            float4 v;
            const uint32_t *xs = reinterpret_cast<const uint32_t *>(xk);
            v.x = __uint_as_float(sc1_load(xs + i0));
            v.y = i0 + 1 < k ? __uint_as_float(sc1_load(xs + i0 + 1)) : 0.0f;
            v.z = i0 + 2 < k ? __uint_as_float(sc1_load(xs + i0 + 2)) : 0.0f;
            v.w = i0 + 3 < k ? __uint_as_float(sc1_load(xs + i0 + 3)) : 0.0f;
            const uint4 rd = draws4<KIND>(rng, 0, i0);
            Range rg;
            rg.add4(v);
            const float4 ql = (dv.fast && !rg.slow(dv)) ? quot4_fast(v, dv) : quot4_ieee(v, norm);
            lane[i0] = (uint16_t)enc_lane(v.x, ql.x, s, qmax, rd.x);
            if (i0 + 1 < k)
                lane[i0 + 1] = (uint16_t)enc_lane(v.y, ql.y, s, qmax, rd.y);
            if (i0 + 2 < k)
                lane[i0 + 2] = (uint16_t)enc_lane(v.z, ql.z, s, qmax, rd.z);
            if (i0 + 3 < k)
                lane[i0 + 3] = (uint16_t)enc_lane(v.w, ql.w, s, qmax, rd.w);
        }
        __syncthreads();
        for (uint32_t p = threadIdx.x; p < M; p += kRkThreads) {
            uint32_t acc = 0;
            for (uint32_t j = 0; j < L; ++j) {
                const uint32_t e = p + j * M;
                if (e < k)
                    acc |= (uint32_t)lane[e] << (j * w);
            }
            words[p] = acc;
        }
    }
}

}  // namespace gc

using namespace gc;

extern "C" {

size_t gc_randk_workspace_size(void) { return gc_absmax_workspace_size(); }

static int randk_gather(const char *what, const float *x, const int64_t *idx, uint64_t k, float *xk, float *norm,
                        const gc_lanes *lanes, uint32_t bits, const gc_rng *rng, uint32_t *words, void *workspace,
                        gc_stream_t stream, const gc_segments *segs = nullptr)
{
    GC_REQUIRE((x || segs) && idx && norm && workspace && (k == 0 || xk), "%s: null pointer", what);
    GC_REQUIRE(k < (1ull << 31), "%s: K too large", what);
    SegArg sg{};
    int rc;
    if (segs && (rc = seg_arg(segs, segs->n, &sg, what)))
        return rc;
    if (k == 0)
        return hipMemsetAsync(norm, 0, sizeof(float), as_stream(stream)) == hipSuccess ? GC_OK : launch_status(what);
    const unsigned blocks = (unsigned)((k + kRkThreads - 1) / kRkThreads);
    GC_REQUIRE(blocks <= kRkMaxBlocks, "%s: K = %llu above %u (use gc_absmax_f32 + gc_qsgd_encode)", what,
               (unsigned long long)k, kRkMaxBlocks * kRkThreads);
    hipStream_t st = as_stream(stream);
    uint32_t *ws = reinterpret_cast<uint32_t *>(workspace);
    RngArgs ra{};
#define GC_RKG(F_, K_, ...)                                                                                       \
    do {                                                                                                          \
        if (segs)                                                                                                 \
            hipLaunchKernelGGL((k_randk_gather<F_, K_, true>), dim3(blocks), dim3(kRkThreads), 0, st, __VA_ARGS__, sg); \
        else                                                                                                      \
            hipLaunchKernelGGL((k_randk_gather<F_, K_, false>), dim3(blocks), dim3(kRkThreads), 0, st, __VA_ARGS__, sg); \
    } while (0)
    if (!words) {
        GC_RKG(false, 0, x, idx, (uint32_t)k, xk, ws, norm, 0.0f, 0, 0u, 0u, 0u, ra, nullptr);
        return launch_status(what);
    }
    const uint32_t s = (1u << bits) - 1u;
    ra.seed = rng->seed;
    ra.offset = rng->offset;
    ra.stream = rng->stream;
    ra.n = k;
    const uint32_t M = (uint32_t)lanes->plane_words;
    if (rng->kind == GC_RNG_PHILOX)
        GC_RKG(true, 0, x, idx, (uint32_t)k, xk, ws, norm, (float)s, (int32_t)s, lanes->bits, lanes->per_word, M, ra,
               words);
    else
        GC_RKG(true, 1, x, idx, (uint32_t)k, xk, ws, norm, (float)s, (int32_t)s, lanes->bits, lanes->per_word, M, ra,
               words);
#undef GC_RKG
    return launch_status(what);
}

static int randk_encode_w1_check(const char *what, uint64_t k, uint32_t bits, const gc_lanes *lanes, const gc_rng *rng,
                                 uint32_t *words)
{
    int rc;
    if ((rc = check_bits(bits, what)) || (rc = check_lanes(lanes, k, what)))
        return rc;
    const uint32_t s = (1u << bits) - 1u;
    GC_REQUIRE(lanes->offset == s && lanes->range == 2ull * s && lanes->world == 1,
               "%s: lanes not made by gc_qsgd_layout(k, bits, 1)", what);
    GC_REQUIRE(k <= kRkFusedMax, "%s: K = %llu above %llu", what, (unsigned long long)k,
               (unsigned long long)kRkFusedMax);
    // lanes are staged as uint16 in LDS: a lane value reaches 2 s = 2^(b+1) - 2
    GC_REQUIRE(bits <= kRkFusedMaxBits, "%s: %u bits above %u (16-bit LDS lanes; use the gather + gc_qsgd_encode)",
               what, bits, kRkFusedMaxBits);
    GC_REQUIRE(rng && (rng->kind == GC_RNG_PHILOX || (rng->kind == GC_RNG_STREAM && rng->stream)), "%s: bad rng", what);
    GC_REQUIRE(words, "%s: null words", what);
    if (k == 0 && lanes->plane_words)
        return fail(GC_EINVAL, "%s: layout / K mismatch", what);
    return GC_OK;
}

int gc_randk_gather_absmax(const float *x, const int64_t *idx, uint64_t k, float *xk, float *norm, void *workspace,
                           gc_stream_t stream)
{
    return randk_gather("gc_randk_gather_absmax", x, idx, k, xk, norm, nullptr, 0, nullptr, nullptr, workspace, stream);
}

int gc_randk_encode_w1(const float *x, const int64_t *idx, uint64_t k, float *xk, float *norm, uint32_t bits,
                       const gc_lanes *lanes, const gc_rng *rng, uint32_t *words, void *workspace, gc_stream_t stream)
{
    int rc;
    if ((rc = randk_encode_w1_check("gc_randk_encode_w1", k, bits, lanes, rng, words)))
        return rc;
    if (k == 0)
        return GC_OK;
    return randk_gather("gc_randk_encode_w1", x, idx, k, xk, norm, lanes, bits, rng, words, workspace, stream);
}

int gc_randk_gather_absmax_segments(const gc_segments *segs, const int64_t *idx, uint64_t k, float *xk, float *norm,
                                    void *workspace, gc_stream_t stream)
{
    GC_REQUIRE(segs, "gc_randk_gather_absmax_segments: null segments");
    return randk_gather("gc_randk_gather_absmax_segments", nullptr, idx, k, xk, norm, nullptr, 0, nullptr, nullptr,
                        workspace, stream, segs);
}

int gc_randk_encode_w1_segments(const gc_segments *segs, const int64_t *idx, uint64_t k, float *xk, float *norm,
                                uint32_t bits, const gc_lanes *lanes, const gc_rng *rng, uint32_t *words,
                                void *workspace, gc_stream_t stream)
{
    int rc;
    GC_REQUIRE(segs, "gc_randk_encode_w1_segments: null segments");
    if ((rc = randk_encode_w1_check("gc_randk_encode_w1_segments", k, bits, lanes, rng, words)))
        return rc;
    if (k == 0)
        return GC_OK;
    return randk_gather("gc_randk_encode_w1_segments", nullptr, idx, k, xk, norm, lanes, bits, rng, words, workspace,
                        stream, segs);
}

}  // extern "C"
