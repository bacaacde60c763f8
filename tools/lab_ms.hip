// lab_ms.hip — measurement harness for the multi-scale / two-scale kernels
// (not product code).  BASELINE config 3 bucket (ResNet50, 23,520,842 fp32),
// levels [2, 4], W = 1: the product entry points, lab variants of the dense
// fast kernels (ms_fast.h VAR flags), and the memory rooflines of each
// kernel's access pattern.  Variant outputs are compared with the product's.
// Build: make -C tools lab_ms ; run: tools/lab_ms [n]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <vector>

#include "gcodec.h"
#include "ms_common.h"
#include "ms_fast.h"
#include "absmax.h"

using namespace gc;

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(2);                                                                        \
        }                                                                                   \
    } while (0)
#define GK(x)                                                                 \
    do {                                                                      \
        if ((x) != GC_OK) {                                                   \
            fprintf(stderr, "gcodec %s at %d: %s\n", #x, __LINE__, gc_last_error()); \
            exit(3);                                                          \
        }                                                                     \
    } while (0)

// N(0, 0.01)-like values from a counter hash (sum of 4 uniforms)
__global__ void k_fill(float *x, uint64_t n, uint32_t seed)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        float acc = 0.0f;
        for (int j = 0; j < 4; ++j) {
            uint32_t h = (uint32_t)(i * 4 + j) * 2654435761u ^ seed;
            h ^= h >> 15;
            h *= 2246822519u;
            h ^= h >> 13;
            acc += (float)(h >> 8) * 0x1p-24f - 0.5f;
        }
        x[i] = acc * 0.0173f;
    }
}

// N(0, 0.01) by Box-Muller from the same counter hash (LAB_NORMAL=1: the
// bench's torch.randn-like data, with its tails: norm ~ 5.4 sigma at 23.5 M)
__global__ void k_fill_normal(float *x, uint64_t n, uint32_t seed)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        uint32_t g = h * 3266489917u + 0x9E3779B9u;
        g ^= g >> 16;
        g *= 2246822519u;
        g ^= g >> 13;
        const float u1 = ((float)(h >> 8) + 0.5f) * 0x1p-24f, u2 = (float)(g >> 8) * 0x1p-24f;
        x[i] = 0.01f * sqrtf(-2.0f * logf(u1)) * cosf(6.2831853f * u2);
    }
}

__global__ __launch_bounds__(256) void k_read_nt(const float4 *x, uint64_t n4, uint32_t *out)
{
    uint32_t m = 0;
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < n4; t += gridDim.x * 256ull) {
        const float4 v = ld_nt(x + t);
        m = max(m, max(max(__float_as_uint(v.x), __float_as_uint(v.y)), max(__float_as_uint(v.z), __float_as_uint(v.w))));
    }
    if (m == 0x7fffffffu)
        out[0] = m;
}

__global__ __launch_bounds__(256) void k_write_nt(float4 *o, uint64_t n4)
{
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < n4; t += gridDim.x * 256ull)
        st_nt4(reinterpret_cast<float *>(o + t), make_float4((float)t, 1.0f, 2.0f, 3.0f));
}

// select-like pattern: L planes of x -> one packed word quad
template <int L>
__global__ __launch_bounds__(256) void k_rw_planar(const float *x, uint32_t M, uint32_t *words, uint32_t n)
{
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < (M >> 2); t += gridDim.x * 256u) {
        uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < L; ++k) {
            if (k * M + 4 * t + 4 > n)  // planes past the bucket (the coupled W = 1 mask layout pads to 32)
                break;
            const float4 v = ld_nt(reinterpret_cast<const float4 *>(x + k * M + 4 * t));
            acc.x ^= __float_as_uint(v.x);
            acc.y ^= __float_as_uint(v.y);
            acc.z ^= __float_as_uint(v.z);
            acc.w ^= __float_as_uint(v.w);
        }
        st_nt4u(words + 4 * t, acc);
    }
}

// decode-like pattern: one word quad -> L planes of floats
template <int L>
__global__ __launch_bounds__(256) void k_wr_planar(const uint32_t *words, uint32_t M, float *out, uint32_t n)
{
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < (M >> 2); t += gridDim.x * 256u) {
        const uint4 w = *reinterpret_cast<const uint4 *>(words + 4 * t);
#pragma unroll
        for (int k = 0; k < L; ++k)
            if (k * M + 4 * t + 4 <= n)  // padded planes end past the bucket
            st_nt4(out + k * M + 4 * t, make_float4((float)(w.x >> k), (float)(w.y >> k), (float)(w.z >> k),
                                                    (float)(w.w >> k)));
    }
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    hipStream_t st = 0;  // the stream the events are recorded on (the variants' own)
    template <class F>
    float run(F f, int reps = 20)
    {
        f();
        f();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, st));
        for (int i = 0; i < reps; ++i)
            f();
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms / reps;
    }
};

static void row(const char *name, float ms, double bytes)
{
    double gbs = bytes / (ms * 1e-3) / 1e9;
    printf("%-52s %9.1f us  %8.1f GB/s  %5.1f%% of 8 TB/s\n", name, ms * 1e3, gbs, 100.0 * gbs / 8000.0);
    fflush(stdout);
}

static unsigned grid(uint64_t quads, unsigned cap = 16384)
{
    uint64_t b = (quads + 255) / 256;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(b, cap));
}

// select from the q cache without the mask words (every element at level 1):
// the cost of the W-summed mask reads in k_ms_select_cache
__global__ __launch_bounds__(256) void k_sel_cache_nomask(const uint8_t *__restrict__ cache, uint32_t n, uint32_t Mq,
                                                          uint32_t wq, uint32_t cb, uint32_t *__restrict__ words)
{
    const uint32_t cm = (1u << cb) - 1u, quads = Mq >> 2;
    __shared__ uint4 part[3][64];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    for (uint32_t tb = blockIdx.x * 64; tb < quads; tb += gridDim.x * 64) {
        const uint32_t t = tb + lane;
        uint4 acc = make_uint4(0u, 0u, 0u, 0u);
        if (t < quads) {
            for (int j = 0; j < 3; ++j) {
                const uint32_t p = wave + 4u * j;
                if (p >= 10u)
                    break;
                const uint32_t i0 = p * Mq + 4u * t;
                if (i0 >= n)
                    break;
                const uint4 c = cache_cells<1>(cache_load<1>(cache, i0, n));
                const uint32_t sh = p * wq;
                acc.x += ((c.x >> cb) & cm) << sh;
                acc.y += ((c.y >> cb) & cm) << sh;
                acc.z += ((c.z >> cb) & cm) << sh;
                acc.w += ((c.w >> cb) & cm) << sh;
            }
        }
        if (wave)
            part[wave - 1][lane] = acc;
        __syncthreads();
        if (wave == 0 && t < quads) {
            const uint4 a = part[0][lane], b = part[1][lane], c = part[2][lane];
            words[4 * t] = acc.x + a.x + b.x + c.x;
            words[4 * t + 1] = acc.y + a.y + b.y + c.y;
            words[4 * t + 2] = acc.z + a.z + b.z + c.z;
            words[4 * t + 3] = acc.w + a.w + b.w + c.w;
        }
        __syncthreads();
    }
}

int main(int argc, char **argv)
{
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 23520842ull;
    gc_levels lv{};
    lv.count = 2;
    lv.bits[0] = 2;
    lv.bits[1] = 4;
    gc_lanes ql, ml;
    GK(gc_ms_layout(n, &lv, 1, &ql));
    GK(gc_ms_mask_layout(n, &lv, 1, &ml));
    printf("n=%llu  q lanes w=%u L=%u M=%llu  mask lanes w=%u L=%u M=%llu\n", (unsigned long long)n, ql.bits,
           ql.per_word, (unsigned long long)ql.plane_words, ml.bits, ml.per_word, (unsigned long long)ml.plane_words);
    if (ql.per_word != 10 || ml.per_word != 32) {
        fprintf(stderr, "lab expects L=10 q lanes and L=32 mask lanes\n");
        return 1;
    }
    const uint32_t Mq = (uint32_t)ql.plane_words, Mm = (uint32_t)ml.plane_words;
    float *x, *norm, *out, *out2;
    uint32_t *mw, *mw2, *wq, *wq2, *scratch;
    CK(hipMalloc(&x, n * 4 + 64));
    CK(hipMalloc(&out, n * 4 + 64));
    CK(hipMalloc(&out2, n * 4 + 64));
    CK(hipMalloc(&norm, 64));
    CK(hipMalloc(&mw, (size_t)Mm * 4 + 64));
    CK(hipMalloc(&mw2, (size_t)Mm * 4 + 64));
    CK(hipMalloc(&wq, (size_t)Mq * 4 + 64));
    CK(hipMalloc(&wq2, (size_t)Mq * 4 + 64));
    CK(hipMalloc(&scratch, 64));
    if (getenv("LAB_NORMAL"))
        hipLaunchKernelGGL(k_fill_normal, dim3(4096), dim3(256), 0, 0, x, n, 11u);
    else
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, x, n, 11u);
    GK(gc_absmax_f32(x, nullptr, n, norm, nullptr, nullptr));
    CK(hipDeviceSynchronize());

    gc_rng rng = {GC_RNG_PHILOX, 0, 5, 0, nullptr};
    auto p_mask = [&] { GK(gc_ms_mask_encode(x, nullptr, n, norm, &lv, &rng, &ml, mw, nullptr)); };
    auto p_sel = [&] { GK(gc_ms_select_encode(x, nullptr, n, norm, &lv, &rng, mw, &ml, &ql, wq, nullptr)); };
    auto p_dec = [&](int order) {
        return [&, order] {
            GK(gc_ms_decode(wq, mw, nullptr, n, norm, &lv, &ml, &ql, order, 1.0f, out, nullptr));
        };
    };

    // kernel arguments as multiscale.hip builds them
    LevelsArg la;
    la.count = lv.count;
    la.maxv = (1 << lv.bits[0]) - 1;
    MsFastArg fa;
    for (int i = 0; i < GC_MAX_LEVELS; ++i) {
        la.s[i] = i < (int)lv.count ? (float)((1u << lv.bits[i]) - 1u) : 1.0f;
        fa.S24[i] = la.s[i] * 16777216.0f;
        fa.y[i] = 1.0f / la.s[i];
    }
    fa.thr = -la.maxv * (1 << 24);
    RngArgs ra{5, 0, nullptr, n};
    MaskArg mk{mw, Mm, ml.bits, lv.count - 1, 1};
    const FastDiv fd = make_fastdiv(Mm);
    const uint32_t n32 = (uint32_t)n;
    const int32_t qmax = (int32_t)ql.offset, sub = (int32_t)ql.offset;

    auto v_mask = [&](auto kern, uint32_t *dst) {
        return [=] {
            hipLaunchKernelGGL(kern, dim3(grid(Mm / 4)), dim3(256), 0, 0, x, n32, norm, la, fa, ra, Mm, ml.bits,
                               lv.count - 1, dst, (void *)nullptr, 0, 0u);
        };
    };
    auto v_sel = [&](auto kern, uint32_t *dst) {
        return [=] {
            hipLaunchKernelGGL(kern, dim3(grid(Mq / 4)), dim3(256), 0, 0, x, n32, norm, la, fa, ra, mk, fd, Mq,
                               ql.bits, qmax, dst);
        };
    };
    auto v_mask64 = [&](auto kern, uint32_t *dst) {
        return [=] {
            hipLaunchKernelGGL(kern, dim3((Mm / 4 + 63) / 64), dim3(256), 0, 0, x, n32, norm, la, fa, ra, Mm, ml.bits,
                               lv.count - 1, dst, (void *)nullptr, 0, 0u);
        };
    };
    auto v_sel64 = [&](auto kern, uint32_t *dst) {
        return [=] {
            hipLaunchKernelGGL(kern, dim3((Mq / 4 + 63) / 64), dim3(256), 0, 0, x, n32, norm, la, fa, ra, mk, fd, Mq,
                               ql.bits, qmax, dst);
        };
    };
    auto v_dec = [&](auto kern, float *dst) {
        return [=] {
            hipLaunchKernelGGL(kern, dim3(grid(Mq / 4)), dim3(256), 0, 0, wq, mk, fd, n32, norm, la, fa, Mq, ql.bits,
                               sub, 1.0f, dst);
        };
    };

    // ---- equality of the lab variants with the product ----
    auto cmp = [&](const char *nm, const void *a, const void *b, size_t bytes) {
        std::vector<uint8_t> ha(bytes), hb(bytes);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(ha.data(), a, bytes, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hb.data(), b, bytes, hipMemcpyDeviceToHost));
        printf("%-40s == product: %s\n", nm, memcmp(ha.data(), hb.data(), bytes) == 0 ? "yes" : "NO");
    };
    // launch shapes: per-quad kernels one quad per lane, octet kernels (dense
    // two-level stream, ms_fast.h *_o2) two quads per lane, 64 lanes per tile
    auto g4 = [](uint32_t M) { return dim3((M / 4 + 63) / 64); };
    auto g8 = [](uint32_t M) { return dim3((M / 8 + 63) / 64); };
    uint32_t cby = 0;
    GK(gc_ms_cache_bytes(n, &lv, &cby));
    uint8_t *cache, *cache2;
    CK(hipMalloc(&cache, n * cby + 64));
    CK(hipMalloc(&cache2, n * cby + 64));
    const double cbytes = (double)n * cby;
    auto p_maskc = [&] { GK(gc_ms_mask_encode_cached(x, n, norm, &lv, &rng, &ml, mw2, cache, nullptr)); };
    auto p_selc = [&] { GK(gc_ms_select_cached(cache, n, &lv, mw, &ml, &ql, wq2, nullptr)); };
    auto mask4 = [&](auto kern, uint32_t *dst, void *cdst) {
        return [=] {
            hipLaunchKernelGGL(kern, g4(Mm), dim3(256), 0, 0, x, n32, norm, la, fa, ra, Mm, ml.bits, lv.count - 1, dst,
                               cdst, qmax, 3u);
        };
    };
    auto mask8 = [&](auto kern, uint32_t *dst, void *cdst) {
        return [=] {
            hipLaunchKernelGGL(kern, g8(Mm), dim3(256), 0, 0, x, n32, norm, la, fa, ra, Mm, ml.bits, dst, cdst, qmax,
                               3u);
        };
    };
    auto sel = [&](auto kern, dim3 g, uint32_t *dst) {
        return [=] {
            hipLaunchKernelGGL(kern, g, dim3(256), 0, 0, x, n32, norm, la, fa, ra, mk, fd, Mq, ql.bits, qmax, dst);
        };
    };
    const uint32_t rr = 32u / ql.per_word;
    uint32_t *mw3, *wq3;
    CK(hipMalloc(&mw3, (size_t)Mm * 4 + 64));
    CK(hipMalloc(&wq3, (size_t)Mq * 4 + 64));
    uint32_t Cw3 = 0;
    for (uint32_t k = 0; k < ql.per_word; ++k)
        Cw3 += (uint32_t)qmax << (k * ql.bits);
    const uint32_t pend3 = (uint32_t)((n + Mm - 1) / Mm);
    auto w1 = [&](auto kern, dim3 g) {
        return [=] {
            hipLaunchKernelGGL(kern, g, dim3(64 * rr), 0, 0, x, n32, norm, la, fa, ra, Mm, rr, ql.per_word, ql.bits,
                               qmax, Cw3, pend3, mw3, wq3);
        };
    };
    auto p_w1 = [&] { GK(gc_ms_encode_w1(x, n, norm, &lv, &rng, &ml, &ql, mw3, wq3, nullptr)); };

    p_mask();
    p_sel();
    p_dec(0)();
    mask8(k_ms_mask_fast_o2<32, 0, 0>, mw2, nullptr)();
    cmp("mask octet unrolled", mw, mw2, (size_t)Mm * 4);
    mask4(k_ms_mask_fast<32, 2, 2, 0, 0>, mw2, nullptr)();
    cmp("mask per-quad dense", mw, mw2, (size_t)Mm * 4);
    sel(k_ms_select_fast_o2<10, 0>, g8(Mq), wq2)();
    cmp("select octet unrolled", wq, wq2, (size_t)Mq * 4);
    sel(k_ms_select_fast<10, 2, 2, 0>, g4(Mq), wq2)();
    cmp("select per-quad dense", wq, wq2, (size_t)Mq * 4);
    p_maskc();
    cmp("cached mask", mw, mw2, (size_t)Mm * 4);
    mask8(k_ms_mask_fast_o2<32, 0, 1>, mw2, cache2)();
    cmp("cached mask octet unrolled", mw, mw2, (size_t)Mm * 4);
    cmp("cache cells octet unrolled", cache, cache2, (size_t)n * cby);
    mask4(k_ms_mask_fast<32, 2, 2, 0, 1>, mw2, cache2)();
    cmp("cache cells per-quad dense", cache, cache2, (size_t)n * cby);
    p_selc();
    cmp("select from cache", wq, wq2, (size_t)Mq * 4);
    CK(hipMemset(out2, 0, n * 4));
    v_dec(k_ms_decode_fast<10, 0, 2, MSV_PLAINST>, out2)();
    cmp("decode plain stores", out, out2, n * 4);
    p_w1();
    cmp("one-pass mask == two-pass", mw, mw3, (size_t)Mm * 4);
    cmp("one-pass words == two-pass", wq, wq3, (size_t)Mq * 4);
    w1(k_ms_fused_w1_o2<0>, g8(Mm))();
    cmp("one-pass no-prefetch words", wq, wq3, (size_t)Mq * 4);
    w1(k_ms_fused_w1<2, 2, MSV_EAGER0, 2>, g4(Mm))();
    cmp("one-pass per-quad dense words", wq, wq3, (size_t)Mq * 4);
    // the tail forms of the cached mask (cells and mask words equal the product's)
    auto cmpmask = [&](const char *nm, auto kern) {
        CK(hipMemset(mw2, 0, (size_t)Mm * 4));
        CK(hipMemset(cache2, 0, (size_t)n * cby));
        mask8(kern, mw2, cache2)();
        char b1[96], b2[96];
        snprintf(b1, sizeof b1, "cached mask %s", nm);
        snprintf(b2, sizeof b2, "cache cells %s", nm);
        cmp(b1, mw, mw2, (size_t)Mm * 4);
        cmp(b2, cache, cache2, (size_t)n * cby);
    };
    cmpmask("ROLL", k_ms_mask_fast_o2<32, MSV_ROLL, 1>);
    cmpmask("ROLL UFLAG", k_ms_mask_fast_o2<32, MSV_ROLL | MSV_UFLAG, 1>);
    CK(hipMemset(mw2, 0, (size_t)Mm * 4));
    mask8(k_ms_mask_fast_o2<32, MSV_ROLL | MSV_UFLAG, 0>, mw2, nullptr)();
    cmp("mask ROLL UFLAG", mw, mw2, (size_t)Mm * 4);

    // ---- settled interleaved A/B ----
    Timer T;
    const double xb = 4.0 * n, mb = 4.0 * Mm, qb = 4.0 * Mq;
    float tot = 0;
    while (tot < 300.0f)
        tot += 50 * T.run([&] { p_mask(); p_sel(); p_dec(0)(); }, 50);
    struct V {
        const char *name;
        std::function<void()> f;
        double bytes;
        std::vector<float> t;
        hipStream_t st = 0;
    };
    std::vector<V> vs;
    vs.push_back({"roof: read x (NT)", [&] {
                      hipLaunchKernelGGL(k_read_nt, dim3(4096), dim3(256), 0, 0, (const float4 *)x, n / 4, scratch);
                  }, xb, {}});
    vs.push_back({"product mask encode (octet)", p_mask, xb + mb, {}});
    vs.push_back({"mask octet unrolled", mask8(k_ms_mask_fast_o2<32, 0, 0>, mw2, nullptr), xb + mb, {}});
    vs.push_back({"mask per-quad dense", mask4(k_ms_mask_fast<32, 2, 2, 0, 0>, mw2, nullptr), xb + mb, {}});
    vs.push_back({"mask per-quad KIND0 (r03)", mask4(k_ms_mask_fast<32, 0, 2, 0, 0>, mw2, nullptr), xb + mb, {}});
    vs.push_back({"product select encode (octet)", p_sel, xb + mb + qb, {}});
    vs.push_back({"select octet unrolled", sel(k_ms_select_fast_o2<10, 0>, g8(Mq), wq2), xb + mb + qb, {}});
    vs.push_back({"select per-quad dense", sel(k_ms_select_fast<10, 2, 2, 0>, g4(Mq), wq2), xb + mb + qb, {}});
    vs.push_back({"select per-quad KIND0 (r03)", sel(k_ms_select_fast<10, 0, 2, 0>, g4(Mq), wq2), xb + mb + qb, {}});
    vs.push_back({"product mask + cache (octet)", p_maskc, xb + mb + cbytes, {}});
    vs.push_back({"mask + cache octet unrolled", mask8(k_ms_mask_fast_o2<32, 0, 1>, mw2, cache2), xb + mb + cbytes, {}});
    vs.push_back({"mask + cache per-quad dense", mask4(k_ms_mask_fast<32, 2, 2, 0, 1>, mw2, cache2), xb + mb + cbytes, {}});
    vs.push_back({"mask + cache per-quad KIND0 (r03)", mask4(k_ms_mask_fast<32, 0, 2, 0, 1>, mw2, cache2), xb + mb + cbytes, {}});
    vs.push_back({"product select from cache", p_selc, cbytes + mb + qb, {}});
    vs.push_back({"product one-pass W=1 (octet)", p_w1, xb + mb + qb, {}});
    // the product's octet configurations compiled into the lab (GC_MS_WPE builds pin their occupancy)
    vs.push_back({"lab one-pass octet PREFETCH", w1(k_ms_fused_w1_o2<MSV_PREFETCH>, g8(Mm)), xb + mb + qb, {}});
    vs.push_back({"lab mask + cache octet ROLL", mask8(k_ms_mask_fast_o2<32, MSV_ROLL, 1>, mw2, cache2),
                  xb + mb + cbytes, {}});
    vs.push_back({"lab select octet ROLL", sel(k_ms_select_fast_o2<10, MSV_ROLL>, g8(Mq), wq2), xb + mb + qb, {}});
    vs.push_back({"lab mask + cache octet ROLL UFLAG",
                  mask8(k_ms_mask_fast_o2<32, MSV_ROLL | MSV_UFLAG, 1>, mw2, cache2), xb + mb + cbytes, {}});
    vs.push_back({"lab mask octet ROLL", mask8(k_ms_mask_fast_o2<32, MSV_ROLL, 0>, mw2, nullptr), xb + mb, {}});
    vs.push_back({"lab mask octet ROLL UFLAG", mask8(k_ms_mask_fast_o2<32, MSV_ROLL | MSV_UFLAG, 0>, mw2, nullptr),
                  xb + mb, {}});
    vs.push_back({"one-pass octet no prefetch", w1(k_ms_fused_w1_o2<0>, g8(Mm)), xb + mb + qb, {}});
    vs.push_back({"one-pass per-quad dense EAGER0 U2", w1(k_ms_fused_w1<2, 2, MSV_EAGER0, 2>, g4(Mm)), xb + mb + qb, {}});
    vs.push_back({"one-pass per-quad KIND0 EAGER0 U2 (r03)", w1(k_ms_fused_w1<0, 2, MSV_EAGER0, 2>, g4(Mm)), xb + mb + qb, {}});
    vs.push_back({"product decode order 0", p_dec(0), xb + mb + qb, {}});
    vs.push_back({"roof: write 4n (NT float4)", [&] {
                      hipLaunchKernelGGL(k_write_nt, dim3(4096), dim3(256), 0, 0, (float4 *)out2, n / 4);
                  }, xb, {}});
    vs.push_back({"product absmax (memset + atomicMax)", [&] { gc_absmax_f32(x, nullptr, n, norm, nullptr, nullptr); },
                  xb, {}});
    void *aws;
    CK(hipMalloc(&aws, gc_absmax_workspace_size()));
    CK(hipMemset(aws, 0, gc_absmax_workspace_size()));
    vs.push_back({"product absmax (workspace: tickets)", [&] { gc_absmax_f32(x, nullptr, n, norm, aws, nullptr); }, xb,
                  {}});
    // the ticket chain A/B: one group ticket (all blocks) against 16 (one per XCD pair)
    const unsigned agrid = (unsigned)std::min<uint64_t>((n / 4 + kAbsmaxThreads - 1) / kAbsmaxThreads, 256);
    vs.push_back({"lab absmax, 1 ticket group", [&] {
                      hipLaunchKernelGGL((k_absmax<0, true, kAbsmaxThreads, 4, true, 1>), dim3(agrid),
                                         dim3(kAbsmaxThreads), 0, 0, x, nullptr, n, (uint32_t *)norm, (uint32_t *)aws);
                  }, xb, {}});
    for (unsigned gm : {1u, 2u, 4u}) {  // 256 / 512 / 1024 blocks of 1024 threads
        static char nm[3][64];
        const int ix = gm == 1 ? 0 : (gm == 2 ? 1 : 2);
        snprintf(nm[ix], 64, "lab absmax, 16 ticket groups, %u blocks", agrid * gm);
        const unsigned gg = std::min<unsigned>(agrid * gm, kAbsmaxMaxBlocks);
        vs.push_back({nm[ix], [&, gg] {
                          hipLaunchKernelGGL((k_absmax<0, true, kAbsmaxThreads, 4, true, 16>), dim3(gg),
                                             dim3(kAbsmaxThreads), 0, 0, x, nullptr, n, (uint32_t *)norm,
                                             (uint32_t *)aws);
                      }, xb, {}});
    }
    // whole steps in sequence (the bucket fits the Infinity Cache, so a kernel's own loop is optimistic):
    // the decode's store policy decides how much dirty data the next step's absmax waits for
    vs.push_back({"seq: absmax + one-pass + decode NT (product)", [&] {
                      gc_absmax_f32(x, nullptr, n, norm, aws, nullptr);
                      p_w1();
                      p_dec(0)();
                  }, xb * 3 + mb * 2 + qb * 2, {}});
    // the decode reading what the one-pass kernel just wrote (NT or plain stores)
    auto dec3 = [&] { GK(gc_ms_decode(wq3, mw3, nullptr, n, norm, &lv, &ml, &ql, 1, 1.0f, out, nullptr)); };
    vs.push_back({"seq: one-pass + decode of its own words (NT stores)", [&] {
                      p_w1();
                      dec3();
                  }, 0, {}});
    vs.push_back({"seq: one-pass plain stores + decode of its own words", [&] {
                      w1(k_ms_fused_w1_o2<MSV_PREFETCH | MSV_PLAINST>, g8(Mm))();
                      dec3();
                  }, 0, {}});
    auto decv = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(grid(Mq / 4)), dim3(256), 0, 0, wq3, MaskArg{mw3, Mm, ml.bits, lv.count - 1, 1},
                           fd, n32, norm, la, fa, Mq, ql.bits, sub, 1.0f, out);
    };
    vs.push_back({"seq: one-pass + decode (lab launch) of its own words", [&] {
                      p_w1();
                      decv(k_ms_decode_fast<10, 1, 2, 0>);
                  }, 0, {}});
    vs.push_back({"seq: one-pass + decode PERTHREAD (words loaded once per lane)", [&] {
                      p_w1();
                      hipLaunchKernelGGL((k_ms_decode_fast<10, 1, 2, MSV_PERTHREAD>), dim3((Mq / 4 + 255) / 256),
                                         dim3(256), 0, 0, wq3, MaskArg{mw3, Mm, ml.bits, lv.count - 1, 1}, fd, n32,
                                         norm, la, fa, Mq, ql.bits, sub, 1.0f, out);
                  }, 0, {}});
    auto decpt = [&](const uint32_t *wsrc, const uint32_t *msrc) {
        hipLaunchKernelGGL((k_ms_decode_fast<10, 1, 2, MSV_PERTHREAD>), dim3((Mq / 4 + 255) / 256), dim3(256), 0, 0,
                           wsrc, MaskArg{msrc, Mm, ml.bits, lv.count - 1, 1}, fd, n32, norm, la, fa, Mq, ql.bits, sub,
                           1.0f, out);
    };
    vs.push_back({"STEP: absmax + one-pass + decode (product)", [&] {
                      gc_absmax_f32(x, nullptr, n, norm, aws, nullptr);
                      p_w1();
                      dec3();
                  }, 0, {}});
    vs.push_back({"STEP: absmax + one-pass + decode PERTHREAD", [&] {
                      gc_absmax_f32(x, nullptr, n, norm, aws, nullptr);
                      p_w1();
                      decpt(wq3, mw3);
                  }, 0, {}});
    vs.push_back({"STEP: absmax + one-pass plain stores + decode PERTHREAD", [&] {
                      gc_absmax_f32(x, nullptr, n, norm, aws, nullptr);
                      w1(k_ms_fused_w1_o2<MSV_PREFETCH | MSV_PLAINST>, g8(Mm))();
                      decpt(wq3, mw3);
                  }, 0, {}});
    vs.push_back({"one-pass plain stores alone", w1(k_ms_fused_w1_o2<MSV_PREFETCH | MSV_PLAINST>, g8(Mm)), 0, {}});
    vs.push_back({"STEP q-cache: absmax + mask/cache + select + decode (product)", [&] {
                      gc_absmax_f32(x, nullptr, n, norm, aws, nullptr);
                      GK(gc_ms_mask_encode_cached(x, n, norm, &lv, &rng, &ml, mw2, cache, nullptr));
                      GK(gc_ms_select_cached(cache, n, &lv, mw2, &ml, &ql, wq2, nullptr));
                      GK(gc_ms_decode(wq2, mw2, nullptr, n, norm, &lv, &ml, &ql, 1, 1.0f, out, nullptr));
                  }, 0, {}});
    vs.push_back({"STEP q-cache: ... + decode PERTHREAD", [&] {
                      gc_absmax_f32(x, nullptr, n, norm, aws, nullptr);
                      GK(gc_ms_mask_encode_cached(x, n, norm, &lv, &rng, &ml, mw2, cache, nullptr));
                      GK(gc_ms_select_cached(cache, n, &lv, mw2, &ml, &ql, wq2, nullptr));
                      decpt(wq2, mw2);
                  }, 0, {}});
    auto selc2 = [&](auto kern, const uint32_t *msrc, uint32_t *dst) {
        hipLaunchKernelGGL(kern, g8(Mq), dim3(256), 0, 0, (const void *)cache2, n32,
                           MaskArg{msrc, Mm, ml.bits, lv.count - 1, 1}, fd, Mq, ql.bits, 3u, dst);
    };
    vs.push_back({"STEP q-cache, lab launches, NT stores", [&] {
                      gc_absmax_f32(x, nullptr, n, norm, aws, nullptr);
                      mask8(k_ms_mask_fast_o2<32, MSV_ROLL | MSV_UFLAG, 1>, mw2, cache2)();
                      selc2(k_ms_select_cache_o2<10, 2, 1, true>, mw2, wq2);
                      decpt(wq2, mw2);
                  }, 0, {}});
    vs.push_back({"STEP q-cache, lab launches, plain stores", [&] {
                      gc_absmax_f32(x, nullptr, n, norm, aws, nullptr);
                      mask8(k_ms_mask_fast_o2<32, MSV_ROLL | MSV_UFLAG | MSV_PLAINST, 1>, mw2, cache2)();
                      selc2(k_ms_select_cache_o2<10, 2, 1, false>, mw2, wq2);
                      decpt(wq2, mw2);
                  }, 0, {}});
    vs.push_back({"mask + cache plain stores alone", mask8(k_ms_mask_fast_o2<32, MSV_ROLL | MSV_UFLAG | MSV_PLAINST, 1>,
                                                           mw2, cache2), 0, {}});
    vs.push_back({"decode PERTHREAD alone", [&] {
                      hipLaunchKernelGGL((k_ms_decode_fast<10, 1, 2, MSV_PERTHREAD>), dim3((Mq / 4 + 255) / 256),
                                         dim3(256), 0, 0, wq3, MaskArg{mw3, Mm, ml.bits, lv.count - 1, 1}, fd, n32,
                                         norm, la, fa, Mq, ql.bits, sub, 1.0f, out);
                  }, 0, {}});
    vs.push_back({"seq: one-pass + decode: fresh words, old mask", [&] {
                      p_w1();
                      GK(gc_ms_decode(wq3, mw, nullptr, n, norm, &lv, &ml, &ql, 1, 1.0f, out, nullptr));
                  }, 0, {}});
    vs.push_back({"seq: one-pass + decode: old words, fresh mask", [&] {
                      p_w1();
                      GK(gc_ms_decode(wq, mw3, nullptr, n, norm, &lv, &ml, &ql, 1, 1.0f, out, nullptr));
                  }, 0, {}});
    vs.push_back({"seq: one-pass + decode of other words", [&] {
                      p_w1();
                      GK(gc_ms_decode(wq, mw, nullptr, n, norm, &lv, &ml, &ql, 1, 1.0f, out, nullptr));
                  }, 0, {}});
    vs.push_back({"seq: absmax + one-pass + decode plain stores", [&] {
                      gc_absmax_f32(x, nullptr, n, norm, aws, nullptr);
                      p_w1();
                      v_dec(k_ms_decode_fast<10, 0, 2, MSV_PLAINST>, out2)();
                  }, xb * 3 + mb * 2 + qb * 2, {}});
    vs.push_back({"seq: absmax + mask/cache + select + decode NT (product)", [&] {
                      gc_absmax_f32(x, nullptr, n, norm, aws, nullptr);
                      p_maskc();
                      p_selc();
                      p_dec(0)();
                  }, 0, {}});
    vs.push_back({"seq: absmax + mask/cache + select + decode plain stores", [&] {
                      gc_absmax_f32(x, nullptr, n, norm, aws, nullptr);
                      p_maskc();
                      p_selc();
                      v_dec(k_ms_decode_fast<10, 0, 2, MSV_PLAINST>, out2)();
                  }, 0, {}});
    // the same sequences on a created (non-null) stream, as a torch process runs them
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    vs.push_back({"seq on a created stream: absmax + one-pass + decode NT", [&] {
                      gc_absmax_f32(x, nullptr, n, norm, aws, s2);
                      GK(gc_ms_encode_w1(x, n, norm, &lv, &rng, &ml, &ql, mw3, wq3, s2));
                      GK(gc_ms_decode(wq, mw, nullptr, n, norm, &lv, &ml, &ql, 0, 1.0f, out, s2));
                  }, 0, {}, s2});
    for (auto &v : vs) {  // each variant once, synchronised, named first (a fault names its variant)
        printf("run-check %s\n", v.name);
        fflush(stdout);
        v.f();
        CK(hipDeviceSynchronize());
    }
    for (int rep = 0; rep < 5; ++rep)
        for (auto &v : vs) {
            T.st = v.st;
            v.t.push_back(T.run(v.f, 30));
        }
    for (auto &v : vs) {
        std::sort(v.t.begin(), v.t.end());
        row(v.name, v.t[v.t.size() / 2], v.bytes);
    }
    return 0;
}
