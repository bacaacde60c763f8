// lab2.hip — measurement harness, round-1 second pass (not product code).
//   1. integer stochastic rounding (ENC_INT) vs the product encode: equality
//      of the packed words, settled interleaved A/B timing, compute floors;
//   2. Infinity-Cache (MALL) reuse between the two passes of one step:
//      after a read-only flush, is a re-read of x served on-die, and in which
//      traversal order?
// Build: make -C tools lab2 ; run: tools/lab2 [n]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <vector>

#include "gcodec.h"
#include "absmax.h"
#include "encode_lab_kernel.h"

using namespace gc;
using namespace gclab;

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(2);                                                                        \
        }                                                                                   \
    } while (0)

__global__ void k_fill(float *x, uint64_t n, uint32_t seed)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        float u = (float)(int32_t)h * 0x1p-31f;
        x[i] = u * u * u * 0.05f;
    }
}

// linear read, forward or backward (absmax-like), 2 float4 in flight per thread
template <bool REV>
__global__ __launch_bounds__(256) void k_read(const float4 *x, uint64_t n4, uint32_t *out)
{
    uint32_t m = 0;
    const uint64_t stride = gridDim.x * 256ull;
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < n4; t += stride) {
        const float4 v = x[REV ? n4 - 1 - t : t];
        m = max(m, max(max(__float_as_uint(v.x), __float_as_uint(v.y)), max(__float_as_uint(v.z), __float_as_uint(v.w))));
    }
    if (m == 0x7fffffffu)
        out[0] = m;
}

// planar read in the encode's tile order (tile t = L float4s at k*M + 4t)
template <int L, bool REV>
__global__ __launch_bounds__(256) void k_read_planar(const float *x, uint32_t M, uint32_t *out)
{
    uint32_t m = 0;
    const uint32_t tiles = M >> 2;
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < tiles; t += gridDim.x * 256u) {
        const uint32_t tt = REV ? tiles - 1 - t : t;
#pragma unroll
        for (int k = 0; k < L; ++k) {
            const float4 v = *reinterpret_cast<const float4 *>(x + k * M + 4 * tt);
            m = max(m, max(max(__float_as_uint(v.x), __float_as_uint(v.y)), max(__float_as_uint(v.z), __float_as_uint(v.w))));
        }
    }
    if (m == 0x7fffffffu)
        out[0] = m;
}

template <bool NT>
__global__ __launch_bounds__(256) void k_write(uint4 *o, uint64_t n4)
{
    typedef uint32_t u4v __attribute__((ext_vector_type(4)));
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < n4; t += gridDim.x * 256ull) {
        const u4v v = {(uint32_t)t, 1u, 2u, 3u};
        if (NT)
            __builtin_nontemporal_store(v, reinterpret_cast<u4v *>(o + t));
        else
            *reinterpret_cast<u4v *>(o + t) = v;
    }
}

// read-only flush: fills the Infinity Cache with clean lines of another buffer
__global__ __launch_bounds__(256) void k_flush(const uint4 *o, uint64_t n4, uint32_t *out)
{
    uint32_t acc = 0;
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < n4; t += gridDim.x * 256ull)
        acc ^= o[t].x;
    if (acc == 0x12345678u)
        out[0] = acc;
}

// the encode's memory pattern with no arithmetic, NT loads / NT stores
template <int L, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_copy_planar(const float *x, uint32_t M, uint32_t *words)
{
    typedef float f4v __attribute__((ext_vector_type(4)));
    typedef uint32_t u4v __attribute__((ext_vector_type(4)));
    const uint32_t quads = M >> 2;
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < quads; t += gridDim.x * 256u) {
        u4v acc = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < L; ++k) {
            const f4v *p = reinterpret_cast<const f4v *>(x + k * M + 4 * t);
            const f4v v = NTL ? __builtin_nontemporal_load(p) : *p;
            acc ^= __builtin_bit_cast(u4v, v);
        }
        if (NTS)
            __builtin_nontemporal_store(acc, reinterpret_cast<u4v *>(words + 4 * t));
        else
            *reinterpret_cast<u4v *>(words + 4 * t) = acc;
    }
}

// dense decode (qsgd.hip k_qsgd_decode MODE 0) with variants: NT stores,
// U words per thread in flight
template <int L, bool NTS, int U>
__global__ __launch_bounds__(256) void k_decode_lab(const uint32_t *__restrict__ words, uint64_t n,
                                                    const float *__restrict__ normp, float s, int32_t sub, uint32_t w,
                                                    uint64_t M, float alpha, float *__restrict__ out)
{
    typedef float f4v __attribute__((ext_vector_type(4)));
    const float c = *normp / s;
    const uint32_t mask = (1u << w) - 1u;
    const uint32_t quads = (uint32_t)(M >> 2);
    const uint32_t stride = gridDim.x * 256u;
    for (uint32_t t0 = blockIdx.x * 256u + threadIdx.x; t0 < quads; t0 += U * stride) {
        uint4 wd[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (t0 + u * stride < quads)
                wd[u] = *reinterpret_cast<const uint4 *>(words + 4ull * (t0 + u * stride));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t t = t0 + u * stride;
            if (t >= quads)
                break;
#pragma unroll
            for (int k = 0; k < L; ++k) {
                const uint64_t i0 = (uint64_t)k * M + 4ull * t;
                if (i0 + 4 <= n) {
                    const uint32_t sh = (uint32_t)k * w;
                    f4v o;
                    o.x = (c * (float)((int32_t)((wd[u].x >> sh) & mask) - sub)) * alpha;
                    o.y = (c * (float)((int32_t)((wd[u].y >> sh) & mask) - sub)) * alpha;
                    o.z = (c * (float)((int32_t)((wd[u].z >> sh) & mask) - sub)) * alpha;
                    o.w = (c * (float)((int32_t)((wd[u].w >> sh) & mask) - sub)) * alpha;
                    if (NTS)
                        __builtin_nontemporal_store(o, reinterpret_cast<f4v *>(out + i0));
                    else
                        *reinterpret_cast<f4v *>(out + i0) = o;
                }
            }
        }
    }
}

// Markstein quotient by a level scale s = 2^b - 1 (ms_fast.h order-0 decode):
// every positive float a with exponent in [-100, 113], against IEEE a / s
__global__ __launch_bounds__(256) void k_divcheck_s(float s, unsigned long long *bad, uint32_t *example)
{
    const float y = 1.0f / s;
    unsigned long long nb = 0;
    const uint32_t first = (uint32_t)(127 - 100) << 23, last = (uint32_t)(127 + 114) << 23;
    for (uint32_t u = first + blockIdx.x * 256u + threadIdx.x; u < last; u += gridDim.x * 256u) {
        const float a = __uint_as_float(u);
        const float q0 = a * y;
        const float d = fmaf(fmaf(-s, q0, a), y, q0);
        if (__float_as_uint(d) != __float_as_uint(a / s)) {
            ++nb;
            example[0] = u;
        }
    }
    if (nb)
        atomicAdd(bad, nb);
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    template <class F>
    float run(F f, int reps = 20)
    {
        f();
        f();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < reps; ++i)
            f();
        CK(hipEventRecord(b, 0));
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

int main(int argc, char **argv)
{
    uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 100000000ull;
    const uint32_t bits = 4;
    gc_lanes ln;
    if (gc_qsgd_layout(n, bits, 1, &ln) != GC_OK) {
        fprintf(stderr, "layout: %s\n", gc_last_error());
        return 1;
    }
    const uint32_t M = (uint32_t)ln.plane_words;
    float *x, *norm, *dec_out;
    uint32_t *words, *words2, *scratch;
    uint4 *fl;
    const uint64_t flbytes = 600ull << 20;
    CK(hipMalloc(&x, n * 4 + 64));
    CK(hipMalloc(&norm, 64));
    CK(hipMalloc(&dec_out, n * 4 + 64));
    CK(hipMalloc(&words, (size_t)M * 4 + 64));
    CK(hipMalloc(&words2, (size_t)M * 4 + 64));
    CK(hipMalloc(&scratch, 64));
    CK(hipMalloc(&fl, flbytes));
    CK(hipMemset(fl, 0, flbytes));
    void *ws;
    CK(hipMalloc(&ws, gc_absmax_workspace_size()));
    CK(hipMemset(ws, 0, gc_absmax_workspace_size()));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, x, n, 7u);
    CK(hipDeviceSynchronize());
    gc_absmax_f32(x, nullptr, n, norm, ws, nullptr);
    CK(hipDeviceSynchronize());
    printf("n=%llu  M=%u words  lanes w=%u L=%u\n", (unsigned long long)n, M, ln.bits, ln.per_word);
    const double enc_bytes = 4.0 * n + 4.0 * M, rd_bytes = 4.0 * n, step_bytes = 8.0 * n + 4.0 * M;
    Timer T;

    RngArgs ra{42, 0, nullptr, n};
    const float s = 15.0f;
    const int32_t qmax = 15;
    gc_rng rng = {GC_RNG_PHILOX, 0, 42, 0, nullptr};
    auto enc = [&](auto kern, unsigned g, uint32_t *dst) {
        return [=] {
            hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, x, (const int64_t *)nullptr, n, norm, s, qmax, ln.bits,
                               (uint64_t)M, ra, dst);
        };
    };
    auto product_enc = [&] { gc_qsgd_encode(x, nullptr, n, norm, bits, &ln, &rng, words, nullptr); };
    auto product_am = [&] { gc_absmax_f32(x, nullptr, n, norm, ws, nullptr); };

    // ---- 1. equality ----
    std::vector<uint32_t> a(M), b(M);
    product_enc();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(a.data(), words, (size_t)M * 4, hipMemcpyDeviceToHost));
    auto same = [&](const char *nm, std::function<void()> f) {
        CK(hipMemset(words2, 0, (size_t)M * 4));
        f();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(b.data(), words2, (size_t)M * 4, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint32_t i = 0; i < M; ++i)
            bad += a[i] != b[i];
        printf("%-40s == product: %s (%llu words differ)\n", nm, bad == 0 ? "yes" : "NO", (unsigned long long)bad);
    };
    same("ENC_INT", enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT>, 2048, words2));
    same("ENC_INT | ENC_REV", enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT | ENC_REV>, 2048, words2));
    same("ENC_INT | ENC_NT", enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT | ENC_NT>, 8192, words2));
    same("ENC_INT | ENC_NT | ENC_NTS", enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT | ENC_NT | ENC_NTS>, 8192, words2));
    {
        // lab decode == product decode
        float *d2;
        CK(hipMalloc(&d2, n * 4 + 64));
        gc_qsgd_decode(words, nullptr, n, norm, bits, &ln, 1.0f, dec_out, nullptr);
        hipLaunchKernelGGL((k_decode_lab<6, true, 2>), dim3(4096), dim3(256), 0, 0, words, n, norm, s, qmax, ln.bits,
                           (uint64_t)M, 1.0f, d2);
        CK(hipDeviceSynchronize());
        std::vector<uint32_t> da(n), db(n);
        CK(hipMemcpy(da.data(), dec_out, n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(db.data(), d2, n * 4, hipMemcpyDeviceToHost));
        printf("%-40s == product: %s\n", "decode lab NTS U2", memcmp(da.data(), db.data(), n * 4) == 0 ? "yes" : "NO");
        CK(hipFree(d2));
    }

    if (getenv("LAB_DIVS")) {
        unsigned long long *bad;
        uint32_t *ex;
        CK(hipMalloc(&bad, 8));
        CK(hipMalloc(&ex, 8));
        for (int b = 1; b <= 16; ++b) {
            CK(hipMemset(bad, 0, 8));
            hipLaunchKernelGGL(k_divcheck_s, dim3(16384), dim3(256), 0, 0, (float)((1u << b) - 1u), bad, ex);
            unsigned long long h = 0;
            uint32_t e = 0;
            CK(hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&e, ex, 4, hipMemcpyDeviceToHost));
            printf("divcheck s=2^%d-1: %llu mismatches over every a in [2^-100, 2^114)%s\n", b, h, h ? " (see example)" : "");
            if (h)
                printf("   e.g. a=%08x\n", e);
        }
        return 0;
    }
    // ---- 2. settled interleaved A/B ----
    {
        float tot = 0;
        while (tot < 500.0f)
            tot += 100 * T.run([&] { product_am(); product_enc(); }, 100);
        struct V {
            const char *name;
            std::function<void()> f;
            double bytes;
            std::vector<float> t;
        };
        std::vector<V> vs;
        auto step = [&](std::function<void()> am, std::function<void()> en) {
            return [=] { am(); en(); };
        };
        vs.push_back({"AB: step product", step(product_am, product_enc), step_bytes, {}});
        vs.push_back({"AB: encode product", product_enc, enc_bytes, {}});
        static char names[64][96];
        int ni = 0;
        (void)ni;
        auto cp = [&](auto kern, unsigned g) {
            return [=] { hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, x, M, words2); };
        };
        vs.push_back({"roof: planar R+W plain g=8192", cp(k_copy_planar<6, false, false>, 8192), enc_bytes, {}});
        vs.push_back({"roof: planar R+W NT loads g=8192", cp(k_copy_planar<6, true, false>, 8192), enc_bytes, {}});
        vs.push_back({"roof: planar R+W NT loads g=12288", cp(k_copy_planar<6, true, false>, 12288), enc_bytes, {}});
        vs.push_back({"roof: planar R+W NT ld+st g=12288", cp(k_copy_planar<6, true, true>, 12288), enc_bytes, {}});
        vs.push_back({"roof: planar R+W NT ld+st g=16384", cp(k_copy_planar<6, true, true>, 16384), enc_bytes, {}});
        vs.push_back({"AB: encode INT NT g=12288 (product)", enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT | ENC_NT>, 12288, words2), enc_bytes, {}});
        vs.push_back({"AB: encode INT NT NTS g=12288", enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT | ENC_NT | ENC_NTS>, 12288, words2), enc_bytes, {}});
        vs.push_back({"AB: encode INT NT g=16384", enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT | ENC_NT>, 16384, words2), enc_bytes, {}});
        vs.push_back({"AB: encode INT NT NTS g=16384", enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT | ENC_NT | ENC_NTS>, 16384, words2), enc_bytes, {}});
        vs.push_back({"AB: encode INT NT g=24576", enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT | ENC_NT>, 24576, words2), enc_bytes, {}});
        vs.push_back({"AB: encode INT NT MINW=5 g=12288", enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT | ENC_NT, 5>, 12288, words2), enc_bytes, {}});
        vs.push_back({"AB: step product", step(product_am, product_enc), step_bytes, {}});
        vs.push_back({"AB: step + NTS", step(product_am, enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT | ENC_NT | ENC_NTS>, 12288, words2)), step_bytes, {}});
        vs.push_back({"AB: step + NTS g=16384", step(product_am, enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT | ENC_NT | ENC_NTS>, 16384, words2)), step_bytes, {}});
        vs.push_back({"AB: compute only INT g=12288", enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT | ENC_ABL_L2>, 12288, words2), enc_bytes, {}});
        const double dec_bytes = 4.0 * n + 4.0 * M;
        auto dec = [&](auto kern, unsigned g) {
            return [=] {
                hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, words, n, norm, s, qmax, ln.bits, (uint64_t)M, 1.0f,
                                   dec_out);
            };
        };
        vs.push_back({"AB: decode product", [&] { gc_qsgd_decode(words, nullptr, n, norm, bits, &ln, 1.0f, dec_out, nullptr); }, dec_bytes, {}});
        vs.push_back({"AB: decode lab U1 g=2048", dec(k_decode_lab<6, false, 1>, 2048), dec_bytes, {}});
        vs.push_back({"AB: decode lab U1 g=16384", dec(k_decode_lab<6, false, 1>, 16384), dec_bytes, {}});
        vs.push_back({"AB: decode lab NTS U1 g=2048", dec(k_decode_lab<6, true, 1>, 2048), dec_bytes, {}});
        vs.push_back({"AB: decode lab NTS U1 g=16384", dec(k_decode_lab<6, true, 1>, 16384), dec_bytes, {}});
        vs.push_back({"AB: decode lab U2 g=4096", dec(k_decode_lab<6, false, 2>, 4096), dec_bytes, {}});
        vs.push_back({"AB: decode lab NTS U2 g=4096", dec(k_decode_lab<6, true, 2>, 4096), dec_bytes, {}});
        vs.push_back({"roof: write-only 400 MB", [&] {
                          hipLaunchKernelGGL(k_write<false>, dim3(8192), dim3(256), 0, 0, (uint4 *)dec_out, n / 4);
                      }, rd_bytes, {}});
        vs.push_back({"roof: write-only 400 MB NT", [&] {
                          hipLaunchKernelGGL(k_write<true>, dim3(8192), dim3(256), 0, 0, (uint4 *)dec_out, n / 4);
                      }, rd_bytes, {}});
        vs.push_back({"AB: absmax product", product_am, rd_bytes, {}});
        vs.push_back({"AB: read-only roofline", [&] {
                          hipLaunchKernelGGL(k_read<false>, dim3(2048), dim3(256), 0, 0, (const float4 *)x, n / 4, scratch);
                      }, rd_bytes, {}});
        for (int rep = 0; rep < 7; ++rep)
            for (auto &v : vs)
                v.t.push_back(T.run(v.f, 30));
        for (auto &v : vs) {
            std::sort(v.t.begin(), v.t.end());
            row(v.name, v.t[v.t.size() / 2], v.bytes);
        }
    }
    if (getenv("LAB_MALL") == nullptr)
        return 0;

    // ---- 3. MALL reuse: flush, run `pre` untimed, time `body` ----
    {
        hipEvent_t e0, e1, e2;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventCreate(&e2));
        auto cold = [&](const char *nm, std::function<void()> pre, std::function<void()> body, double bytes,
                        double pre_bytes) {
            std::vector<float> tp, tb;
            for (int i = 0; i < 12; ++i) {
                hipLaunchKernelGGL(k_flush, dim3(8192), dim3(256), 0, 0, fl, flbytes / 16, scratch);
                CK(hipEventRecord(e0, 0));
                pre();
                CK(hipEventRecord(e1, 0));
                body();
                CK(hipEventRecord(e2, 0));
                CK(hipEventSynchronize(e2));
                float m1, m2;
                CK(hipEventElapsedTime(&m1, e0, e1));
                CK(hipEventElapsedTime(&m2, e1, e2));
                if (i >= 2) {
                    tp.push_back(m1);
                    tb.push_back(m2);
                }
            }
            std::sort(tp.begin(), tp.end());
            std::sort(tb.begin(), tb.end());
            char nm2[128];
            if (pre_bytes > 0) {
                snprintf(nm2, sizeof nm2, "%s [first]", nm);
                row(nm2, tp[tp.size() / 2], pre_bytes);
            }
            snprintf(nm2, sizeof nm2, "%s [second]", nm);
            row(nm2, tb[tb.size() / 2], bytes);
            if (pre_bytes > 0) {
                snprintf(nm2, sizeof nm2, "%s [both]", nm);
                row(nm2, tp[tp.size() / 2] + tb[tb.size() / 2], bytes + pre_bytes);
            }
        };
        const uint64_t n4 = n / 4;
        auto rd = [&](bool rev, uint64_t q4) {
            return [=] {
                if (rev)
                    hipLaunchKernelGGL(k_read<true>, dim3(2048), dim3(256), 0, 0, (const float4 *)x, q4, scratch);
                else
                    hipLaunchKernelGGL(k_read<false>, dim3(2048), dim3(256), 0, 0, (const float4 *)x, q4, scratch);
            };
        };
        auto nothing = [] {};
        cold("MALL: cold read 400MB fwd", nothing, rd(false, n4), rd_bytes, 0);
        cold("MALL: cold read 400MB rev", nothing, rd(true, n4), rd_bytes, 0);
        cold("MALL: read fwd then fwd", rd(false, n4), rd(false, n4), rd_bytes, rd_bytes);
        cold("MALL: read fwd then rev", rd(false, n4), rd(true, n4), rd_bytes, rd_bytes);
        cold("MALL: 200MB read fwd then fwd", rd(false, n4 / 2), rd(false, n4 / 2), rd_bytes / 2, rd_bytes / 2);
        cold("MALL: 128MB read fwd then fwd", rd(false, n4 / 25 * 8), rd(false, n4 / 25 * 8), rd_bytes * 0.32,
             rd_bytes * 0.32);
        auto pl = [&](bool rev) {
            return [=] {
                if (rev)
                    hipLaunchKernelGGL((k_read_planar<6, true>), dim3(2048), dim3(256), 0, 0, x, M, scratch);
                else
                    hipLaunchKernelGGL((k_read_planar<6, false>), dim3(2048), dim3(256), 0, 0, x, M, scratch);
            };
        };
        cold("MALL: planar read fwd then planar rev", pl(false), pl(true), rd_bytes, rd_bytes);
        cold("MALL: planar read fwd then planar fwd", pl(false), pl(false), rd_bytes, rd_bytes);
        cold("step: absmax -> encode product", product_am, product_enc, enc_bytes, rd_bytes);
        cold("step: absmax -> encode INT", product_am, enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT>, 2048, words2), enc_bytes,
             rd_bytes);
        cold("step: absmax -> encode INT REV", product_am, enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT | ENC_REV>, 2048, words2),
             enc_bytes, rd_bytes);
        cold("step: planar read fwd -> encode INT REV", pl(false),
             enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT | ENC_REV>, 2048, words2), enc_bytes, rd_bytes);
        cold("step: planar read fwd -> encode INT", pl(false), enc(gclab::k_qsgd_encode<6, 0, 0, ENC_INT>, 2048, words2),
             enc_bytes, rd_bytes);
    }
    return 0;
}
