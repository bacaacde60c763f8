// encode_lab.hip — measurement harness for the QSGD encode path (not product
// code).  Times, with HIP events, on a 100M-fp32 bucket:
//   * memory rooflines with the encode's exact access pattern (read-only,
//     read L planes + write packed words),
//   * the product entry points through the C ABI (gc_absmax_f32,
//     gc_qsgd_encode, gc_qsgd_decode),
//   * ablations of the encode kernel (no Philox / no exact division) and
//     grid sizes, to locate the bound.
// Build: make -C tools encode_lab ; run: tools/encode_lab [n]
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

// read-only stream (absmax-like roofline)
__global__ __launch_bounds__(256) void k_read(const float4 *x, uint64_t n4, uint32_t *out)
{
    uint32_t m = 0;
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < n4; t += gridDim.x * 256ull) {
        float4 v = x[t];
        m = max(m, max(max(__float_as_uint(v.x), __float_as_uint(v.y)), max(__float_as_uint(v.z), __float_as_uint(v.w))));
    }
    if (m == 0x7fffffffu)
        out[0] = m;
}

// the encode's exact memory pattern with no arithmetic: L float4 planes -> uint4
template <int L>
__global__ __launch_bounds__(256) void k_copy_planar(const float *x, uint32_t M, uint32_t *words)
{
    const uint32_t quads = M >> 2;
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < quads; t += gridDim.x * 256u) {
        uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < L; ++k) {
            float4 v = *reinterpret_cast<const float4 *>(x + k * M + 4 * t);
            acc.x ^= __float_as_uint(v.x);
            acc.y ^= __float_as_uint(v.y);
            acc.z ^= __float_as_uint(v.z);
            acc.w ^= __float_as_uint(v.w);
        }
        *reinterpret_cast<uint4 *>(words + 4 * t) = acc;
    }
}

// tiled-planar pattern: one wave owns a tile of 256 words = 6 x 256-float
// chunks that are ADJACENT in memory (6 KB contiguous per wave)
template <int L>
__global__ __launch_bounds__(256) void k_copy_tiled(const float *x, uint32_t tiles, uint32_t *words)
{
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t tile = (blockIdx.x * 256u + threadIdx.x) >> 6; tile < tiles; tile += gridDim.x * 4u) {
        const float *base = x + (size_t)tile * (L * 256u) + 4u * lane;
        uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < L; ++k) {
            float4 v = *reinterpret_cast<const float4 *>(base + k * 256);
            acc.x ^= __float_as_uint(v.x);
            acc.y ^= __float_as_uint(v.y);
            acc.z ^= __float_as_uint(v.z);
            acc.w ^= __float_as_uint(v.w);
        }
        *reinterpret_cast<uint4 *>(words + (size_t)tile * 256u + 4u * lane) = acc;
    }
}

template <int L>
__global__ __launch_bounds__(256) void k_read_planar(const float *x, uint32_t M, uint32_t *out)
{
    uint32_t m = 0;
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < (M >> 2); t += gridDim.x * 256u) {
#pragma unroll
        for (int k = 0; k < L; ++k) {
            float4 v = *reinterpret_cast<const float4 *>(x + k * M + 4 * t);
            m = max(m, max(max(__float_as_uint(v.x), __float_as_uint(v.y)), max(__float_as_uint(v.z), __float_as_uint(v.w))));
        }
    }
    if (m == 0x7fffffffu)
        out[0] = m;
}

__global__ __launch_bounds__(256) void k_write(uint4 *o, uint64_t n4)
{
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < n4; t += gridDim.x * 256ull)
        o[t] = make_uint4((uint32_t)t, 1, 2, 3);
}

__global__ __launch_bounds__(256) void k_write_nt(uint4 *o, uint64_t n4)
{
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < n4; t += gridDim.x * 256ull) {
        uint4 v = make_uint4((uint32_t)t, 1, 2, 3);
        __builtin_nontemporal_store(v.x, &o[t].x);
        __builtin_nontemporal_store(v.y, &o[t].y);
        __builtin_nontemporal_store(v.z, &o[t].z);
        __builtin_nontemporal_store(v.w, &o[t].w);
    }
}

// read-only flush: fills the Infinity Cache with CLEAN lines of another buffer
__global__ __launch_bounds__(256) void k_flush(uint4 *o, uint64_t n4)
{
    uint32_t acc = 0;
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < n4; t += gridDim.x * 256ull)
        acc ^= o[t].x;
    if (acc == 0x12345678u)
        o[0].y = acc;
}

// absmax walking the array downward (lab variant of the product's k_absmax)
__global__ __launch_bounds__(1024) void k_absmax_rev(const float4 *x, uint64_t n4, uint32_t *out)
{
    uint32_t m = 0;
    const uint64_t stride = gridDim.x * 1024ull;
    for (uint64_t t = blockIdx.x * 1024ull + threadIdx.x; t < n4; t += stride) {
        float4 v = x[n4 - 1 - t];
        m = max(m, max(max(__float_as_uint(v.x) & 0x7fffffffu, __float_as_uint(v.y) & 0x7fffffffu),
                       max(__float_as_uint(v.z) & 0x7fffffffu, __float_as_uint(v.w) & 0x7fffffffu)));
    }
    for (int o = 32; o > 0; o >>= 1)
        m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
    if ((threadIdx.x & 63) == 0 && m)
        atomicMax(out, m);
}

// Markstein one-correction quotient vs the IEEE division, on random operand
// pairs inside the fast-path range (same make_div / Range as the kernel)
__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_divcheck(uint64_t seed, uint64_t count, int allones,
                                                  unsigned long long *stats, uint32_t *example)
{
    unsigned long long tested = 0, bad1 = 0, bad2 = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < count; i += gridDim.x * 256ull) {
        const uint64_t h = mix64(seed * 0x100000000ull + i);
        const int eb = (int)(h % 201) - 100;                   // norm exponent in [-100, 100]
        const int eq = (int)((h >> 8) % 186) - 121;            // quotient exponent in [-121, 64]
        const uint32_t mb = allones ? 0x7fffffu : (uint32_t)(h >> 16) & 0x7fffffu;
        const uint32_t ma = (uint32_t)(h >> 40) & 0x7fffffu;
        int ea = eb + eq;
        if (ea < -126 || ea > 127)
            continue;
        const float b = __uint_as_float((uint32_t)(127 + eb) << 23 | mb);
        const float a = __uint_as_float((uint32_t)(127 + ea) << 23 | ma);
        const gc::DivNorm d = gc::make_div(b);
        gc::Range rg;
        rg.add4(make_float4(a, a, a, a));
        if (!d.fast || rg.slow(d))
            continue;
        ++tested;
        const float ref = a / b;
        const float q1 = gc::div_fast(a, d), q2 = gc::div_fast2(a, d);
        if (__float_as_uint(q1) != __float_as_uint(ref)) {
            ++bad1;
            example[0] = __float_as_uint(a);
            example[1] = __float_as_uint(b);
        }
        if (__float_as_uint(q2) != __float_as_uint(ref))
            ++bad2;
    }
    atomicAdd(&stats[0], tested);
    if (bad1)
        atomicAdd(&stats[1], bad1);
    if (bad2)
        atomicAdd(&stats[2], bad2);
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
    printf("%-44s %9.1f us  %8.1f GB/s  %5.1f%% of 8 TB/s\n", name, ms * 1e3, gbs, 100.0 * gbs / 8000.0);
}

int main(int argc, char **argv)
{
    uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 100000000ull;
    const bool quick = argc > 2;  // small-n run: rooflines + product + ablations only
    const uint32_t bits = 4;
    gc_lanes ln;
    if (gc_qsgd_layout(n, bits, 1, &ln) != GC_OK) {
        fprintf(stderr, "layout: %s\n", gc_last_error());
        return 1;
    }
    const uint32_t M = (uint32_t)ln.plane_words;
    float *x, *norm, *dec;
    uint32_t *words, *words2, *scratch;
    CK(hipMalloc(&x, n * 4 + 64));
    CK(hipMalloc(&dec, n * 4 + 64));
    CK(hipMalloc(&norm, 64));
    CK(hipMalloc(&words, (size_t)M * 4 + 64));
    CK(hipMalloc(&words2, (size_t)M * 4 + 64));
    CK(hipMalloc(&scratch, 64));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, x, n, 7u);
    CK(hipDeviceSynchronize());
    printf("n=%llu  M=%u words  lanes w=%u L=%u\n", (unsigned long long)n, M, ln.bits, ln.per_word);
    const double enc_bytes = 4.0 * n + 4.0 * M, rd_bytes = 4.0 * n;
    Timer T;

    row("roofline: read-only stream (n fp32)", T.run([&] {
            hipLaunchKernelGGL(k_read, dim3(2048), dim3(256), 0, 0, (const float4 *)x, n / 4, scratch);
        }), rd_bytes);
    for (unsigned g : {1024u, 2048u, 4096u, 8192u}) {
        char nm[96];
        snprintf(nm, sizeof nm, "roofline: planar read + packed write g=%u", g);
        row(nm, T.run([&] { hipLaunchKernelGGL(k_copy_planar<6>, dim3(g), dim3(256), 0, 0, x, M, words2); }),
            enc_bytes);
    }
    for (unsigned g : {2048u, 8192u, 16384u}) {
        char nm[96];
        snprintf(nm, sizeof nm, "roofline: TILED read + packed write g=%u", g);
        const uint32_t tiles = (uint32_t)(n / (6 * 256));
        row(nm, T.run([&] { hipLaunchKernelGGL(k_copy_tiled<6>, dim3(g), dim3(256), 0, 0, x, tiles, words2); }),
            (double)tiles * 6 * 256 * 4 + (double)tiles * 256 * 4);
    }
    row("roofline: planar read only g=2048", T.run([&] {
            hipLaunchKernelGGL(k_read_planar<6>, dim3(2048), dim3(256), 0, 0, x, M, scratch);
        }), rd_bytes);
    row("roofline: planar read only g=16384", T.run([&] {
            hipLaunchKernelGGL(k_read_planar<6>, dim3(16384), dim3(256), 0, 0, x, M, scratch);
        }), rd_bytes);
    row("roofline: write-only 400 MB", T.run([&] {
            hipLaunchKernelGGL(k_write, dim3(8192), dim3(256), 0, 0, (uint4 *)dec, n / 4);
        }), rd_bytes);
    row("roofline: write-only 400 MB nontemporal", T.run([&] {
            hipLaunchKernelGGL(k_write_nt, dim3(8192), dim3(256), 0, 0, (uint4 *)dec, n / 4);
        }), rd_bytes);
    row("product gc_absmax_f32 (memset + kernel)", T.run([&] { gc_absmax_f32(x, nullptr, n, norm, nullptr, nullptr); }),
        rd_bytes);
    void *ws;
    CK(hipMalloc(&ws, gc_absmax_workspace_size()));
    CK(hipMemset(ws, 0, gc_absmax_workspace_size()));
    row("product gc_absmax_f32 (workspace, 1 launch)", T.run([&] { gc_absmax_f32(x, nullptr, n, norm, ws, nullptr); }),
        rd_bytes);
    {
        // max-norm grid / loads-in-flight sweep (two-level ticket above 256 blocks)
        uint32_t ref = 0, got = 0;
        CK(hipMemcpy(&ref, norm, 4, hipMemcpyDeviceToHost));
        float *nm2;
        CK(hipMalloc(&nm2, 64));
        auto am = [&](const char *nm, auto kern, unsigned grid, unsigned bt) {
            row(nm, T.run([&] {
                    hipLaunchKernelGGL(kern, dim3(grid), dim3(bt), 0, 0, x, (const int64_t *)nullptr, n,
                                       (uint32_t *)nm2, (uint32_t *)ws);
                }), rd_bytes);
            CK(hipMemcpy(&got, nm2, 4, hipMemcpyDeviceToHost));
            if (got != ref)
                printf("   ^ WRONG NORM %08x vs %08x\n", got, ref);
        };
        for (int rep = 0; rep < 2; ++rep) {
            am("absmax 256x1024 U4 (product)", k_absmax<0, true, 1024, 4>, 256, 1024);
            am("absmax 256x1024 U8", k_absmax<0, true, 1024, 8>, 256, 1024);
            am("absmax 512x1024 U4 (2-level)", k_absmax<0, true, 1024, 4>, 512, 1024);
            am("absmax 512x1024 U2 (2-level)", k_absmax<0, true, 1024, 2>, 512, 1024);
            am("absmax 512x512 U4 (2-level)", k_absmax<0, true, 512, 4>, 512, 512);
            am("absmax 1024x512 U4 (2-level)", k_absmax<0, true, 512, 4>, 1024, 512);
            am("absmax 1024x256 U4 (2-level)", k_absmax<0, true, 256, 4>, 1024, 256);
            am("absmax 2048x256 U2 (2-level)", k_absmax<0, true, 256, 2>, 2048, 256);
            am("absmax 2048x256 U1 (2-level)", k_absmax<0, true, 256, 1>, 2048, 256);
            am("absmax 4096x256 U1 (2-level)", k_absmax<0, true, 256, 1>, 4096, 256);
        }
        CK(hipFree(nm2));
    }
    gc_rng rng = {GC_RNG_PHILOX, 0, 42, 0, nullptr};
    row("product gc_qsgd_encode", T.run([&] { gc_qsgd_encode(x, nullptr, n, norm, bits, &ln, &rng, words, nullptr); }),
        enc_bytes);
    row("product absmax + encode (one step)", T.run([&] {
            gc_absmax_f32(x, nullptr, n, norm, ws, nullptr);
            gc_qsgd_encode(x, nullptr, n, norm, bits, &ln, &rng, words, nullptr);
        }), 8.0 * n + 4.0 * M);
    row("product gc_qsgd_decode", T.run([&] { gc_qsgd_decode(words, nullptr, n, norm, bits, &ln, 1.0f, dec, nullptr); }),
        4.0 * n + 4.0 * M);

    RngArgs ra{42, 0, nullptr, n};
    const float s = 15.0f;
    const int32_t qmax = 15;
    auto enc = [&](auto kern, unsigned g) {
        return [=] {
            hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, x, (const int64_t *)nullptr, n, norm, s, qmax, ln.bits,
                               (uint64_t)M, ra, words2);
        };
    };
    if (getenv("LAB_PLACE")) {
        // placement: do the HBM addresses of the 6 plane read streams and the
        // write stream (relative to each other) change the encode time?
        float *xp;
        uint32_t *wp;
        const uint64_t padf = 1u << 20;
        CK(hipMalloc(&xp, (n + padf) * 4));
        CK(hipMalloc(&wp, ((size_t)M + padf) * 4));
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, xp, n + padf, 7u);
        CK(hipDeviceSynchronize());
        auto encp = [&](const float *xb, uint32_t *wb, uint64_t Mp) {
            return [=] {
                hipLaunchKernelGGL((gclab::k_qsgd_encode<6, 0, 0, 0>), dim3(2048), dim3(256), 0, 0, xb,
                                   (const int64_t *)nullptr, n, norm, s, qmax, ln.bits, Mp, ra, wb);
            };
        };
        for (int rep = 0; rep < 2; ++rep) {
            row("place: product dst=words", T.run(encp(x, words, M)), enc_bytes);
            row("place: product dst=words2", T.run(encp(x, words2, M)), enc_bytes);
            row("place: product dst=wp", T.run(encp(x, wp, M)), enc_bytes);
            row("place: xp dst=wp", T.run(encp(xp, wp, M)), enc_bytes);
        }
        for (uint64_t woff : {0ull, 64ull, 512ull, 1024ull, 4096ull, 65536ull}) {
            char nm[96];
            snprintf(nm, sizeof nm, "place: dst=wp+%llu words", (unsigned long long)woff);
            row(nm, T.run(encp(xp, wp + woff, M)), enc_bytes);
        }
        for (uint64_t xoff : {64ull, 512ull, 1024ull, 4096ull, 65536ull}) {
            char nm[96];
            snprintf(nm, sizeof nm, "place: x=xp+%llu floats", (unsigned long long)xoff);
            row(nm, T.run(encp(xp + xoff, wp, M)), enc_bytes);
        }
        for (uint64_t d : {64ull, 128ull, 256ull, 512ull, 1024ull, 2048ull, 4096ull, 8192ull, 16384ull}) {
            char nm[96];
            snprintf(nm, sizeof nm, "place: plane stride M+%llu", (unsigned long long)d);
            row(nm, T.run(encp(xp, wp, M + d)), enc_bytes);
        }
        for (uint64_t d : {0ull, 64ull, 256ull, 1024ull, 4096ull}) {
            char nm[96];
            snprintf(nm, sizeof nm, "place: copy_planar stride M+%llu", (unsigned long long)d);
            row(nm, T.run([&] { hipLaunchKernelGGL(k_copy_planar<6>, dim3(2048), dim3(256), 0, 0, xp, (uint32_t)(M + d), wp); }),
                enc_bytes);
        }
        CK(hipFree(xp));
        CK(hipFree(wp));
    }
    for (unsigned g : {2048u, 8192u, 16384u, 32768u}) {
        char nm[96];
        snprintf(nm, sizeof nm, "encode ABL=0 (exact) g=%u", g);
        row(nm, T.run(enc(gclab::k_qsgd_encode<6, 0, 0, 0>, g)), enc_bytes);
    }
    row("encode philox impl 0 (64b mad, xor2)", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_PHX0>, 2048)), enc_bytes);
    row("encode philox impl 2 (mul_hi/lo, xor3)", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_PHX2>, 2048)), enc_bytes);
    row("encode max+min clamp", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_MED3>, 2048)), enc_bytes);
    row("encode max+min clamp g=16384", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_MED3>, 16384)), enc_bytes);
    row("encode NORNG|NODIV g=16384", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_ABL_NORNG | ENC_ABL_NODIV>, 16384)), enc_bytes);
    for (int rep = 0; rep < 3; ++rep) {
        row("A/B: encode product (MINW=1) g=2048", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, 0>, 2048)), enc_bytes);
        row("A/B: encode PF g=2048", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_PF>, 2048)), enc_bytes);
        row("A/B: encode PF g=1536", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_PF>, 1536)), enc_bytes);
        row("A/B: encode PF g=3072", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_PF>, 3072)), enc_bytes);
        row("A/B: encode PF MINW=4 g=2048", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_PF, 4>, 2048)), enc_bytes);
        row("A/B: encode planes in pairs", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_GRP2>, 2048)), enc_bytes);
        row("A/B: encode planes in triples", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_GRP3>, 2048)), enc_bytes);
        row("A/B: encode SEQ planes", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_SEQ>, 2048)), enc_bytes);
        row("A/B: encode SEQ planes >=6 waves", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_SEQ, 6>, 2048)), enc_bytes);
        row("A/B: encode SEQ planes >=8 waves", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_SEQ, 8>, 2048)), enc_bytes);
        row("A/B: encode SEQ planes >=8 waves g=4096", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_SEQ, 8>, 4096)), enc_bytes);
    }
    {
        // Infinity-Cache reuse inside one step: flush 600 MB, then time absmax -> encode
        uint4 *fl;
        CK(hipMalloc(&fl, 600ull << 20));
        CK(hipMemset(fl, 0, 600ull << 20));
        CK(hipDeviceSynchronize());
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        auto pair = [&](const char *nm, auto am, auto en) {
            float tot = 0;
            for (int i = 0; i < 12; ++i) {
                hipLaunchKernelGGL(k_flush, dim3(8192), dim3(256), 0, 0, fl, (600ull << 20) / 16);
                CK(hipEventRecord(a, 0));
                am();
                en();
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (i >= 2)
                    tot += ms;
            }
            row(nm, tot / 10, 8.0 * n + 4.0 * M);
        };
        auto am_fwd = [&] { gc_absmax_f32(x, nullptr, n, norm, ws, nullptr); };
        auto am_rev = [&] {
            CK(hipMemsetAsync(norm, 0, 4, 0));
            hipLaunchKernelGGL(k_absmax_rev, dim3(256), dim3(1024), 0, 0, (const float4 *)x, n / 4, (uint32_t *)norm);
        };
        for (int rep = 0; rep < 2; ++rep) {
            pair("COLD step: absmax fwd + encode fwd", am_fwd, enc(gclab::k_qsgd_encode<6, 0, 0, 0>, 2048));
            pair("COLD step: absmax fwd + encode REV", am_fwd, enc(gclab::k_qsgd_encode<6, 0, 0, ENC_REV>, 2048));
            pair("COLD step: absmax REV + encode fwd", am_rev, enc(gclab::k_qsgd_encode<6, 0, 0, 0>, 2048));
            pair("COLD step: absmax REV + encode REV", am_rev, enc(gclab::k_qsgd_encode<6, 0, 0, ENC_REV>, 2048));
        }
        pair("COLD encode only (after flush)", [] {}, enc(gclab::k_qsgd_encode<6, 0, 0, 0>, 2048));
        pair("COLD absmax only (after flush)", am_fwd, [] {});
        CK(hipFree(fl));
    }
    row("encode COMPUTE ONLY (16KB window) g=2048", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_ABL_L2>, 2048)), enc_bytes);
    row("encode COMPUTE ONLY g=8192", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_ABL_L2>, 8192)), enc_bytes);
    row("encode COMPUTE ONLY, no Philox", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_ABL_L2 | ENC_ABL_NORNG>, 2048)), enc_bytes);
    row("encode COMPUTE ONLY, no div", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_ABL_L2 | ENC_ABL_NODIV>, 2048)), enc_bytes);
    row("encode ABL=NORNG g=2048", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_ABL_NORNG>, 2048)), enc_bytes);
    row("encode ABL=NODIV g=2048", T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_ABL_NODIV>, 2048)), enc_bytes);
    row("encode ABL=NORNG|NODIV g=2048",
        T.run(enc(gclab::k_qsgd_encode<6, 0, 0, ENC_ABL_NORNG | ENC_ABL_NODIV>, 2048)), enc_bytes);

    // the same product rows again, late in the process (clock / power ramp check)
    row("late: product gc_qsgd_encode", T.run([&] { gc_qsgd_encode(x, nullptr, n, norm, bits, &ln, &rng, words, nullptr); }),
        enc_bytes);
    row("late: product absmax + encode (one step)", T.run([&] {
            gc_absmax_f32(x, nullptr, n, norm, ws, nullptr);
            gc_qsgd_encode(x, nullptr, n, norm, bits, &ln, &rng, words, nullptr);
        }), 8.0 * n + 4.0 * M);
    row("late: product absmax + encode x200", T.run([&] {
            gc_absmax_f32(x, nullptr, n, norm, ws, nullptr);
            gc_qsgd_encode(x, nullptr, n, norm, bits, &ln, &rng, words, nullptr);
        }, 200), 8.0 * n + 4.0 * M);

    {
        unsigned long long *st;
        uint32_t *ex;
        CK(hipMalloc(&st, 32));
        CK(hipMalloc(&ex, 16));
        for (int allones = 0; allones < 2; ++allones) {
            CK(hipMemset(st, 0, 32));
            const uint64_t cnt = allones ? 4000000000ull : 40000000000ull;
            hipLaunchKernelGGL(k_divcheck, dim3(8192), dim3(256), 0, 0, 7ull + allones, cnt, allones, st, ex);
            unsigned long long h[3];
            uint32_t e[2];
            CK(hipMemcpy(h, st, 24, hipMemcpyDeviceToHost));
            CK(hipMemcpy(e, ex, 8, hipMemcpyDeviceToHost));
            printf("divcheck%s: %llu pairs in range, Markstein mismatches %llu (e.g. a=%08x b=%08x), 2-step mismatches %llu\n",
                   allones ? " (norm significand all ones)" : "", h[0], h[1], h[1] ? e[0] : 0u, h[1] ? e[1] : 0u, h[2]);
        }
        CK(hipFree(st));
        CK(hipFree(ex));
    }
    {
        // settled, interleaved A/B: 0.5 s of steps first (clock ramp), then 7
        // rounds over all variants; report each variant's median
        auto settle = [&] {
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            float tot = 0;
            while (tot < 500.0f) {
                CK(hipEventRecord(a, 0));
                for (int i = 0; i < 100; ++i) {
                    gc_absmax_f32(x, nullptr, n, norm, ws, nullptr);
                    gc_qsgd_encode(x, nullptr, n, norm, bits, &ln, &rng, words, nullptr);
                }
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                tot += ms;
            }
        };
        struct V {
            const char *name;
            std::function<void()> f;
            double bytes;
            std::vector<float> t;
        };
        std::vector<V> vs;
        vs.push_back({"AB: encode product", enc(gclab::k_qsgd_encode<6, 0, 0, 0>, 2048), enc_bytes, {}});
        vs.push_back({"AB: encode DIV2 (two corrections)", enc(gclab::k_qsgd_encode<6, 0, 0, ENC_DIV2>, 2048), enc_bytes, {}});
        vs.push_back({"AB: encode NT loads", enc(gclab::k_qsgd_encode<6, 0, 0, ENC_NT>, 2048), enc_bytes, {}});
        vs.push_back({"AB: encode NT + DIV2", enc(gclab::k_qsgd_encode<6, 0, 0, ENC_DIV2 | ENC_NT>, 2048), enc_bytes, {}});
        vs.push_back({"AB: absmax product", [&] { gc_absmax_f32(x, nullptr, n, norm, ws, nullptr); }, rd_bytes, {}});
        vs.push_back({"AB: step product (absmax+encode)", [&] {
                          gc_absmax_f32(x, nullptr, n, norm, ws, nullptr);
                          enc(gclab::k_qsgd_encode<6, 0, 0, 0>, 2048)();
                      }, 8.0 * n + 4.0 * M, {}});
        vs.push_back({"AB: step absmax + encode DIV2", [&] {
                          gc_absmax_f32(x, nullptr, n, norm, ws, nullptr);
                          enc(gclab::k_qsgd_encode<6, 0, 0, ENC_DIV2>, 2048)();
                      }, 8.0 * n + 4.0 * M, {}});
        vs.push_back({"AB: step absmax + encode NT", [&] {
                          gc_absmax_f32(x, nullptr, n, norm, ws, nullptr);
                          enc(gclab::k_qsgd_encode<6, 0, 0, ENC_NT>, 2048)();
                      }, 8.0 * n + 4.0 * M, {}});
        settle();
        for (int rep = 0; rep < 7; ++rep)
            for (auto &v : vs)
                v.t.push_back(T.run(v.f, 50));
        for (auto &v : vs) {
            std::sort(v.t.begin(), v.t.end());
            row(v.name, v.t[v.t.size() / 2], v.bytes);
        }
    }
    // the lab's ABL=0 instantiation must equal the product's words
    hipLaunchKernelGGL((gclab::k_qsgd_encode<6, 0, 0, 0>), dim3(2048), dim3(256), 0, 0, x, (const int64_t *)nullptr, n, norm,
                       s, qmax, ln.bits, (uint64_t)M, ra, words2);
    gc_qsgd_encode(x, nullptr, n, norm, bits, &ln, &rng, words, nullptr);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> a(M), b(M);
    CK(hipMemcpy(a.data(), words, (size_t)M * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), words2, (size_t)M * 4, hipMemcpyDeviceToHost));
    printf("lab ABL=0 == product: %s\n", memcmp(a.data(), b.data(), (size_t)M * 4) == 0 ? "yes" : "NO");
    // exact variants (same outputs by construction) must agree bit for bit
    auto same = [&](const char *nm, auto kern) {
        CK(hipMemset(words2, 0, (size_t)M * 4));
        enc(kern, 2048)();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(b.data(), words2, (size_t)M * 4, hipMemcpyDeviceToHost));
        printf("%-28s == product: %s\n", nm, memcmp(a.data(), b.data(), (size_t)M * 4) == 0 ? "yes" : "NO");
    };
    same("philox impl 0", gclab::k_qsgd_encode<6, 0, 0, ENC_PHX0>);
    same("philox impl 2", gclab::k_qsgd_encode<6, 0, 0, ENC_PHX2>);
    same("max+min clamp", gclab::k_qsgd_encode<6, 0, 0, ENC_MED3>);
    same(">=8 waves/SIMD", gclab::k_qsgd_encode<6, 0, 0, 0, 8>);
    same("reverse tile order", gclab::k_qsgd_encode<6, 0, 0, ENC_REV>);
    same("planes in pairs", gclab::k_qsgd_encode<6, 0, 0, ENC_GRP2>);
    same("SEQ planes", gclab::k_qsgd_encode<6, 0, 0, ENC_SEQ>);
    same("SEQ planes >=8 waves", gclab::k_qsgd_encode<6, 0, 0, ENC_SEQ, 8>);
    same("register prefetch", gclab::k_qsgd_encode<6, 0, 0, ENC_PF>);
    same("register prefetch MINW=4", gclab::k_qsgd_encode<6, 0, 0, ENC_PF, 4>);
    same("two-correction division", gclab::k_qsgd_encode<6, 0, 0, ENC_DIV2>);
    same("nontemporal loads", gclab::k_qsgd_encode<6, 0, 0, ENC_NT>);
    return 0;
}
