// rng_packers.hip — the torch-CPU-generator stream and the reference-compatible
// packers.
//
//   k_mt19937_generate   MT19937 draws exactly as torch's CPU generator
//                        (at::mt19937, seeded by torch.manual_seed, seed.py:6-11)
//                        hands them to torch.bernoulli (compressors.py:310).
//                        Reference-parity mode: one workgroup walks the serial
//                        stream; each 624-word twist is three dependency-free
//                        phases (k<227, k<454, k<624) of LDS-resident state.
//   k_bytepack8 / k_byteunpack8   extensions/Extension CPU BP/bytepacking.cpp:6-64
//   gc_greedy4_pack/_unpack       extensions/Extension CPU/bitpacking.cpp:5-124
//                                 (host code: the format is sequential)
#include <string.h>

#include "gc_device.h"
#include "gc_host.h"

namespace gc {

constexpr int MT_N = 624;
constexpr int MT_M = 397;
constexpr int kMtThreads = 256;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y)
{
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t c)
{
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// s[k] = s[k+M] ^ twist(s[k], s[k+1]) for k in order 0..623 (in place):
// phase A k<227 reads only old words; phase B k<454 reads s[k-227] from A;
// phase C k<624 reads s[k-227] from B (and s[0] from A for k=623).
__device__ void mt_twist_block(uint32_t *s)
{
    const int tid = threadIdx.x;
    uint32_t v[3];
    // phase A
    for (int r = 0; r < 1; ++r) {
        int k = tid;
        v[0] = 0;
        if (k < MT_N - MT_M)
            v[0] = mt_mix(s[k], s[k + 1], s[k + MT_M]);
    }
    __syncthreads();
    if (tid < MT_N - MT_M)
        s[tid] = v[0];
    __syncthreads();
    // phase B: k = 227 + tid, tid < 227
    {
        const int k = MT_N - MT_M + tid;
        if (tid < MT_N - MT_M)
            v[1] = mt_mix(s[k], s[k + 1], s[k - (MT_N - MT_M)]);
    }
    __syncthreads();
    if (tid < MT_N - MT_M)
        s[MT_N - MT_M + tid] = v[1];
    __syncthreads();
    // phase C: k = 454 + tid, tid < 170
    {
        const int k = 2 * (MT_N - MT_M) + tid;
        if (k < MT_N - 1)
            v[2] = mt_mix(s[k], s[k + 1], s[k - (MT_N - MT_M)]);
        else if (k == MT_N - 1)
            v[2] = mt_mix(s[k], s[0], s[MT_M - 1]);
    }
    __syncthreads();
    if (2 * (MT_N - MT_M) + tid < MT_N)
        s[2 * (MT_N - MT_M) + tid] = v[2];
    __syncthreads();
}

__global__ __launch_bounds__(kMtThreads) void k_mt19937_generate(uint32_t *__restrict__ state,
                                                                 uint32_t *__restrict__ out, uint64_t count)
{
    __shared__ uint32_t s[MT_N];
    for (int i = threadIdx.x; i < MT_N; i += kMtThreads)
        s[i] = state[i];
    uint32_t idx = state[MT_N];
    __syncthreads();
    uint64_t done = 0;
    while (done < count) {
        if (idx >= (uint32_t)MT_N) {
            mt_twist_block(s);
            idx = 0;
        }
        const uint64_t left = count - done;
        const uint32_t take = (uint32_t)min((uint64_t)(MT_N - idx), left);
        for (uint32_t j = threadIdx.x; j < take; j += kMtThreads)
            out[done + j] = mt_temper(s[idx + j]);
        done += take;
        idx += take;
        __syncthreads();  // all reads of s done before the next twist
    }
    for (int i = threadIdx.x; i < MT_N; i += kMtThreads)
        state[i] = s[i];
    if (threadIdx.x == 0)
        state[MT_N] = idx;
}

// ---------------------------------------------------------------------------
// byte packer: word w = sum_j (src[8w+j] & 0xFF) << 8*(7-j); last word zero-padded
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kBlock) void k_bytepack8(const T *__restrict__ src, uint64_t n, int64_t *__restrict__ out)
{
    const uint64_t nw = (n + 7) >> 3;
    for (uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * kBlock) {
        uint64_t code = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint64_t i = w * 8 + j;
            if (i < n)
                code |= ((uint64_t)(int64_t)src[i] & 0xffull) << (8 * (7 - j));
        }
        out[w] = (int64_t)code;
    }
}

__global__ __launch_bounds__(kBlock) void k_byteunpack8(const int64_t *__restrict__ src, uint64_t nw,
                                                        int8_t *__restrict__ out)
{
    for (uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * kBlock) {
        const uint64_t code = (uint64_t)src[w];
        // byte j of the output = bits 63-8j..56-8j: a byte swap of the word
        const uint64_t le = __builtin_bswap64(code);
        *reinterpret_cast<uint64_t *>(out + 8 * w) = le;
    }
}

// the big-endian byte word of 4 values' low bytes: v0 in bits 31:24 .. v3 in 7:0
__device__ __forceinline__ uint32_t be_bytes4(uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3)
{
    const uint32_t lo = __builtin_amdgcn_perm(v2, v3, 0x0c0c0400u);  // [v3.b0 v2.b0 0 0] (low to high)
    const uint32_t hi = __builtin_amdgcn_perm(v0, v1, 0x0c0c0400u);  // [v1.b0 v0.b0 0 0]
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);               // [v3 v2 v1 v0] = v0 << 24 | ...
}

// 16-byte vector forms (src and out 16-byte aligned): a thread packs 16
// values into two words with one 16-byte store; int8 sources are one 16-byte
// load + two byte swaps.  The last partial group goes through the scalar code.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_bytepack8_v(const T *__restrict__ src, uint64_t n,
                                                        int64_t *__restrict__ out)
{
    const uint64_t groups = n >> 4;  // full 16-value groups
    for (uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x; p <= groups; p += (uint64_t)gridDim.x * kBlock) {
        if (p == groups) {  // the tail: words 2p and 2p+1 if they hold values
            for (uint64_t w = 2 * p; w < (n + 7) >> 3; ++w) {
                uint64_t code = 0;
                for (int j = 0; j < 8; ++j)
                    if (w * 8 + j < n)
                        code |= ((uint64_t)(int64_t)src[w * 8 + j] & 0xffull) << (8 * (7 - j));
                out[w] = (int64_t)code;
            }
            continue;
        }
        uint32_t h[4];  // big-endian 4-byte pieces: words 2p = h0:h1, 2p+1 = h2:h3 (high half first)
        if constexpr (sizeof(T) == 1) {
            const uint4 v = *reinterpret_cast<const uint4 *>(src + 16 * p);
            h[0] = __builtin_bswap32(v.x);
            h[1] = __builtin_bswap32(v.y);
            h[2] = __builtin_bswap32(v.z);
            h[3] = __builtin_bswap32(v.w);
        } else if constexpr (sizeof(T) == 4) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 v = *reinterpret_cast<const uint4 *>(src + 16 * p + 4 * k);
                h[k] = be_bytes4(v.x, v.y, v.z, v.w);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int64_t *q = reinterpret_cast<const int64_t *>(src) + 16 * p + 4 * k;
                const ulonglong2 a = *reinterpret_cast<const ulonglong2 *>(q);
                const ulonglong2 b = *reinterpret_cast<const ulonglong2 *>(q + 2);
                h[k] = be_bytes4((uint32_t)a.x, (uint32_t)a.y, (uint32_t)b.x, (uint32_t)b.y);
            }
        }
        // int64 word = h_hi << 32 | h_lo; little-endian dwords: (lo, hi)
        *reinterpret_cast<uint4 *>(out + 2 * p) = make_uint4(h[1], h[0], h[3], h[2]);
    }
}

// 16 bytes per thread: two words -> one 16-byte store
__global__ __launch_bounds__(kBlock) void k_byteunpack8_v(const int64_t *__restrict__ src, uint64_t nw,
                                                          int8_t *__restrict__ out)
{
    const uint64_t pairs = nw >> 1;
    for (uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x; p <= pairs; p += (uint64_t)gridDim.x * kBlock) {
        if (p == pairs) {
            if (nw & 1)
                *reinterpret_cast<uint64_t *>(out + 8 * (nw - 1)) = __builtin_bswap64((uint64_t)src[nw - 1]);
            continue;
        }
        const uint4 v = *reinterpret_cast<const uint4 *>(src + 2 * p);  // (lo0, hi0, lo1, hi1)
        *reinterpret_cast<uint4 *>(out + 16 * p) =
            make_uint4(__builtin_bswap32(v.y), __builtin_bswap32(v.x), __builtin_bswap32(v.w), __builtin_bswap32(v.z));
    }
}

// QSGDBP decompress (compressors.py:375-376): out = (c * sgn) * float(xi),
// sgn = -1 where the unpacked sign bit is 1, else +1 — c * (+-1) is exact, so
// one rounding, as the reference's fp32 tensor ops give (a negative x that
// rounded to 0 decodes to -0.0).  Four elements per thread, 16-byte accesses.
__global__ __launch_bounds__(kBlock) void k_qsgdbp_decode(const int32_t *__restrict__ sign, const int32_t *__restrict__ xi,
                                                          uint64_t n, const float *__restrict__ cp, float *__restrict__ out)
{
    const float c = *cp, nc = -c;
    const uint64_t quads = n >> 2;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t <= quads; t += (uint64_t)gridDim.x * kBlock) {
        if (t == quads) {  // the n % 4 tail
            for (uint64_t i = 4 * quads; i < n; ++i)
                out[i] = (sign[i] == 1 ? nc : c) * (float)xi[i];
            continue;
        }
        const int4 s = *reinterpret_cast<const int4 *>(sign + 4 * t);
        const int4 q = *reinterpret_cast<const int4 *>(xi + 4 * t);
        *reinterpret_cast<float4 *>(out + 4 * t) =
            make_float4((s.x == 1 ? nc : c) * (float)q.x, (s.y == 1 ? nc : c) * (float)q.y,
                        (s.z == 1 ? nc : c) * (float)q.z, (s.w == 1 ? nc : c) * (float)q.w);
    }
}

}  // namespace gc

using namespace gc;

extern "C" {

int gc_qsgdbp_decode(const int32_t *sign, const int32_t *xi, uint64_t n, const float *c, float *out,
                     gc_stream_t stream)
{
    GC_REQUIRE(n == 0 || (sign && xi && c && out), "gc_qsgdbp_decode: null pointer");
    GC_REQUIRE(aligned16(sign) && aligned16(xi) && aligned16(out), "gc_qsgdbp_decode: buffers must be 16-byte aligned");
    if (n == 0)
        return GC_OK;
    hipLaunchKernelGGL(k_qsgdbp_decode, dim3(grid_for((n >> 2) + 1)), dim3(kBlock), 0, as_stream(stream), sign, xi, n, c,
                       out);
    return launch_status("gc_qsgdbp_decode");
}

int gc_mt19937_seed(uint64_t seed, uint32_t *state)
{
    GC_REQUIRE(state, "gc_mt19937_seed: null state");
    state[0] = (uint32_t)(seed & 0xffffffffu);
    for (uint32_t i = 1; i < (uint32_t)MT_N; ++i)
        state[i] = 1812433253u * (state[i - 1] ^ (state[i - 1] >> 30)) + i;
    state[MT_N] = MT_N;
    return GC_OK;
}

int gc_mt19937_generate(uint32_t *state_dev, uint32_t *out, uint64_t count, gc_stream_t stream)
{
    GC_REQUIRE(state_dev, "gc_mt19937_generate: null state");
    GC_REQUIRE(count == 0 || out, "gc_mt19937_generate: null out");
    hipLaunchKernelGGL(k_mt19937_generate, dim3(1), dim3(kMtThreads), 0, as_stream(stream), state_dev, out, count);
    return launch_status("gc_mt19937_generate");
}

int gc_bytepack8(const void *src, uint32_t src_dtype, uint64_t n, int64_t *out, gc_stream_t stream)
{
    GC_REQUIRE(src_dtype == GC_I8 || src_dtype == GC_I32 || src_dtype == GC_I64,
               "gc_bytepack8: src_dtype must be GC_I8, GC_I32 or GC_I64");
    GC_REQUIRE(n == 0 || (src && out), "gc_bytepack8: null pointer");
    if (n == 0)
        return GC_OK;
    hipStream_t st = as_stream(stream);
    if (aligned16(src) && aligned16(out)) {  // the 16-byte vector kernels
        const unsigned g = grid_for((n >> 4) + 1);
        if (src_dtype == GC_I8)
            hipLaunchKernelGGL((k_bytepack8_v<int8_t>), dim3(g), dim3(kBlock), 0, st,
                               reinterpret_cast<const int8_t *>(src), n, out);
        else if (src_dtype == GC_I32)
            hipLaunchKernelGGL((k_bytepack8_v<int32_t>), dim3(g), dim3(kBlock), 0, st,
                               reinterpret_cast<const int32_t *>(src), n, out);
        else
            hipLaunchKernelGGL((k_bytepack8_v<int64_t>), dim3(g), dim3(kBlock), 0, st,
                               reinterpret_cast<const int64_t *>(src), n, out);
        return launch_status("gc_bytepack8");
    }
    const unsigned grid = grid_for((n + 7) >> 3);
    if (src_dtype == GC_I8)
        hipLaunchKernelGGL((k_bytepack8<int8_t>), dim3(grid), dim3(kBlock), 0, st,
                           reinterpret_cast<const int8_t *>(src), n, out);
    else if (src_dtype == GC_I32)
        hipLaunchKernelGGL((k_bytepack8<int32_t>), dim3(grid), dim3(kBlock), 0, st,
                           reinterpret_cast<const int32_t *>(src), n, out);
    else
        hipLaunchKernelGGL((k_bytepack8<int64_t>), dim3(grid), dim3(kBlock), 0, st,
                           reinterpret_cast<const int64_t *>(src), n, out);
    return launch_status("gc_bytepack8");
}

int gc_byteunpack8(const int64_t *src, uint64_t nwords, int8_t *out, gc_stream_t stream)
{
    GC_REQUIRE(nwords == 0 || (src && out), "gc_byteunpack8: null pointer");
    GC_REQUIRE(aligned16(out) || (reinterpret_cast<uintptr_t>(out) & 7u) == 0, "gc_byteunpack8: out must be 8-byte aligned");
    if (nwords == 0)
        return GC_OK;
    if (aligned16(src) && aligned16(out))
        hipLaunchKernelGGL(k_byteunpack8_v, dim3(grid_for((nwords >> 1) + 1)), dim3(kBlock), 0, as_stream(stream), src,
                           nwords, out);
    else
        hipLaunchKernelGGL(k_byteunpack8, dim3(grid_for(nwords)), dim3(kBlock), 0, as_stream(stream), src, nwords,
                           out);
    return launch_status("gc_byteunpack8");
}

// host forms of the byte packer (the reference's "Extension CPU BP" is a CPU op)
int gc_bytepack8_host(const int64_t *src, uint64_t n, int64_t *out)
{
    if (n && (!src || !out))
        return fail(GC_EINVAL, "gc_bytepack8_host: null pointer");
    for (uint64_t w = 0; w < (n + 7) / 8; ++w) {
        uint64_t code = 0;
        for (int j = 0; j < 8 && w * 8 + j < n; ++j)
            code |= ((uint64_t)src[w * 8 + j] & 0xffull) << (8 * (7 - j));
        out[w] = (int64_t)code;
    }
    return GC_OK;
}

int gc_byteunpack8_host(const int64_t *src, uint64_t nwords, int8_t *out)
{
    if (nwords && (!src || !out))
        return fail(GC_EINVAL, "gc_byteunpack8_host: null pointer");
    for (uint64_t w = 0; w < nwords; ++w)
        for (int j = 0; j < 8; ++j)
            out[8 * w + j] = (int8_t)(((uint64_t)src[w] >> (8 * (7 - j))) & 0xffu);
    return GC_OK;
}

// Greedy 4-mode packer (host).  Modes by the max of the next 15/7/4/3
// values: 15 x 2 bit (<4), 7 x 4 bit (<16), 4 x 7 bit (<128), 3 x 8 bit
// (<256); MSB-first fields below a 2-bit mode tag.  The reference never
// terminates on a value >= 256 and corrupts the tag on negatives; here both
// return GC_ERANGE before writing.
static const int kG4Count[4] = {15, 7, 4, 3};
static const int kG4Bits[4] = {2, 4, 7, 8};
static const int kG4Top[4] = {28, 26, 23, 22};

int64_t gc_greedy4_pack(const int32_t *src, uint64_t n, int32_t *out, uint64_t cap)
{
    if (n && (!src || !out))
        return fail(GC_EINVAL, "gc_greedy4_pack: null pointer");
    for (uint64_t i = 0; i < n; ++i)
        if (src[i] < 0 || src[i] > 255)
            return fail(GC_ERANGE, "gc_greedy4_pack: value %d at %llu outside [0, 255]", src[i],
                        (unsigned long long)i);
    uint64_t ind = 0, nw = 0;
    while (ind < n) {
        // running max over the 15-window gives all four window maxima at once
        int32_t mx15 = 0, mx7 = 0, mx4 = 0, mx3 = 0;
        for (uint64_t j = 0; j < 15 && ind + j < n; ++j) {
            const int32_t v = src[ind + j];
            mx15 = v > mx15 ? v : mx15;
            if (j < 7) mx7 = v > mx7 ? v : mx7;
            if (j < 4) mx4 = v > mx4 ? v : mx4;
            if (j < 3) mx3 = v > mx3 ? v : mx3;
        }
        const int mode = mx15 < 4 ? 0 : (mx7 < 16 ? 1 : (mx4 < 128 ? 2 : 3));
        (void)mx3;
        uint32_t code = (uint32_t)mode << 30;
        for (int j = 0; j < kG4Count[mode] && ind + (uint64_t)j < n; ++j)
            code |= (uint32_t)src[ind + j] << (kG4Top[mode] - j * kG4Bits[mode]);
        if (nw >= cap)
            return fail(GC_ENOSPC, "gc_greedy4_pack: output capacity %llu too small", (unsigned long long)cap);
        out[nw++] = (int32_t)code;
        ind += (uint64_t)kG4Count[mode];
    }
    return (int64_t)nw;
}

int64_t gc_greedy4_unpack(const int32_t *src, uint64_t nwords, int32_t *out, uint64_t cap)
{
    if (nwords && (!src || !out))
        return fail(GC_EINVAL, "gc_greedy4_unpack: null pointer");
    uint64_t cnt = 0;
    for (uint64_t w = 0; w < nwords; ++w) {
        const uint32_t code = (uint32_t)src[w];
        const int mode = (int)(code >> 30);
        const uint32_t mask = (1u << kG4Bits[mode]) - 1u;
        if (cnt + (uint64_t)kG4Count[mode] > cap)
            return fail(GC_ENOSPC, "gc_greedy4_unpack: output capacity %llu too small", (unsigned long long)cap);
        for (int j = 0; j < kG4Count[mode]; ++j)
            out[cnt++] = (int32_t)((code >> (kG4Top[mode] - j * kG4Bits[mode])) & mask);
    }
    return (int64_t)cnt;
}

}  // extern "C"
