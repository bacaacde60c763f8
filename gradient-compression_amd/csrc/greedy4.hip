// greedy4.hip — the reference's greedy 4-mode bit packer on the GPU
// (extensions/Extension CPU/bitpacking.cpp:5-124, identical to Extension
// GPU/gpu_bitpacking.cpp:5-125, which runs on the host despite its name).
//
// Format: 32-bit words, mode in bits 31:30; mode m packs CNT[m] values of
// BITS[m] bits MSB-first (15x2, 7x4, 4x7, 3x8).  At position i the mode is the
// first m whose window max(v[i .. i+CNT[m]) ∩ [0, n)) < LIM[m] (mode 3
// otherwise); the next word starts at i + CNT[mode].  Values must lie in
// [0, 255] (the reference corrupts negatives and loops forever on >= 256).
//
// The word starts form a chain next(i) = i + CNT[mode(i)] — list ranking, not
// a scan.  Three phases:
//   k_g4_chunk    per 2048-element chunk (LDS): modes, then pointer-doubling
//                 tables nxt_k = next^(2^k); for each of the 15 possible entry
//                 offsets (a word starting before the chunk ends at most 14
//                 into it) binary-lift to the chunk's exit offset and count
//                 the words -> a 15-state transition table per chunk.
//   k_g4_group / k_g4_walk / k_g4_spread
//                 compose the transitions of 256-chunk groups, walk the groups
//                 from offset 0 (one thread; groups are few), then each group
//                 walks its chunks: every chunk gets its entry offset and
//                 output word base.
//   k_g4_emit     per chunk: rebuild the tables, word j of the chunk starts at
//                 next^j(entry) (binary decomposition of j over the tables),
//                 pack it, store it at base + j.  Fully parallel.
// Unpack: per-word element counts -> block sums -> one-block scan -> emit.
#include "gc_device.h"
#include "gc_host.h"

#include <algorithm>

namespace gc {

constexpr int G4_CHUNK = 2048;                 // elements per chunk
constexpr int G4_HALO = 16;                    // >= 14 values past the chunk
constexpr int G4_LEVELS = 10;                  // 2^10 > max words per chunk (683)
constexpr int G4_TAB = G4_CHUNK + G4_HALO;     // table entries per level
constexpr int G4_GROUP = 256;                  // chunks per group
constexpr unsigned G4_THREADS = 256;
constexpr uint32_t G4_STATUS_RANGE = 1u, G4_STATUS_NOSPC = 2u;

__constant__ int c_g4_cnt[4] = {15, 7, 4, 3};
__constant__ int c_g4_bits[4] = {2, 4, 7, 8};
__constant__ int c_g4_top[4] = {28, 26, 23, 22};

struct G4Smem {
    uint8_t v[G4_CHUNK + 32];           // values (0-padded past n)
    uint16_t nxt[G4_LEVELS][G4_TAB];    // next^(2^k), local indices; >= len: absorbing
};

// load chunk values + halo, compute next (level 0) and the doubling levels.
// len = elements of the chunk that are < n.  Returns via smem.
__device__ void g4_build(G4Smem &sm, const int32_t *__restrict__ src, uint64_t n, uint64_t start, uint32_t len,
                         uint32_t *__restrict__ status)
{
    const unsigned tid = threadIdx.x;
    bool bad = false;
    for (uint32_t i = tid; i < G4_CHUNK + 32; i += G4_THREADS) {
        const uint64_t g = start + i;
        int32_t v = 0;
        if (g < n && i < G4_CHUNK + G4_HALO) {
            v = src[g];
            bad |= (uint32_t)v > 255u;
        }
        sm.v[i] = (uint8_t)v;
    }
    if (bad)
        atomicOr(status, G4_STATUS_RANGE);
    __syncthreads();
    // level 0: positions [0, G4_TAB); >= len absorbing
    for (uint32_t i = tid; i < (uint32_t)G4_TAB; i += G4_THREADS) {
        uint32_t nx = i;
        if (i < len) {
            uint32_t m15 = 0, m7 = 0, m4 = 0;
#pragma unroll
            for (int j = 0; j < 15; ++j) {
                const uint32_t v = sm.v[i + j];  // i + 14 < G4_CHUNK + 32
                m15 = max(m15, v);
                if (j < 7)
                    m7 = max(m7, v);
                if (j < 4)
                    m4 = max(m4, v);
            }
            const int mode = m15 < 4 ? 0 : (m7 < 16 ? 1 : (m4 < 128 ? 2 : 3));
            nx = i + (uint32_t)c_g4_cnt[mode];
        }
        sm.nxt[0][i] = (uint16_t)nx;
    }
    __syncthreads();
    for (int k = 1; k < G4_LEVELS; ++k) {
        for (uint32_t i = tid; i < (uint32_t)G4_TAB; i += G4_THREADS) {
            const uint32_t a = sm.nxt[k - 1][i];
            sm.nxt[k][i] = a < (uint32_t)G4_TAB ? sm.nxt[k - 1][a] : (uint16_t)a;
        }
        __syncthreads();
    }
}

// from local entry e (< 15): words until the chain leaves [0, len) and the
// exit offset past len.  (exit, words) packed as words << 8 | exit.
__device__ __forceinline__ uint32_t g4_lift(const G4Smem &sm, uint32_t e, uint32_t len)
{
    if (e >= len)
        return (e - len) & 0xffu;
    uint32_t pos = e, cnt = 0;
#pragma unroll
    for (int k = G4_LEVELS - 1; k >= 0; --k) {
        const uint32_t p2 = sm.nxt[k][pos];
        if (p2 < len) {
            pos = p2;
            cnt += 1u << k;
        }
    }
    pos = sm.nxt[0][pos];  // the step that leaves the chunk
    return ((cnt + 1) << 8) | ((pos - len) & 0xffu);
}

__global__ __launch_bounds__(G4_THREADS) void k_g4_chunk(const int32_t *__restrict__ src, uint64_t n,
                                                         uint32_t *__restrict__ trans, uint32_t *__restrict__ status)
{
    __shared__ G4Smem sm;
    const uint64_t c = blockIdx.x;
    const uint64_t start = c * G4_CHUNK;
    const uint32_t len = (uint32_t)std::min<uint64_t>(G4_CHUNK, n - start);
    g4_build(sm, src, n, start, len, status);
    if (threadIdx.x < 16)
        trans[c * 16 + threadIdx.x] = threadIdx.x < 15 ? g4_lift(sm, threadIdx.x, len) : 0u;
}

// compose the transitions of each group of G4_GROUP chunks (15 walkers)
__global__ __launch_bounds__(G4_THREADS) void k_g4_group(const uint32_t *__restrict__ trans, uint64_t chunks,
                                                         uint32_t *__restrict__ gtrans)
{
    __shared__ uint32_t t[G4_GROUP * 16];
    const uint64_t c0 = (uint64_t)blockIdx.x * G4_GROUP;
    const uint32_t cnt = (uint32_t)std::min<uint64_t>(G4_GROUP, chunks - c0);
    for (uint32_t i = threadIdx.x; i < cnt * 16; i += G4_THREADS)
        t[i] = trans[c0 * 16 + i];
    __syncthreads();
    if (threadIdx.x < 16) {
        uint32_t state = threadIdx.x, words = 0;
        if (threadIdx.x < 15) {
            for (uint32_t j = 0; j < cnt; ++j) {
                const uint32_t x = t[j * 16 + state];
                words += x >> 8;
                state = x & 0xffu;
            }
        }
        gtrans[(uint64_t)blockIdx.x * 16 + threadIdx.x] = (words << 8) | state;  // words <= 256*683 < 2^24
    }
}

// one block: walk the groups from offset 0; group entry + word base; total
__global__ __launch_bounds__(G4_THREADS) void k_g4_walk(const uint32_t *__restrict__ gtrans, uint64_t groups,
                                                        uint32_t *__restrict__ gentry, uint64_t *__restrict__ gbase,
                                                        uint64_t *__restrict__ nwords, uint64_t cap,
                                                        uint32_t *__restrict__ status)
{
    constexpr uint32_t TILE = 1024;
    __shared__ uint32_t t[TILE * 16];
    __shared__ uint32_t st_state;
    __shared__ uint64_t st_base;
    if (threadIdx.x == 0) {
        st_state = 0;
        st_base = 0;
    }
    for (uint64_t g0 = 0; g0 < groups; g0 += TILE) {
        const uint32_t cnt = (uint32_t)std::min<uint64_t>(TILE, groups - g0);
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < cnt * 16; i += G4_THREADS)
            t[i] = gtrans[g0 * 16 + i];
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t state = st_state;
            uint64_t base = st_base;
            for (uint32_t j = 0; j < cnt; ++j) {
                gentry[g0 + j] = state;
                gbase[g0 + j] = base;
                const uint32_t x = t[j * 16 + state];
                base += x >> 8;
                state = x & 0xffu;
            }
            st_state = state;
            st_base = base;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        *nwords = st_base;
        if (st_base > cap)
            atomicOr(status, G4_STATUS_NOSPC);
    }
}

// per group: walk its chunks from the group entry -> chunk entry + base
__global__ __launch_bounds__(G4_THREADS) void k_g4_spread(const uint32_t *__restrict__ trans, uint64_t chunks,
                                                          const uint32_t *__restrict__ gentry,
                                                          const uint64_t *__restrict__ gbase,
                                                          uint32_t *__restrict__ centry, uint64_t *__restrict__ cbase)
{
    __shared__ uint32_t t[G4_GROUP * 16];
    const uint64_t c0 = (uint64_t)blockIdx.x * G4_GROUP;
    const uint32_t cnt = (uint32_t)std::min<uint64_t>(G4_GROUP, chunks - c0);
    for (uint32_t i = threadIdx.x; i < cnt * 16; i += G4_THREADS)
        t[i] = trans[c0 * 16 + i];
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t state = gentry[blockIdx.x];
        uint64_t base = gbase[blockIdx.x];
        for (uint32_t j = 0; j < cnt; ++j) {
            centry[c0 + j] = state;
            cbase[c0 + j] = base;
            const uint32_t x = t[j * 16 + state];
            base += x >> 8;
            state = x & 0xffu;
        }
    }
}

__global__ __launch_bounds__(G4_THREADS) void k_g4_emit(const int32_t *__restrict__ src, uint64_t n,
                                                        const uint32_t *__restrict__ trans,
                                                        const uint32_t *__restrict__ centry,
                                                        const uint64_t *__restrict__ cbase, int32_t *__restrict__ out,
                                                        uint64_t cap, uint32_t *__restrict__ status)
{
    __shared__ G4Smem sm;
    const uint64_t c = blockIdx.x;
    const uint64_t start = c * G4_CHUNK;
    const uint32_t len = (uint32_t)std::min<uint64_t>(G4_CHUNK, n - start);
    g4_build(sm, src, n, start, len, status);
    const uint32_t entry = centry[c];
    const uint64_t base = cbase[c];
    const uint32_t words = trans[c * 16 + entry] >> 8;
    if (*status != 0)  // out-of-domain value or too small an output: write nothing
        return;
    for (uint32_t j = threadIdx.x; j < words; j += G4_THREADS) {
        uint32_t p = entry;
#pragma unroll
        for (int k = 0; k < G4_LEVELS; ++k)
            if ((j >> k) & 1u)
                p = sm.nxt[k][p];
        const uint32_t step = sm.nxt[0][p] - p;
        const int mode = step == 15 ? 0 : step == 7 ? 1 : step == 4 ? 2 : 3;
        uint32_t code = (uint32_t)mode << 30;
        const int top = c_g4_top[mode], b = c_g4_bits[mode];
        for (uint32_t q = 0; q < step; ++q)  // zero-padded past n: OR of 0
            code |= (uint32_t)sm.v[p + q] << (top - (int)q * b);
        if (base + j < cap)
            out[base + j] = (int32_t)code;
    }
}

// ---- unpack ---------------------------------------------------------------
constexpr uint32_t G4U_PER_THREAD = 16;
constexpr uint32_t G4U_BLOCK_WORDS = G4_THREADS * G4U_PER_THREAD;

__device__ __forceinline__ uint32_t g4_count(int32_t w) { return (uint32_t)c_g4_cnt[(uint32_t)w >> 30]; }

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *total)
{
    __shared__ uint32_t wsum[G4_THREADS / 64];
    const unsigned lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, o, 64);
        if (lane >= (unsigned)o)
            inc += y;
    }
    if (lane == 63)
        wsum[wv] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (unsigned i = 0; i < G4_THREADS / 64; ++i) {
        if (i < wv)
            off += wsum[i];
        tot += wsum[i];
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

__global__ void k_g4_init(uint64_t *count, uint32_t *status)
{
    *count = 0;
    *status = 0;
}

__global__ __launch_bounds__(G4_THREADS) void k_g4u_sums(const int32_t *__restrict__ words, uint64_t nw,
                                                         uint32_t *__restrict__ bsum)
{
    const uint64_t w0 = (uint64_t)blockIdx.x * G4U_BLOCK_WORDS + (uint64_t)threadIdx.x * G4U_PER_THREAD;
    uint32_t s = 0;
    for (uint32_t i = 0; i < G4U_PER_THREAD; ++i)
        if (w0 + i < nw)
            s += g4_count(words[w0 + i]);
    uint32_t tot;
    block_excl_scan(s, &tot);
    if (threadIdx.x == 0)
        bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(G4_THREADS) void k_g4u_scan(const uint32_t *__restrict__ bsum, uint64_t nb,
                                                         uint64_t *__restrict__ bbase, uint64_t *__restrict__ count,
                                                         uint64_t cap, uint32_t *__restrict__ status)
{
    __shared__ uint64_t carry;
    if (threadIdx.x == 0)
        carry = 0;
    __syncthreads();
    for (uint64_t b0 = 0; b0 < nb; b0 += G4_THREADS) {
        const uint64_t b = b0 + threadIdx.x;
        const uint32_t v = b < nb ? bsum[b] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_scan(v, &tot);
        const uint64_t c = carry;
        if (b < nb)
            bbase[b] = c + ex;
        __syncthreads();
        if (threadIdx.x == 0)
            carry = c + tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        *count = carry;
        if (carry > cap)
            atomicOr(status, G4_STATUS_NOSPC);
    }
}

__global__ __launch_bounds__(G4_THREADS) void k_g4u_emit(const int32_t *__restrict__ words, uint64_t nw,
                                                         const uint64_t *__restrict__ bbase, int32_t *__restrict__ out,
                                                         const uint32_t *__restrict__ status)
{
    if (*status != 0)
        return;
    const uint64_t w0 = (uint64_t)blockIdx.x * G4U_BLOCK_WORDS + (uint64_t)threadIdx.x * G4U_PER_THREAD;
    uint32_t s = 0;
    for (uint32_t i = 0; i < G4U_PER_THREAD; ++i)
        if (w0 + i < nw)
            s += g4_count(words[w0 + i]);
    uint32_t tot;
    uint64_t o = bbase[blockIdx.x] + block_excl_scan(s, &tot);
    for (uint32_t i = 0; i < G4U_PER_THREAD && w0 + i < nw; ++i) {
        const uint32_t code = (uint32_t)words[w0 + i];
        const int mode = (int)(code >> 30);
        const int cnt = c_g4_cnt[mode], top = c_g4_top[mode], b = c_g4_bits[mode];
        const uint32_t mask = (1u << b) - 1u;
        for (int j = 0; j < cnt; ++j)
            out[o + j] = (int32_t)((code >> (top - j * b)) & mask);
        o += (uint64_t)cnt;
    }
}

// workspace layout (bytes, 256-aligned pieces)
struct G4Ws {
    uint32_t *trans, *gtrans, *gentry, *centry;
    uint64_t *gbase, *cbase;
};

static inline uint64_t al256(uint64_t b) { return (b + 255) & ~255ull; }

static uint64_t g4_ws(uint64_t n, char *base, G4Ws *w)
{
    const uint64_t chunks = (n + G4_CHUNK - 1) / G4_CHUNK;
    const uint64_t groups = (chunks + G4_GROUP - 1) / G4_GROUP;
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) {
        char *p = base ? base + off : nullptr;
        off += al256(bytes);
        return p;
    };
    G4Ws t;
    t.trans = (uint32_t *)take(chunks * 64);
    t.gtrans = (uint32_t *)take(groups * 64);
    t.gentry = (uint32_t *)take(groups * 4);
    t.gbase = (uint64_t *)take(groups * 8);
    t.centry = (uint32_t *)take(chunks * 4);
    t.cbase = (uint64_t *)take(chunks * 8);
    if (w)
        *w = t;
    return off;
}

static uint64_t g4u_ws(uint64_t nw, char *base, G4Ws *w)
{
    const uint64_t nb = (nw + G4U_BLOCK_WORDS - 1) / G4U_BLOCK_WORDS;
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) {
        char *p = base ? base + off : nullptr;
        off += al256(bytes);
        return p;
    };
    G4Ws t{};
    t.trans = (uint32_t *)take(nb * 4);   // block sums
    t.gbase = (uint64_t *)take(nb * 8);   // block bases
    if (w)
        *w = t;
    return off;
}

}  // namespace gc

using namespace gc;

extern "C" {

size_t gc_greedy4_workspace_size(uint64_t n) { return (size_t)std::max<uint64_t>(g4_ws(n, nullptr, nullptr), 256); }

size_t gc_greedy4_unpack_workspace_size(uint64_t nwords)
{
    return (size_t)std::max<uint64_t>(g4u_ws(nwords, nullptr, nullptr), 256);
}

int gc_greedy4_pack_device(const int32_t *src, uint64_t n, int32_t *out, uint64_t cap, uint64_t *nwords,
                           uint32_t *status, void *workspace, gc_stream_t stream)
{
    GC_REQUIRE(workspace && nwords && status, "gc_greedy4_pack_device: null workspace / nwords / status");
    GC_REQUIRE(n == 0 || (src && out), "gc_greedy4_pack_device: null pointer");
    GC_REQUIRE(n < (1ull << 40), "gc_greedy4_pack_device: n too large");
    hipStream_t st = as_stream(stream);
    G4Ws w;
    g4_ws(n, reinterpret_cast<char *>(workspace), &w);
    hipLaunchKernelGGL(k_g4_init, dim3(1), dim3(1), 0, st, nwords, status);
    if (n == 0)
        return launch_status("gc_greedy4_pack_device");
    const uint64_t chunks = (n + G4_CHUNK - 1) / G4_CHUNK;
    const uint64_t groups = (chunks + G4_GROUP - 1) / G4_GROUP;
    hipLaunchKernelGGL(k_g4_chunk, dim3((unsigned)chunks), dim3(G4_THREADS), 0, st, src, n, w.trans, status);
    hipLaunchKernelGGL(k_g4_group, dim3((unsigned)groups), dim3(G4_THREADS), 0, st, w.trans, chunks, w.gtrans);
    hipLaunchKernelGGL(k_g4_walk, dim3(1), dim3(G4_THREADS), 0, st, w.gtrans, groups, w.gentry, w.gbase, nwords, cap,
                       status);
    hipLaunchKernelGGL(k_g4_spread, dim3((unsigned)groups), dim3(G4_THREADS), 0, st, w.trans, chunks, w.gentry,
                       w.gbase, w.centry, w.cbase);
    hipLaunchKernelGGL(k_g4_emit, dim3((unsigned)chunks), dim3(G4_THREADS), 0, st, src, n, w.trans, w.centry,
                       w.cbase, out, cap, status);
    return launch_status("gc_greedy4_pack_device");
}

int gc_greedy4_unpack_device(const int32_t *words, uint64_t nwords, int32_t *out, uint64_t cap, uint64_t *count,
                             uint32_t *status, void *workspace, gc_stream_t stream)
{
    GC_REQUIRE(workspace && count && status, "gc_greedy4_unpack_device: null workspace / count / status");
    GC_REQUIRE(nwords == 0 || (words && out), "gc_greedy4_unpack_device: null pointer");
    GC_REQUIRE(nwords < (1ull << 40), "gc_greedy4_unpack_device: too many words");
    hipStream_t st = as_stream(stream);
    G4Ws w;
    g4u_ws(nwords, reinterpret_cast<char *>(workspace), &w);
    hipLaunchKernelGGL(k_g4_init, dim3(1), dim3(1), 0, st, count, status);
    if (nwords == 0)
        return launch_status("gc_greedy4_unpack_device");
    const uint64_t nb = (nwords + G4U_BLOCK_WORDS - 1) / G4U_BLOCK_WORDS;
    hipLaunchKernelGGL(k_g4u_sums, dim3((unsigned)nb), dim3(G4_THREADS), 0, st, words, nwords, w.trans);
    hipLaunchKernelGGL(k_g4u_scan, dim3(1), dim3(G4_THREADS), 0, st, w.trans, nb, w.gbase, count, cap, status);
    hipLaunchKernelGGL(k_g4u_emit, dim3((unsigned)nb), dim3(G4_THREADS), 0, st, words, nwords, w.gbase, out, status);
    return launch_status("gc_greedy4_unpack_device");
}

}  // extern "C"
