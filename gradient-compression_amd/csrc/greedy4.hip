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
// The word starts form a chain next(i) = i + CNT[mode(i)] from i = 0: a scan
// whose elements are FUNCTIONS.  Cut the positions into segments of 32; a
// word that starts in one segment ends at most 14 positions into the next, so
// a segment maps the offset its first word starts at (0..14, or 15 = past n)
// to the offset its chain leaves at and the words it emitted: a 16-entry
// table, and tables compose associatively.
//   k_g4p_tile     per 8192-element tile (256 threads x one segment): window
//                  flags by SWAR byte tests, the segment table by a backward
//                  recurrence held in registers (static indices only), then a
//                  reduction tree of the 256 tables in LDS -> the tile's
//                  table.  Also stores the values as bytes for the emit.
//   k_g4p_group    per 256 tiles: reduction tree -> the group's table
//   k_g4p_top      one block: walks the group tables from offset 0 (LDS) ->
//                  each group's entry offset and word base; the total
//   k_g4p_spread   per group: the tree again, then a down-sweep from the
//                  group's entry -> every tile's entry offset and word base
//   k_g4p_emit     per tile: the tile's tree again (from the bytes), a
//                  down-sweep from its entry -> every segment's entry and
//                  base; each thread packs its segment's words into LDS, the
//                  block stores the tile's words coalesced.
// HBM: src read once (4n), the bytes written and read (2n), the words written.
// Unpack: per-word element counts -> block sums -> one-block scan -> decode
// into LDS -> coalesced stores.
#include "gc_device.h"
#include "gc_host.h"

#include <algorithm>

namespace gc {

constexpr unsigned G4_THREADS = 256;
constexpr uint32_t G4_SEG = 32;                         // positions per segment (one thread)
constexpr uint32_t G4_TILE = G4_SEG * G4_THREADS;       // 8192 positions per tile
constexpr uint32_t G4_GROUP = 256;                      // tiles per group
constexpr uint32_t G4_DEAD = 15;                        // table state: the chain has passed n
constexpr uint32_t G4_TOP_CHUNK = 64;                   // group tables staged in LDS per top step
constexpr uint32_t G4_STATUS_RANGE = 1u, G4_STATUS_NOSPC = 2u;

// per-mode constants as nibble / byte tables in an immediate (a per-lane mode
// index into __constant__ arrays became vector memory loads in the emit loops)
__device__ __forceinline__ uint32_t g4_cnt(uint32_t m) { return (0x347fu >> (4 * m)) & 15u; }   // 15 7 4 3
__device__ __forceinline__ uint32_t g4_bits(uint32_t m) { return (0x8742u >> (4 * m)) & 15u; }  // 2 4 7 8
__device__ __forceinline__ uint32_t g4_top(uint32_t m) { return (0x16171a1cu >> (8 * m)) & 0xffu; }  // 28 26 23 22

// 4 byte-threshold flags of one dword (bytes b0..b3): bit j set iff byte j has
// a bit of `hi` set (hi = ~(lim - 1) for a power-of-two limit)
__device__ __forceinline__ uint32_t byte_flags(uint32_t w, uint32_t hi)
{
    const uint32_t x = w & hi;
    const uint32_t y = ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x;  // byte's top bit set iff byte != 0
    return ((y & 0x80808080u) * 0x00204081u) >> 28;           // gather the 4 top bits
}

// table entries: exit offset (4 bits) | words << 4

struct G4Tile {
    uint32_t v[(G4_TILE + 32) / 4];  // values as bytes (0 past n), 32-byte halo
    uint16_t node[2 * G4_THREADS][16];  // reduction tree: leaves 256..511, root 1
};

// modes of this thread's G4_SEG positions (2 bits each) from the LDS bytes,
// and its segment table (entries 0..14, exit | words << 4) by the backward
// recurrence f[p] = 1 word + f[p + cnt(p)], where a successor past the
// segment is its offset there, p + cnt - G4_SEG (0..14).  All indices are
// static (the recurrence is unrolled), so f stays in registers.
// seg0 = global position of the segment, n = bucket size.
__device__ __forceinline__ void g4_segment(const G4Tile &sm, uint64_t seg0, uint64_t n, uint64_t &modes,
                                           uint32_t f[G4_SEG])
{
    constexpr int DW = G4_SEG / 4 + 4;  // the segment's dwords + 16 bytes of the next (windows reach +14)
    const unsigned t = threadIdx.x;
    uint32_t w[DW];
#pragma unroll
    for (int k = 0; k < DW; k += 4)
        *reinterpret_cast<uint4 *>(&w[k]) = *reinterpret_cast<const uint4 *>(&sm.v[(G4_SEG / 4) * t + k]);
    uint64_t ge4 = 0, ge16 = 0, ge128 = 0;  // bit j: byte j (position seg0 + j)
#pragma unroll
    for (int k = 0; k < DW; ++k) {
        ge4 |= (uint64_t)byte_flags(w[k], 0xfcfcfcfcu) << (4 * k);
        ge16 |= (uint64_t)byte_flags(w[k], 0xf0f0f0f0u) << (4 * k);
        ge128 |= (uint64_t)byte_flags(w[k], 0x80808080u) << (4 * k);
    }
    modes = 0;
    const uint32_t live = seg0 >= n ? 0u : (uint32_t)std::min<uint64_t>(G4_SEG, n - seg0);  // positions < n
#pragma unroll
    for (int p = G4_SEG - 1; p >= 0; --p) {
        const uint32_t m = ((ge4 >> p) & 0x7fffu) == 0 ? 0u : ((ge16 >> p) & 0x7fu) == 0 ? 1u
                                                             : ((ge128 >> p) & 0xfu) == 0 ? 2u : 3u;
        modes |= (uint64_t)m << (2 * p);
        // the four possible successors (static indices)
        const uint32_t s3 = p + 3 < (int)G4_SEG ? f[(p + 3) % G4_SEG] : (uint32_t)(p + 3 - (int)G4_SEG);
        const uint32_t s4 = p + 4 < (int)G4_SEG ? f[(p + 4) % G4_SEG] : (uint32_t)(p + 4 - (int)G4_SEG);
        const uint32_t s7 = p + 7 < (int)G4_SEG ? f[(p + 7) % G4_SEG] : (uint32_t)(p + 7 - (int)G4_SEG);
        const uint32_t s15 = p + 15 < (int)G4_SEG ? f[(p + 15) % G4_SEG] : (uint32_t)(p + 15 - (int)G4_SEG);
        const uint32_t nx = m == 0 ? s15 : m == 1 ? s7 : m == 2 ? s4 : s3;
        f[p] = (uint32_t)p < live ? nx + 16u : G4_DEAD;
    }
}

// one tree level: nodes lvl .. 2 lvl - 1, node i = left child then right
// child.  A thread per (node, entry) pair, so 16 consecutive lanes read one
// node's row (conflict-free; a thread per node put 16 lanes on one bank);
// every pair's two lookups are issued before any store (the rows written
// are never read on the same level)
template <typename T, uint32_t NT>
__device__ __forceinline__ void g4_level(T (*node)[16], uint32_t lvl)
{
    constexpr uint32_t R = 8;  // pairs per thread on the widest level (128 nodes x 16 / 256)
    const uint32_t items = lvl * 16, t = threadIdx.x;
    uint32_t res[R];
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t k = t + r * NT;
        if (k < items) {
            const uint32_t i = lvl + (k >> 4), e = k & 15u;
            const uint32_t x = node[2 * i][e], y = node[2 * i + 1][x & 15u];
            res[r] = (y & 15u) | (((x >> 4) + (y >> 4)) << 4);
        }
    }
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t k = t + r * NT;
        if (k < items)
            node[lvl + (k >> 4)][k & 15u] = (T)res[r];
    }
}

// reduction tree over the 256 leaves node[256 + t] -> node[1]
__device__ __forceinline__ void g4_tree_up(G4Tile &sm)
{
#pragma unroll 1
    for (uint32_t lvl = G4_THREADS / 2; lvl >= 1; lvl >>= 1) {
        __syncthreads();
        g4_level<uint16_t, G4_THREADS>(sm.node, lvl);
    }
    __syncthreads();
}

// load tile `tile` of the values into LDS as bytes (0 past n) + halo.
// From int32 src (range-checked; the bytes also go to vb) or from vb.
template <bool FROM_SRC, bool ALIGNED>
__device__ __forceinline__ void g4_load(G4Tile &sm, const int32_t *__restrict__ src, uint8_t *__restrict__ vb,
                                        uint64_t n, uint64_t start, uint32_t *__restrict__ status)
{
    const unsigned t = threadIdx.x;
    bool bad = false;
#pragma unroll
    for (uint32_t j = 0; j < G4_TILE / (4 * G4_THREADS) + 1; ++j) {
        const uint32_t q = j * G4_THREADS + t;  // dword (4 positions) of the tile
        if (q >= (G4_TILE + 32) / 4)
            break;
        const uint64_t g = start + 4ull * q;
        uint32_t packed = 0;
        if (FROM_SRC) {
            int4 v = make_int4(0, 0, 0, 0);
            if (g + 4 <= n) {
                if (ALIGNED)
                    v = *reinterpret_cast<const int4 *>(src + g);
                else
                    v = make_int4(src[g], src[g + 1], src[g + 2], src[g + 3]);
            } else if (g < n) {
                v.x = src[g];
                v.y = g + 1 < n ? src[g + 1] : 0;
                v.z = g + 2 < n ? src[g + 2] : 0;
            }
            bad |= ((uint32_t)v.x | (uint32_t)v.y | (uint32_t)v.z | (uint32_t)v.w) > 255u;
            packed = ((uint32_t)v.x & 0xffu) | (((uint32_t)v.y & 0xffu) << 8) | (((uint32_t)v.z & 0xffu) << 16) |
                     ((uint32_t)v.w << 24);
            if (q < G4_TILE / 4 && g < n)
                *reinterpret_cast<uint32_t *>(vb + g) = packed;  // vb is padded to whole dwords
        } else if (g < n) {
            packed = *reinterpret_cast<const uint32_t *>(vb + g);  // zero past n (written so by k_g4p_tile)
        }
        sm.v[q] = packed;
    }
    if (FROM_SRC && bad)
        atomicOr(status, G4_STATUS_RANGE);
    __syncthreads();
}

template <bool ALIGNED>
__global__ __launch_bounds__(G4_THREADS) void k_g4p_tile(const int32_t *__restrict__ src, uint64_t n,
                                                         uint8_t *__restrict__ vb, uint32_t *__restrict__ agg,
                                                         uint32_t *__restrict__ status)
{
    __shared__ G4Tile sm;
    const uint64_t start = (uint64_t)blockIdx.x * G4_TILE;
    g4_load<true, ALIGNED>(sm, src, vb, n, start, status);
    uint64_t modes;
    uint32_t f[G4_SEG];
    g4_segment(sm, start + G4_SEG * threadIdx.x, n, modes, f);
    (void)modes;
#pragma unroll
    for (int e = 0; e < 16; ++e)
        sm.node[G4_THREADS + threadIdx.x][e] = (uint16_t)(e == 15 ? G4_DEAD : f[e]);
    g4_tree_up(sm);
    if (threadIdx.x < 16)
        agg[(uint64_t)blockIdx.x * 16 + threadIdx.x] = sm.node[1][threadIdx.x];
}

// tables of up to 256 items (16 x u32 each) in LDS: up-sweep to node[1]
struct G4Group {
    uint32_t node[2 * G4_GROUP][16];
    uint32_t st[2 * G4_GROUP];
    uint64_t bs[2 * G4_GROUP];
};

__device__ __forceinline__ void g4_group_up(G4Group &sm, const uint32_t *__restrict__ items, uint64_t first,
                                            uint32_t cnt)
{
    const unsigned t = threadIdx.x;
    for (uint32_t k = t; k < G4_GROUP * 16; k += G4_THREADS) {  // leaves; past the end: identity (dead = 15)
        const uint32_t i = k >> 4, e = k & 15u;
        sm.node[G4_GROUP + i][e] = i < cnt ? items[(first + i) * 16 + e] : e;
    }
#pragma unroll 1
    for (uint32_t lvl = G4_GROUP / 2; lvl >= 1; lvl >>= 1) {
        __syncthreads();
        g4_level<uint32_t, G4_THREADS>(sm.node, lvl);
    }
    __syncthreads();
}

__global__ __launch_bounds__(G4_THREADS) void k_g4p_group(const uint32_t *__restrict__ agg, uint64_t tiles,
                                                          uint32_t *__restrict__ gagg)
{
    __shared__ G4Group sm;
    const uint64_t first = (uint64_t)blockIdx.x * G4_GROUP;
    g4_group_up(sm, agg, first, (uint32_t)std::min<uint64_t>(G4_GROUP, tiles - first));
    if (threadIdx.x < 16)
        gagg[(uint64_t)blockIdx.x * 16 + threadIdx.x] = sm.node[1][threadIdx.x];
}

// one block: the chain through the groups from offset 0 -> entries, bases, total
__global__ __launch_bounds__(G4_THREADS) void k_g4p_top(const uint32_t *__restrict__ gagg, uint64_t groups,
                                                        uint32_t *__restrict__ gentry, uint64_t *__restrict__ gbase,
                                                        uint64_t *__restrict__ nwords, uint64_t cap,
                                                        uint32_t *__restrict__ status)
{
    __shared__ uint32_t t16[G4_TOP_CHUNK * 16];
    uint32_t state = 0;
    uint64_t base = 0;
    for (uint64_t g0 = 0; g0 < groups; g0 += G4_TOP_CHUNK) {
        const uint32_t cnt = (uint32_t)std::min<uint64_t>(G4_TOP_CHUNK, groups - g0);
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < cnt * 16; k += G4_THREADS)
            t16[k] = gagg[g0 * 16 + k];
        __syncthreads();
        if (threadIdx.x == 0) {
            for (uint32_t j = 0; j < cnt; ++j) {
                gentry[g0 + j] = state;
                gbase[g0 + j] = base;
                const uint32_t x = t16[j * 16 + state];
                base += x >> 4;
                state = x & 15u;
            }
        }
    }
    if (threadIdx.x == 0) {
        *nwords = base;
        if (base > cap)
            atomicOr(status, G4_STATUS_NOSPC);
    }
}

// per group: the tree again, then a down-sweep from the group's entry -> tiles.
// WALK (groups <= G4_TOP_CHUNK, k_g4p_top not launched): the block finds its
// group's entry itself by walking the tables of the groups before it (LDS),
// and the last block writes the total.
template <bool WALK>
__global__ __launch_bounds__(G4_THREADS) void k_g4p_spread(const uint32_t *__restrict__ agg, uint64_t tiles,
                                                           const uint32_t *__restrict__ gagg,
                                                           const uint32_t *__restrict__ gentry,
                                                           const uint64_t *__restrict__ gbase,
                                                           uint32_t *__restrict__ tentry, uint64_t *__restrict__ tbase,
                                                           uint64_t *__restrict__ nwords, uint64_t cap,
                                                           uint32_t *__restrict__ status)
{
    __shared__ G4Group sm;
    __shared__ uint32_t gt[WALK ? G4_TOP_CHUNK * 16 : 1];
    const uint64_t first = (uint64_t)blockIdx.x * G4_GROUP;
    const uint32_t cnt = (uint32_t)std::min<uint64_t>(G4_GROUP, tiles - first);
    const unsigned t = threadIdx.x;
    if (WALK)
        for (uint32_t k = t; k < blockIdx.x * 16u; k += G4_THREADS)
            gt[k] = gagg[k];
    g4_group_up(sm, agg, first, cnt);  // starts and ends with a barrier
    if (t == 0) {
        uint32_t state = 0;
        uint64_t base = 0;
        if (WALK) {
            for (uint32_t j = 0; j < blockIdx.x; ++j) {
                const uint32_t x = gt[j * 16 + state];
                base += x >> 4;
                state = x & 15u;
            }
            if (blockIdx.x + 1 == gridDim.x) {
                const uint64_t total = base + (sm.node[1][state] >> 4);
                *nwords = total;
                if (total > cap)
                    atomicOr(status, G4_STATUS_NOSPC);
            }
        } else {
            state = gentry[blockIdx.x];
            base = gbase[blockIdx.x];
        }
        sm.st[1] = state;
        sm.bs[1] = base;
    }
#pragma unroll 1
    for (uint32_t lvl = 1; lvl < G4_GROUP; lvl <<= 1) {
        __syncthreads();
        if (t < lvl) {
            const uint32_t i = lvl + t, s = sm.st[i];
            const uint32_t e = sm.node[2 * i][s];
            sm.st[2 * i] = s;
            sm.bs[2 * i] = sm.bs[i];
            sm.st[2 * i + 1] = e & 15u;
            sm.bs[2 * i + 1] = sm.bs[i] + (e >> 4);
        }
    }
    __syncthreads();
    if (t < cnt) {
        tentry[first + t] = sm.st[G4_GROUP + t];
        tbase[first + t] = sm.bs[G4_GROUP + t];
    }
}

__global__ __launch_bounds__(G4_THREADS) void k_g4p_emit(const uint8_t *__restrict__ vb, uint64_t n,
                                                         const uint32_t *__restrict__ tentry,
                                                         const uint64_t *__restrict__ tbase,
                                                         int32_t *__restrict__ out, uint64_t cap,
                                                         const uint32_t *__restrict__ status)
{
    __shared__ G4Tile sm;
    __shared__ uint8_t st[2 * G4_THREADS];
    __shared__ uint16_t bs[2 * G4_THREADS];
    __shared__ uint32_t wbuf[G4_TILE / 3 + 2];
    if (*status != 0)  // out-of-domain value or too small an output: write nothing
        return;
    const uint64_t start = (uint64_t)blockIdx.x * G4_TILE;
    g4_load<false, true>(sm, nullptr, const_cast<uint8_t *>(vb), n, start, nullptr);
    const unsigned t = threadIdx.x;
    uint64_t modes;
    uint32_t f[G4_SEG];
    g4_segment(sm, start + G4_SEG * t, n, modes, f);
#pragma unroll
    for (int e = 0; e < 16; ++e)
        sm.node[G4_THREADS + t][e] = (uint16_t)(e == 15 ? G4_DEAD : f[e]);
    g4_tree_up(sm);
    const uint32_t s0 = tentry[blockIdx.x];
    const uint32_t tile_words = sm.node[1][s0] >> 4;
    if (t == 0) {
        st[1] = (uint8_t)s0;
        bs[1] = 0;
    }
#pragma unroll 1
    for (uint32_t lvl = 1; lvl < G4_THREADS; lvl <<= 1) {
        __syncthreads();
        if (t < lvl) {
            const uint32_t i = lvl + t, s = st[i];
            const uint32_t e = sm.node[2 * i][s];
            st[2 * i] = (uint8_t)s;
            bs[2 * i] = bs[i];
            st[2 * i + 1] = (uint8_t)(e & 15u);
            bs[2 * i + 1] = (uint16_t)(bs[i] + (e >> 4));
        }
    }
    __syncthreads();
    // this segment's words: from its entry offset while inside the segment and < n
    uint32_t pos = st[G4_THREADS + t], j = bs[G4_THREADS + t];
    const uint64_t seg0 = start + G4_SEG * t;
    const uint32_t live = seg0 >= n ? 0u : (uint32_t)std::min<uint64_t>(G4_SEG, n - seg0);
    while (pos < live) {
        const uint32_t mode = (uint32_t)(modes >> (2 * pos)) & 3u;
        // bytes pos .. pos+15 of this segment (zero past n): 5 aligned dwords, byte-aligned
        const uint32_t *d = &sm.v[(G4_SEG / 4) * t + (pos >> 2)];
        const uint32_t sh = pos & 3u;
        const uint32_t u0 = d[0], u1 = d[1], u2 = d[2], u3 = d[3], u4 = d[4];
        const uint32_t x[4] = {__builtin_amdgcn_alignbyte(u1, u0, sh), __builtin_amdgcn_alignbyte(u2, u1, sh),
                               __builtin_amdgcn_alignbyte(u3, u2, sh), __builtin_amdgcn_alignbyte(u4, u3, sh)};
        const uint32_t b = g4_bits(mode), top = g4_top(mode), cnt = g4_cnt(mode);
        uint32_t code = mode << 30;
#pragma unroll
        for (uint32_t q = 0; q < 15; ++q)  // values past cnt belong to the next word: left out
            if (q < cnt)
                code |= ((x[q >> 2] >> (8 * (q & 3))) & 0xffu) << (top - q * b);
        wbuf[j++] = code;
        pos += cnt;
    }
    __syncthreads();
    const uint64_t base = tbase[blockIdx.x];
    for (uint32_t k = t; k < tile_words; k += G4_THREADS)
        if (base + k < cap)
            out[base + k] = (int32_t)wbuf[k];
}

// ---- unpack ---------------------------------------------------------------
constexpr uint32_t G4U_PER_THREAD = 4;
constexpr uint32_t G4U_BLOCK_WORDS = G4_THREADS * G4U_PER_THREAD;  // 1024 words -> <= 15360 values

__device__ __forceinline__ uint32_t g4_count(int32_t w) { return g4_cnt((uint32_t)w >> 30); }

template <unsigned NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *total)
{
    __shared__ uint32_t wsum[NT / 64];
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
    for (unsigned i = 0; i < NT / 64; ++i) {
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

// this thread's 4 words (0 past nw: counted as 15 values of mode 0, so only
// whole words may be read past the end — they are not)
__device__ __forceinline__ int4 g4u_words(const int32_t *__restrict__ words, uint64_t nw, uint64_t w0)
{
    if (w0 + 4 <= nw && (reinterpret_cast<uintptr_t>(words) & 15u) == 0)
        return *reinterpret_cast<const int4 *>(words + w0);
    int4 r;
    r.x = w0 < nw ? words[w0] : 0;
    r.y = w0 + 1 < nw ? words[w0 + 1] : 0;
    r.z = w0 + 2 < nw ? words[w0 + 2] : 0;
    r.w = w0 + 3 < nw ? words[w0 + 3] : 0;
    return r;
}

__device__ __forceinline__ uint32_t g4u_cnt4(const int4 &w, uint64_t nw, uint64_t w0)
{
    uint32_t s = 0;
    s += w0 < nw ? g4_count(w.x) : 0u;
    s += w0 + 1 < nw ? g4_count(w.y) : 0u;
    s += w0 + 2 < nw ? g4_count(w.z) : 0u;
    s += w0 + 3 < nw ? g4_count(w.w) : 0u;
    return s;
}

__global__ __launch_bounds__(G4_THREADS) void k_g4u_sums(const int32_t *__restrict__ words, uint64_t nw,
                                                         uint32_t *__restrict__ bsum)
{
    const uint64_t w0 = (uint64_t)blockIdx.x * G4U_BLOCK_WORDS + (uint64_t)threadIdx.x * G4U_PER_THREAD;
    const uint32_t s = g4u_cnt4(g4u_words(words, nw, w0), nw, w0);
    uint32_t tot;
    block_excl_scan<G4_THREADS>(s, &tot);
    if (threadIdx.x == 0)
        bsum[blockIdx.x] = tot;
}

constexpr unsigned G4U_SCAN_THREADS = 1024;

__global__ __launch_bounds__(G4U_SCAN_THREADS) void k_g4u_scan(const uint32_t *__restrict__ bsum, uint64_t nb,
                                                               uint64_t *__restrict__ bbase,
                                                               uint64_t *__restrict__ count, uint64_t cap,
                                                               uint32_t *__restrict__ status)
{
    __shared__ uint64_t carry;
    if (threadIdx.x == 0)
        carry = 0;
    __syncthreads();
    for (uint64_t b0 = 0; b0 < nb; b0 += G4U_SCAN_THREADS) {
        const uint64_t b = b0 + threadIdx.x;
        const uint32_t v = b < nb ? bsum[b] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_scan<G4U_SCAN_THREADS>(v, &tot);
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
    __shared__ uint8_t obuf[G4U_BLOCK_WORDS * 15];
    if (*status != 0)
        return;
    const uint64_t w0 = (uint64_t)blockIdx.x * G4U_BLOCK_WORDS + (uint64_t)threadIdx.x * G4U_PER_THREAD;
    const int4 w4 = g4u_words(words, nw, w0);
    uint32_t tot;
    uint32_t o = block_excl_scan<G4_THREADS>(g4u_cnt4(w4, nw, w0), &tot);
    const int32_t wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
    for (uint32_t i = 0; i < G4U_PER_THREAD; ++i) {
        if (w0 + i >= nw)
            break;
        const uint32_t code = (uint32_t)wv[i];
        const int mode = (int)(code >> 30);
        const uint32_t cnt = g4_cnt(mode), top = g4_top(mode), b = g4_bits(mode);
        const uint32_t mask = (1u << b) - 1u;
#pragma unroll
        for (uint32_t j = 0; j < 15; ++j)
            if (j < cnt)
                obuf[o + j] = (uint8_t)((code >> (top - j * b)) & mask);
        o += cnt;
    }
    __syncthreads();
    const uint64_t base = bbase[blockIdx.x];
    for (uint32_t k = threadIdx.x; k < tot; k += G4_THREADS)
        out[base + k] = (int32_t)obuf[k];
}

// workspace layout (bytes, 256-aligned pieces)
struct G4Ws {
    uint32_t *agg, *gagg, *gentry, *tentry, *bsum;
    uint64_t *gbase, *tbase, *bbase;
    uint8_t *vb;
};

static inline uint64_t al256(uint64_t b) { return (b + 255) & ~255ull; }

static uint64_t g4_ws(uint64_t n, char *base, G4Ws *w)
{
    const uint64_t tiles = (n + G4_TILE - 1) / G4_TILE;
    const uint64_t groups = (tiles + G4_GROUP - 1) / G4_GROUP;
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) {
        char *p = base ? base + off : nullptr;
        off += al256(bytes);
        return p;
    };
    G4Ws t{};
    t.agg = (uint32_t *)take(tiles * 64);
    t.gagg = (uint32_t *)take(groups * 64);
    t.gentry = (uint32_t *)take(groups * 4);
    t.gbase = (uint64_t *)take(groups * 8);
    t.tentry = (uint32_t *)take(tiles * 4);
    t.tbase = (uint64_t *)take(tiles * 8);
    t.vb = (uint8_t *)take(tiles * G4_TILE);  // whole tiles: the dword stores past n stay inside
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
    t.bsum = (uint32_t *)take(nb * 4);   // block sums
    t.bbase = (uint64_t *)take(nb * 8);  // block bases
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
    GC_REQUIRE(aligned16(workspace), "gc_greedy4_pack_device: workspace must be 16-byte aligned");
    hipStream_t st = as_stream(stream);
    G4Ws w;
    g4_ws(n, reinterpret_cast<char *>(workspace), &w);
    hipLaunchKernelGGL(k_g4_init, dim3(1), dim3(1), 0, st, nwords, status);
    if (n == 0)
        return launch_status("gc_greedy4_pack_device");
    const uint64_t tiles = (n + G4_TILE - 1) / G4_TILE;
    const uint64_t groups = (tiles + G4_GROUP - 1) / G4_GROUP;
    if (aligned16(src))
        hipLaunchKernelGGL(k_g4p_tile<true>, dim3((unsigned)tiles), dim3(G4_THREADS), 0, st, src, n, w.vb, w.agg,
                           status);
    else
        hipLaunchKernelGGL(k_g4p_tile<false>, dim3((unsigned)tiles), dim3(G4_THREADS), 0, st, src, n, w.vb, w.agg,
                           status);
    hipLaunchKernelGGL(k_g4p_group, dim3((unsigned)groups), dim3(G4_THREADS), 0, st, w.agg, tiles, w.gagg);
    if (groups <= G4_TOP_CHUNK) {
        hipLaunchKernelGGL(k_g4p_spread<true>, dim3((unsigned)groups), dim3(G4_THREADS), 0, st, w.agg, tiles, w.gagg,
                           w.gentry, w.gbase, w.tentry, w.tbase, nwords, cap, status);
    } else {
        hipLaunchKernelGGL(k_g4p_top, dim3(1), dim3(G4_THREADS), 0, st, w.gagg, groups, w.gentry, w.gbase, nwords,
                           cap, status);
        hipLaunchKernelGGL(k_g4p_spread<false>, dim3((unsigned)groups), dim3(G4_THREADS), 0, st, w.agg, tiles,
                           w.gagg, w.gentry, w.gbase, w.tentry, w.tbase, nwords, cap, status);
    }
    hipLaunchKernelGGL(k_g4p_emit, dim3((unsigned)tiles), dim3(G4_THREADS), 0, st, w.vb, n, w.tentry, w.tbase, out,
                       cap, status);
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
    hipLaunchKernelGGL(k_g4u_sums, dim3((unsigned)nb), dim3(G4_THREADS), 0, st, words, nwords, w.bsum);
    hipLaunchKernelGGL(k_g4u_scan, dim3(1), dim3(G4U_SCAN_THREADS), 0, st, w.bsum, nb, w.bbase, count, cap, status);
    hipLaunchKernelGGL(k_g4u_emit, dim3((unsigned)nb), dim3(G4_THREADS), 0, st, words, nwords, w.bbase, out, status);
    return launch_status("gc_greedy4_unpack_device");
}

}  // extern "C"
