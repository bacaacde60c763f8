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
//   k_g4_init      zero the result pair and the per-group tickets
//   k_g4p_tile     per 8192-element tile (256 threads x one segment): window
//                  masks by SWAR byte tests and OR-doubling, the segment table
//                  by a backward recurrence held in registers (static indices
//                  only), a reduction tree of the 256 tables in LDS -> the
//                  tile's table; the bytes go to the workspace for phase 2.
//                  The last tile of each 128-tile group to finish (a ticket;
//                  ready bits, no fence) builds and stores the group's tree.
//   k_g4p_top      only for > 64 groups: one block walks the group roots ->
//                  group entry offsets and word bases, the total
//   k_g4p_emit     per tile: its entry = walk of the group roots (<= 64
//                  groups) + the left siblings down the group tree; the tile
//                  tree again from the bytes, a down-sweep -> every segment's
//                  entry and word base; each thread packs its segment's words
//                  into LDS, the block stores the tile's words coalesced.
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
constexpr uint32_t G4_GROUP = 128;                      // tiles per group
constexpr uint32_t G4_GDEPTH = 7;                       // log2(G4_GROUP)
constexpr uint32_t G4_DEAD = 15;                        // table state: the chain has passed n
constexpr uint32_t G4_TOP_CHUNK = 128;                  // group tables staged in LDS per top step
constexpr uint32_t G4_WALK_MAX = 64;                    // groups the emit blocks walk themselves (else k_g4p_top)
constexpr uint32_t G4_STATUS_RANGE = 1u, G4_STATUS_NOSPC = 2u;
constexpr uint32_t G4_READY = 0x80000000u;              // agg entry written (tile tables need < 2^16)

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

// a group's tree of tile tables (u32 entries: words up to 256 x 2731)
struct G4GroupTree {
    uint32_t node[2 * G4_GROUP][16];
};

// the mode classes of this thread's segment (bit p = position seg0 + p), from
// the window masks W15 = some value >= 4 in [p, p+15), W7 = some value >= 16
// in [p, p+7), W4 = some value >= 128 in [p, p+4).  W4 ⊆ W7 ⊆ W15, so the
// mode at p is W15[p] + W7[p] + W4[p] = 2 hi[p] + lo[p] with hi = W7 and
// lo = W15 ^ W7 ^ W4 (0: 15 x 2 bits, 1: 7 x 4, 2: 4 x 7, 3: 3 x 8).
struct G4Cls {
    uint32_t lo, hi;
};

__device__ __forceinline__ G4Cls g4_classes(const G4Tile &sm)
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
    // window ORs by doubling: [p, p+2), [p, p+4), [p, p+8), then one overlapping step
    const uint64_t a1 = ge4 | (ge4 >> 1), a2 = a1 | (a1 >> 2), a3 = a2 | (a2 >> 4);
    const uint64_t b1 = ge16 | (ge16 >> 1), b2 = b1 | (b1 >> 2);
    const uint64_t c1 = ge128 | (ge128 >> 1);
    const uint32_t w15 = (uint32_t)(a3 | (a3 >> 7)), w7 = (uint32_t)(b2 | (b2 >> 3)), w4 = (uint32_t)(c1 | (c1 >> 2));
    return G4Cls{w15 ^ w7 ^ w4, w7};
}

__device__ __forceinline__ uint32_t g4_mode(const G4Cls &c, uint32_t p)
{
    return (((c.hi >> p) & 1u) << 1) | ((c.lo >> p) & 1u);
}

// bit p of m as a lane mask (0 or ~0): one v_bfe_i32
__device__ __forceinline__ uint32_t bitmask(uint32_t m, int p) { return (uint32_t)__builtin_amdgcn_sbfe((int)m, p, 1); }

// the segment table (entries 0..14, exit | words << 4) by the backward
// recurrence f[p] = 1 word + f[p + cnt(p)], where a successor past the
// segment is its offset there, p + cnt - G4_SEG (0..14).  All indices are
// static (the recurrence is unrolled), so f stays in registers; the
// successor is picked with three bitfield selects on the class bits.
// TAIL: the tile holds position n (positions >= live are past the chain's end).
template <bool TAIL>
__device__ __forceinline__ void g4_dp(const G4Cls &c, uint32_t live, uint32_t f[G4_SEG])
{
#pragma unroll
    for (int p = G4_SEG - 1; p >= 0; --p) {
        const uint32_t s3 = p + 3 < (int)G4_SEG ? f[(p + 3) % G4_SEG] : (uint32_t)(p + 3 - (int)G4_SEG);
        const uint32_t s4 = p + 4 < (int)G4_SEG ? f[(p + 4) % G4_SEG] : (uint32_t)(p + 4 - (int)G4_SEG);
        const uint32_t s7 = p + 7 < (int)G4_SEG ? f[(p + 7) % G4_SEG] : (uint32_t)(p + 7 - (int)G4_SEG);
        const uint32_t s15 = p + 15 < (int)G4_SEG ? f[(p + 15) % G4_SEG] : (uint32_t)(p + 15 - (int)G4_SEG);
        const uint32_t mlo = bitmask(c.lo, p), mhi = bitmask(c.hi, p);
        // mode 3: s3, 2: s4, 1: s7, 0: s15
        const uint32_t nx = (mhi & ((mlo & s3) | (~mlo & s4))) | (~mhi & ((mlo & s7) | (~mlo & s15)));
        if (TAIL)
            f[p] = (uint32_t)p < live ? nx + 16u : G4_DEAD;
        else
            f[p] = nx + 16u;
    }
}

// reduction tree over the NLEAF leaves node[NLEAF + i] -> node[1] (u16 tile
// tree of 256 segments, u32 group tree of G4_GROUP tiles).  Level by level (unrolled: every level's trip count
// is a constant); node i = left child then right child, a thread per (node,
// entry) pair: entry e = t & 15 of nodes lvl + (t >> 4) + 16 r, so 16
// consecutive lanes read one row (conflict-free) at immediate LDS offsets.
// Composition: exit from the right child's entry at the left's exit, words
// added — (x & ~15) + y.  A level's lookups are all issued before its stores
// (the rows written are never read on the same level).
template <typename T, uint32_t NLEAF>
__device__ __forceinline__ void g4_tree_up(T (*node)[16])
{
    static_assert(NLEAF <= 256 && (NLEAF & (NLEAF - 1)) == 0, "tree width");
    const uint32_t t = threadIdx.x, e = t & 15u, i0 = t >> 4;
#pragma unroll
    for (int L = 7; L >= 0; --L) {
        if ((1u << L) >= NLEAF)
            continue;
        const uint32_t lvl = 1u << L;
        __syncthreads();
        if (lvl >= 16) {
            constexpr uint32_t RMAX = 8;
            const uint32_t R = lvl / 16;
            uint32_t res[RMAX];
#pragma unroll
            for (uint32_t r = 0; r < RMAX; ++r) {
                if (r < R) {
                    const uint32_t i = lvl + i0 + 16 * r;
                    const uint32_t x = node[2 * i][e], y = node[2 * i + 1][x & 15u];
                    res[r] = (x & ~15u) + y;
                }
            }
#pragma unroll
            for (uint32_t r = 0; r < RMAX; ++r)
                if (r < R)
                    node[lvl + i0 + 16 * r][e] = (T)res[r];
        } else if (i0 < lvl) {
            const uint32_t i = lvl + i0;
            const uint32_t x = node[2 * i][e], y = node[2 * i + 1][x & 15u];
            node[i][e] = (T)((x & ~15u) + y);
        }
    }
    __syncthreads();
}

// load tile `tile` of the values into LDS as bytes (0 past n) + halo.
// From int32 src (range-checked; the bytes also go to vb) or from vb.  A tile
// whose halo lies before n (every tile but the last one or two) issues all its
// loads before using any (the guarded form made each wait for the previous).
template <bool FROM_SRC, bool ALIGNED>
__device__ __forceinline__ void g4_load(G4Tile &sm, const int32_t *__restrict__ src, uint8_t *__restrict__ vb,
                                        uint64_t n, uint64_t start, uint32_t *__restrict__ status)
{
    constexpr uint32_t QT = G4_TILE / 4, QH = (G4_TILE + 32) / 4;  // dwords of the tile / with the halo
    constexpr uint32_t J = QT / G4_THREADS;                          // full rounds (8)
    const unsigned t = threadIdx.x;
    if (start + 4ull * QH <= n && (!FROM_SRC || ALIGNED)) {
        if (FROM_SRC) {
            typedef int i4v __attribute__((ext_vector_type(4)));
            int4 v[J + 1];
#pragma unroll
            for (uint32_t j = 0; j < J; ++j) {  // src is streamed once: nontemporal
                const i4v r = __builtin_nontemporal_load(reinterpret_cast<const i4v *>(src + start) + j * G4_THREADS + t);
                v[j] = make_int4(r.x, r.y, r.z, r.w);
            }
            if (t < QH - QT)
                v[J] = *(reinterpret_cast<const int4 *>(src + start) + QT + t);
            uint32_t bad = 0;
#pragma unroll
            for (uint32_t j = 0; j <= J; ++j) {
                if (j == J && t >= QH - QT)
                    break;
                const uint32_t q = j * G4_THREADS + t;
                bad |= (uint32_t)v[j].x | (uint32_t)v[j].y | (uint32_t)v[j].z | (uint32_t)v[j].w;
                const uint32_t packed = __builtin_amdgcn_perm(__builtin_amdgcn_perm(v[j].w, v[j].z, 0x0c0c0400u),
                                                              __builtin_amdgcn_perm(v[j].y, v[j].x, 0x0c0c0400u),
                                                              0x05040100u);
                if (j < J)
                    reinterpret_cast<uint32_t *>(vb + start)[q] = packed;
                sm.v[q] = packed;
            }
            if (bad > 255u)
                atomicOr(status, G4_STATUS_RANGE);
        } else {
            uint32_t v[J + 1];
#pragma unroll
            for (uint32_t j = 0; j < J; ++j)
                v[j] = reinterpret_cast<const uint32_t *>(vb + start)[j * G4_THREADS + t];
            if (t < QH - QT)
                v[J] = reinterpret_cast<const uint32_t *>(vb + start)[QT + t];
#pragma unroll
            for (uint32_t j = 0; j < J; ++j)
                sm.v[j * G4_THREADS + t] = v[j];
            if (t < QH - QT)
                sm.v[QT + t] = v[J];
        }
        __syncthreads();
        return;
    }
    bool bad = false;
    for (uint32_t q = t; q < QH; q += G4_THREADS) {  // the tail: guarded element loads
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
            packed = __builtin_amdgcn_perm(__builtin_amdgcn_perm(v.w, v.z, 0x0c0c0400u),
                                           __builtin_amdgcn_perm(v.y, v.x, 0x0c0c0400u), 0x05040100u);
            if (q < QT && g < n)
                *reinterpret_cast<uint32_t *>(vb + g) = packed;  // vb is padded to whole tiles
        } else if (g < n) {
            packed = *reinterpret_cast<const uint32_t *>(vb + g);  // zero past n (written so by k_g4p_tile)
        }
        sm.v[q] = packed;
    }
    if (FROM_SRC && bad)
        atomicOr(status, G4_STATUS_RANGE);
    __syncthreads();
}

// this thread's segment table (leaves) from the tile's LDS bytes; written to
// node[256 + t] (and returned packed, 8 u32)
__device__ __forceinline__ G4Cls g4_leaf(G4Tile &sm, uint64_t start, uint64_t n, uint4 &l0, uint4 &l1)
{
    const unsigned t = threadIdx.x;
    const G4Cls c = g4_classes(sm);
    uint32_t f[G4_SEG];
    const uint64_t seg0 = start + G4_SEG * t;
    if (start + G4_TILE <= n) {  // uniform: a full tile has no position past n
        g4_dp<false>(c, G4_SEG, f);
    } else {
        const uint32_t live = seg0 >= n ? 0u : (uint32_t)std::min<uint64_t>(G4_SEG, n - seg0);
        g4_dp<true>(c, live, f);
    }
    uint32_t h[8];
#pragma unroll
    for (int e = 0; e < 8; ++e)
        h[e] = f[2 * e] | ((2 * e + 1 == 15 ? G4_DEAD : f[2 * e + 1]) << 16);
    l0 = make_uint4(h[0], h[1], h[2], h[3]);
    l1 = make_uint4(h[4], h[5], h[6], h[7]);
    uint4 *leaf = reinterpret_cast<uint4 *>(sm.node[G4_THREADS + t]);
    leaf[0] = l0;
    leaf[1] = l1;
    return c;
}

// Phase 1 per tile: its table -> agg.  The last tile block of a group to
// finish (a relaxed agent-scope ticket) builds the group's tree of tile
// tables and stores all of it (gtree: 511 nodes x 16 u32).  No fence: every
// agg entry is a single agent-scope atomic store carrying a ready bit (bit 31,
// cleared by k_g4_init), and the winner reads each entry with agent-scope
// atomic loads until its bit is set — coherence of single locations is all it
// needs.  (A release fence per block writes back the whole L2 on gfx950:
// measured 102 against 40 us for the kernel.)
template <bool ALIGNED>
__global__ __launch_bounds__(G4_THREADS) void k_g4p_tile(const int32_t *__restrict__ src, uint64_t n,
                                                         uint64_t tiles, uint8_t *__restrict__ vb,
                                                         uint4 *__restrict__ leaves, uint2 *__restrict__ cls,
                                                         uint32_t *__restrict__ agg, uint32_t *__restrict__ gtree,
                                                         uint32_t *__restrict__ gcount, uint32_t *__restrict__ status)
{
    __shared__ union {
        G4Tile tile;
        G4GroupTree grp;
    } sm;
    __shared__ uint32_t is_last;
    const unsigned t = threadIdx.x;
    const uint64_t tile = blockIdx.x, start = tile * G4_TILE;
    g4_load<true, ALIGNED>(sm.tile, src, vb, n, start, status);
    uint4 l0, l1;
    const G4Cls c = g4_leaf(sm.tile, start, n, l0, l1);
    const uint64_t seg = tile * G4_THREADS + t;  // the emit reads these instead of recomputing them
    leaves[2 * seg] = l0;
    leaves[2 * seg + 1] = l1;
    cls[seg] = make_uint2(c.lo, c.hi);
    g4_tree_up<uint16_t, G4_THREADS>(sm.tile.node);
    if (t < 16)
        __hip_atomic_store(&agg[tile * 16 + t], (uint32_t)sm.tile.node[1][t] | G4_READY, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t g = tile / G4_GROUP, first = g * G4_GROUP;
    const uint32_t cnt = (uint32_t)std::min<uint64_t>(G4_GROUP, tiles - first);
    __syncthreads();
    if (t == 0)
        is_last = __hip_atomic_fetch_add(&gcount[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == cnt - 1;
    __syncthreads();
    if (!is_last)
        return;
    // leaves of the group tree; past the group's end: identity.  All loads are
    // issued first; an entry whose ready bit is not visible yet is re-read
    constexpr uint32_t R = G4_GROUP * 16 / G4_THREADS;
    static_assert(R * G4_THREADS == G4_GROUP * 16, "leaf loads per thread");
    uint32_t x[R];
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t k = t + r * G4_THREADS, i = k >> 4;
        x[r] = i < cnt ? __hip_atomic_load(&agg[(first + i) * 16 + (k & 15u)], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT)
                       : (k & 15u) | G4_READY;
    }
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t k = t + r * G4_THREADS, i = k >> 4;
        while (!(x[r] & G4_READY))  // its block took a ticket, so the store is done; visibility may lag
            x[r] = __hip_atomic_load(&agg[(first + i) * 16 + (k & 15u)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sm.grp.node[G4_GROUP + i][k & 15u] = x[r] & ~G4_READY;
    }
    g4_tree_up<uint32_t, G4_GROUP>(sm.grp.node);
    uint4 *dst = reinterpret_cast<uint4 *>(gtree + g * (2 * G4_GROUP * 16));
    const uint4 *srcn = reinterpret_cast<const uint4 *>(sm.grp.node);
    for (uint32_t k = t; k < 2 * G4_GROUP * 4; k += G4_THREADS)
        dst[k] = srcn[k];
}

// groups > G4_WALK_MAX: one block walks the group roots from offset 0 ->
// each group's entry offset and word base, the total and the capacity check
__global__ __launch_bounds__(G4_THREADS) void k_g4p_top(const uint32_t *__restrict__ gtree, uint64_t groups,
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
            t16[k] = gtree[(g0 + (k >> 4)) * (2 * G4_GROUP * 16) + 16 + (k & 15u)];  // node 1 of group g0 + k/16
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

// Phase 2 per tile: its entry offset and word base (the group's, from a walk
// of the group roots or from k_g4p_top, then down the group tree: the left
// siblings on the path to the tile's leaf), the tile's tree again from the
// bytes, a down-sweep from the entry -> every segment's entry and base; each
// thread packs its segment's words into LDS, the block stores them coalesced.
// WALK (groups <= G4_WALK_MAX): every block walks all group roots, so it
// also knows the total and checks the capacity itself (block 0 reports it).
template <bool WALK>
__global__ __launch_bounds__(G4_THREADS) void k_g4p_emit(const uint8_t *__restrict__ vb,
                                                         const uint4 *__restrict__ leaves,
                                                         const uint2 *__restrict__ cls, uint64_t n, uint64_t groups,
                                                         const uint32_t *__restrict__ gtree,
                                                         const uint32_t *__restrict__ gentry,
                                                         const uint64_t *__restrict__ gbase,
                                                         int32_t *__restrict__ out, uint64_t cap,
                                                         uint64_t *__restrict__ nwords, uint32_t *__restrict__ status)
{
    __shared__ G4Tile sm;
    __shared__ uint8_t st[2 * G4_THREADS];
    __shared__ uint16_t bs[2 * G4_THREADS];
    __shared__ uint32_t roots[WALK ? G4_WALK_MAX * 16 : 1];
    __shared__ uint32_t path[G4_GDEPTH][16];
    __shared__ uint32_t e_state, e_ok;
    __shared__ uint64_t e_base;
    if (*status != 0)  // an out-of-domain value: write nothing
        return;
    const unsigned t = threadIdx.x;
    const uint64_t tile = blockIdx.x, start = tile * G4_TILE;
    const uint64_t g = tile / G4_GROUP;
    const uint32_t j = (uint32_t)(tile - g * G4_GROUP);
    const uint32_t *gt = gtree + g * (2 * G4_GROUP * 16);
    if (t < 16 * G4_GDEPTH) {  // the left siblings of the path root -> leaf G4_GROUP + j
        const uint32_t lvl = t >> 4;
        path[lvl][t & 15u] = gt[((((uint32_t)G4_GROUP + j) >> (G4_GDEPTH - 1 - lvl)) ^ 1u) * 16 + (t & 15u)];
    }
    if (WALK)
        for (uint32_t k = t; k < groups * 16; k += G4_THREADS)
            roots[k] = gtree[(k >> 4) * (2 * G4_GROUP * 16) + 16 + (k & 15u)];
    const uint64_t seg = tile * G4_THREADS + t;  // this thread's segment table and classes (phase 1)
    {
        uint4 *leaf = reinterpret_cast<uint4 *>(sm.node[G4_THREADS + t]);
        leaf[0] = leaves[2 * seg];
        leaf[1] = leaves[2 * seg + 1];
    }
    const uint2 cl = cls[seg];
    const G4Cls c{cl.x, cl.y};
    g4_load<false, true>(sm, nullptr, const_cast<uint8_t *>(vb), n, start, nullptr);  // ends with a barrier
    if (t == 0) {
        uint32_t state = 0;
        uint64_t base = 0, total = 0;
        if (WALK) {
            for (uint32_t q = 0; q < groups; ++q) {
                if (q == g) {
                    e_state = state;
                    e_base = base;
                }
                const uint32_t x = roots[q * 16 + state];
                base += x >> 4;
                state = x & 15u;
            }
            total = base;
            state = e_state;
            base = e_base;
        } else {
            state = gentry[g];
            base = gbase[g];
        }
        for (uint32_t lvl = 0; lvl < G4_GDEPTH; ++lvl) {
            if ((j >> (G4_GDEPTH - 1 - lvl)) & 1u) {  // the path goes right: the left sibling's words come first
                const uint32_t x = path[lvl][state];
                base += x >> 4;
                state = x & 15u;
            }
        }
        e_state = state;
        e_base = base;
        e_ok = 1;
        if (WALK) {
            e_ok = total <= cap;
            if (tile == 0) {
                *nwords = total;
                if (!e_ok)
                    atomicOr(status, G4_STATUS_NOSPC);
            }
        }
    }
    g4_tree_up<uint16_t, G4_THREADS>(sm.node);  // starts with a barrier (e_* visible after)
    if (!e_ok)
        return;
    const uint32_t s0 = e_state;
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
    // the tree is done with: its 16 KB hold the tile's word list, one u16 per
    // word = start position in the tile | mode << 14 (<= 8192 / 3 + 1 words)
    static_assert(sizeof(sm.node) >= (G4_TILE / 3 + 2) * 2 && G4_TILE <= (1u << 14), "word list");
    uint16_t *wl = reinterpret_cast<uint16_t *>(sm.node);
    {  // this segment's word starts: from its entry offset while inside the segment and < n
        uint32_t pos = st[G4_THREADS + t], jw = bs[G4_THREADS + t];
        const uint64_t seg0 = start + G4_SEG * t;
        const uint32_t live = seg0 >= n ? 0u : (uint32_t)std::min<uint64_t>(G4_SEG, n - seg0);
        while (pos < live) {
            const uint32_t mode = g4_mode(c, pos);
            wl[jw++] = (uint16_t)((G4_SEG * t + pos) | (mode << 14));
            pos += g4_cnt(mode);
        }
    }
    __syncthreads();
    // one word per lane: consecutive lanes pack consecutive words and store them coalesced
    const uint64_t base = e_base;
    const uint8_t *vbytes = reinterpret_cast<const uint8_t *>(sm.v);
    for (uint32_t k = t; k < tile_words; k += G4_THREADS) {
        const uint32_t s16 = wl[k], p = s16 & 0x3fffu, mode = s16 >> 14;
        // bytes p .. p+15 of the tile (zero past n): 5 aligned dwords, byte-aligned
        const uint32_t *d = &sm.v[p >> 2];
        const uint32_t sh = p & 3u;
        const uint32_t u0 = d[0], u1 = d[1], u2 = d[2], u3 = d[3], u4 = d[4];
        const uint32_t x[4] = {__builtin_amdgcn_alignbyte(u1, u0, sh), __builtin_amdgcn_alignbyte(u2, u1, sh),
                               __builtin_amdgcn_alignbyte(u3, u2, sh), __builtin_amdgcn_alignbyte(u4, u3, sh)};
        const uint32_t b = g4_bits(mode), top = g4_top(mode), cnt = g4_cnt(mode);
        uint32_t code = mode << 30;
#pragma unroll
        for (uint32_t q = 0; q < 15; ++q)  // values past cnt belong to the next word: left out
            if (q < cnt)
                code |= ((x[q >> 2] >> (8 * (q & 3))) & 0xffu) << (top - q * b);
        if (base + k < cap)
            out[base + k] = (int32_t)code;
    }
    (void)vbytes;
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

// the result pair, the per-group tickets and the ready bits of k_g4p_tile's
// table rows (the workspace needs no initialisation by the caller)
__global__ void k_g4_init(uint64_t *count, uint32_t *status, uint32_t *__restrict__ gcount, uint64_t groups,
                          uint32_t *__restrict__ agg, uint64_t agg_words)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        *count = 0;
        *status = 0;
    }
    for (uint64_t k = i; k < groups; k += (uint64_t)gridDim.x * blockDim.x)
        gcount[k] = 0;
    for (uint64_t k = i; k < agg_words; k += (uint64_t)gridDim.x * blockDim.x)
        agg[k] = 0;
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
// up to this many unpack blocks (4 M words) each emit block sums the block
// totals itself (k_g4u_emit_nb: <= 16 loads per thread from L2) instead of a
// one-block scan launch
constexpr uint64_t G4U_NB_DIRECT = 4096;

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

// the emit without a scan launch: each block sums the block totals before it
// (its base) and all of them (the count and the capacity check) from the
// L2-resident bsum, so no block writes past cap and nothing is written on
// NOSPC; block 0 writes *count and *status (the workspace and result need no
// initialisation launch)
__device__ __forceinline__ uint64_t g4u_wave_sum(uint64_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o, 64);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o, 64);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}

__global__ __launch_bounds__(G4_THREADS) void k_g4u_emit_nb(const int32_t *__restrict__ words, uint64_t nw,
                                                            const uint32_t *__restrict__ bsum, uint64_t nb,
                                                            int32_t *__restrict__ out, uint64_t cap,
                                                            uint64_t *__restrict__ count, uint32_t *__restrict__ status)
{
    __shared__ uint8_t obuf[G4U_BLOCK_WORDS * 15];
    __shared__ uint64_t red[2][G4_THREADS / 64];
    const unsigned t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint64_t b = blockIdx.x;
    uint64_t pre = 0, all = 0;
    for (uint64_t k = t; k < nb; k += G4_THREADS) {
        const uint32_t v = bsum[k];
        all += v;
        pre += k < b ? v : 0u;
    }
    pre = g4u_wave_sum(pre);
    all = g4u_wave_sum(all);
    if (lane == 0) {
        red[0][wv] = pre;
        red[1][wv] = all;
    }
    const uint64_t w0 = b * G4U_BLOCK_WORDS + (uint64_t)t * G4U_PER_THREAD;
    const int4 w4 = g4u_words(words, nw, w0);
    uint32_t tot;
    uint32_t o = block_excl_scan<G4_THREADS>(g4u_cnt4(w4, nw, w0), &tot);  // its barriers publish red
    uint64_t base = 0, total = 0;
#pragma unroll
    for (unsigned i = 0; i < G4_THREADS / 64; ++i) {
        base += red[0][i];
        total += red[1][i];
    }
    if (b == 0 && t == 0) {
        *count = total;
        *status = total > cap ? G4_STATUS_NOSPC : 0u;
    }
    if (total > cap)
        return;
    const int32_t wv4[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
    for (uint32_t i = 0; i < G4U_PER_THREAD; ++i) {
        if (w0 + i >= nw)
            break;
        const uint32_t code = (uint32_t)wv4[i];
        const int mode = (int)(code >> 30);
        const uint32_t cnt = g4_cnt(mode), top = g4_top(mode), bb = g4_bits(mode);
        const uint32_t mask = (1u << bb) - 1u;
#pragma unroll
        for (uint32_t j = 0; j < 15; ++j)
            if (j < cnt)
                obuf[o + j] = (uint8_t)((code >> (top - j * bb)) & mask);
        o += cnt;
    }
    __syncthreads();
    for (uint32_t k = t; k < tot; k += G4_THREADS)
        out[base + k] = (int32_t)obuf[k];
}

// workspace layout (bytes, 256-aligned pieces)
struct G4Ws {
    uint32_t *agg, *gtree, *gcount, *gentry, *bsum;
    uint64_t *gbase, *bbase;
    uint8_t *vb;
    uint4 *leaves;  // per segment: its table, 16 x u16
    uint2 *cls;     // per segment: the mode classes (lo, hi)
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
    t.gtree = (uint32_t *)take(groups * (2 * G4_GROUP * 16 * 4));  // 16 KB per group
    t.gcount = (uint32_t *)take(groups * 4);
    t.gentry = (uint32_t *)take(groups * 4);
    t.gbase = (uint64_t *)take(groups * 8);
    t.vb = (uint8_t *)take(tiles * G4_TILE);  // whole tiles: the dword stores past n stay inside
    t.leaves = (uint4 *)take(tiles * G4_THREADS * 32);
    t.cls = (uint2 *)take(tiles * G4_THREADS * 8);
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
    const uint64_t tiles = (n + G4_TILE - 1) / G4_TILE;
    const uint64_t groups = (tiles + G4_GROUP - 1) / G4_GROUP;
    hipLaunchKernelGGL(k_g4_init, dim3((unsigned)std::min<uint64_t>(1024, std::max<uint64_t>(1, tiles / 16))),
                       dim3(256), 0, st, nwords, status, w.gcount, groups, w.agg, tiles * 16);
    if (n == 0)
        return launch_status("gc_greedy4_pack_device");
    if (aligned16(src))
        hipLaunchKernelGGL(k_g4p_tile<true>, dim3((unsigned)tiles), dim3(G4_THREADS), 0, st, src, n, tiles, w.vb,
                           w.leaves, w.cls, w.agg, w.gtree, w.gcount, status);
    else
        hipLaunchKernelGGL(k_g4p_tile<false>, dim3((unsigned)tiles), dim3(G4_THREADS), 0, st, src, n, tiles, w.vb,
                           w.leaves, w.cls, w.agg, w.gtree, w.gcount, status);
    if (groups <= G4_WALK_MAX) {
        hipLaunchKernelGGL(k_g4p_emit<true>, dim3((unsigned)tiles), dim3(G4_THREADS), 0, st, w.vb, w.leaves, w.cls, n,
                           groups, w.gtree, w.gentry, w.gbase, out, cap, nwords, status);
    } else {
        hipLaunchKernelGGL(k_g4p_top, dim3(1), dim3(G4_THREADS), 0, st, w.gtree, groups, w.gentry, w.gbase, nwords,
                           cap, status);
        hipLaunchKernelGGL(k_g4p_emit<false>, dim3((unsigned)tiles), dim3(G4_THREADS), 0, st, w.vb, w.leaves, w.cls,
                           n, groups, w.gtree, w.gentry, w.gbase, out, cap, nwords, status);
    }
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
    const uint64_t nb = (nwords + G4U_BLOCK_WORDS - 1) / G4U_BLOCK_WORDS;
    if (nwords > 0 && nb <= G4U_NB_DIRECT) {  // every block sums the block totals itself: two launches
        hipLaunchKernelGGL(k_g4u_sums, dim3((unsigned)nb), dim3(G4_THREADS), 0, st, words, nwords, w.bsum);
        hipLaunchKernelGGL(k_g4u_emit_nb, dim3((unsigned)nb), dim3(G4_THREADS), 0, st, words, nwords, w.bsum, nb, out,
                           cap, count, status);
        return launch_status("gc_greedy4_unpack_device");
    }
    hipLaunchKernelGGL(k_g4_init, dim3(1), dim3(256), 0, st, count, status, nullptr, (uint64_t)0, nullptr,
                       (uint64_t)0);
    if (nwords == 0)
        return launch_status("gc_greedy4_unpack_device");
    hipLaunchKernelGGL(k_g4u_sums, dim3((unsigned)nb), dim3(G4_THREADS), 0, st, words, nwords, w.bsum);
    hipLaunchKernelGGL(k_g4u_scan, dim3(1), dim3(G4U_SCAN_THREADS), 0, st, w.bsum, nb, w.bbase, count, cap, status);
    hipLaunchKernelGGL(k_g4u_emit, dim3((unsigned)nb), dim3(G4_THREADS), 0, st, words, nwords, w.bbase, out, status);
    return launch_status("gc_greedy4_unpack_device");
}

}  // extern "C"
