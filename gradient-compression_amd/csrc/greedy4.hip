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
// whose elements are FUNCTIONS.  A range of positions maps the offset its
// first word starts at (0..14, or 15 = the chain has passed n) to the offset
// its chain leaves at and the words it emitted: a 16-entry table (exit |
// words << 4), and tables compose associatively.
//
// Pack: ONE persistent launch, one 1024-thread workgroup per CU (k_g4p_one).
// Round r, block b owns tile r*G + b (C positions, <= 98,304):
//   1. the tile's values -> LDS as bytes (+ a 16-byte halo), range check;
//      loaded by quarters of the block, one after another (g1_load_wave);
//   2. per thread 96 positions: window classes (SWAR byte tests + OR
//      doubling), the table by a backward recurrence chained over three
//      32-position blocks (registers only, static indices);
//   3. per wave a tree of its 64 tables in LDS (u16 entries, 16 lanes per
//      node pair; only LEFT children are kept — the walk down needs nothing
//      else), then a 16-leaf tree of the wave roots -> the tile's table;
//   4. the table goes out as 16 {entry, tag} granules (8-byte sc1 stores);
//      every block re-reads all G tiles' granules (sc1) until the tags match
//      and composes them (a 4-ary tree in LDS) -> its entry state and word
//      base, the round's exit state and total, and whether any tile held a
//      value outside [0, 255];
//   5. walking down the trees gives every thread its entry and word base;
//      the threads list their word starts, then consecutive lanes pack
//      consecutive words from the LDS bytes (coalesced stores).
// HBM: src read once (4n), the words written once — the algorithmic bytes.
// The workspace (header + granules, 64 KB) is zeroed once before its first
// use; tags are unique per launch and round, so nothing is re-armed.
//
// Unpack: per-word element counts -> block sums -> decode into LDS ->
// coalesced stores.
#include "gc_device.h"
#include "gc_host.h"

#include <algorithm>
#include <atomic>
#include <cstdlib>

#ifndef GC_STRICT_HANDOFF
#define GC_STRICT_HANDOFF 0
#endif
#ifndef GC_G4_STRICT  // 1: the release/acquire form of the table hand-off (see g1_store_granule)
#define GC_G4_STRICT GC_STRICT_HANDOFF
#endif
#ifndef GC_G4_STAMPS  // lab builds: per-block phase timestamps of round 0 behind the workspace's granules
#define GC_G4_STAMPS 0
#endif

namespace gc {

constexpr unsigned G4_THREADS = 512;                    // unpack blocks (256: 24.7 us, 512: 23.6, 1024: 33.5 on the ResNet50 xi words; profiles/r06af_g4u_block_threads_ab.json)
constexpr uint32_t G4_SEG = 32;                         // positions per table block
constexpr uint32_t G4_DEAD = 15;                        // table state: the chain has passed n
constexpr uint32_t G4_STATUS_RANGE = 1u, G4_STATUS_NOSPC = 2u, G4_STATUS_TIMEOUT = 4u;

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

// the mode classes of a 32-position block (bit p = position p), from the
// window masks W15 = some value >= 4 in [p, p+15), W7 = some value >= 16 in
// [p, p+7), W4 = some value >= 128 in [p, p+4).  W4 ⊆ W7 ⊆ W15, so the mode at
// p is W15[p] + W7[p] + W4[p] = 2 hi[p] + lo[p] with hi = W7 and
// lo = W15 ^ W7 ^ W4 (0: 15 x 2 bits, 1: 7 x 4, 2: 4 x 7, 3: 3 x 8).
struct G4Cls {
    uint32_t lo, hi;
};

// w: the block's 8 dwords of bytes + the next 4 (windows reach +14)
__device__ __forceinline__ G4Cls g4_classes(const uint32_t *w)
{
    constexpr int DW = G4_SEG / 4 + 4;
    uint64_t ge4 = 0, ge16 = 0, ge128 = 0;  // bit j: byte j
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

// the classes of a thread's 3 blocks from its 24 dwords + the 4 after: each
// dword's threshold flags computed once (the blocks' 16-byte windows overlap)
__device__ __forceinline__ void g4_classes3(const uint32_t (&w)[28], G4Cls (&c)[3])
{
    uint32_t m4[4] = {0, 0, 0, 0}, m16[4] = {0, 0, 0, 0}, m128[4] = {0, 0, 0, 0};  // bit j: position 32i + j
#pragma unroll
    for (int k = 0; k < 28; ++k) {
        m4[k >> 3] |= byte_flags(w[k], 0xfcfcfcfcu) << (4 * (k & 7));
        m16[k >> 3] |= byte_flags(w[k], 0xf0f0f0f0u) << (4 * (k & 7));
        m128[k >> 3] |= byte_flags(w[k], 0x80808080u) << (4 * (k & 7));
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // window ORs by doubling on (block i, block i + 1)
        const uint64_t ge4 = m4[i] | ((uint64_t)m4[i + 1] << 32), ge16 = m16[i] | ((uint64_t)m16[i + 1] << 32),
                       ge128 = m128[i] | ((uint64_t)m128[i + 1] << 32);
        const uint64_t a1 = ge4 | (ge4 >> 1), a2 = a1 | (a1 >> 2), a3 = a2 | (a2 >> 4);
        const uint64_t b1 = ge16 | (ge16 >> 1), b2 = b1 | (b1 >> 2);
        const uint64_t c1 = ge128 | (ge128 >> 1);
        const uint32_t w15 = (uint32_t)(a3 | (a3 >> 7)), w7 = (uint32_t)(b2 | (b2 >> 3)),
                       w4 = (uint32_t)(c1 | (c1 >> 2));
        c[i] = G4Cls{w15 ^ w7 ^ w4, w7};
    }
}

__device__ __forceinline__ uint32_t g4_mode(const G4Cls &c, uint32_t p)
{
    return (((c.hi >> p) & 1u) << 1) | ((c.lo >> p) & 1u);
}

// bit p of m as a lane mask (0 or ~0): one v_bfe_i32
__device__ __forceinline__ uint32_t bitmask(uint32_t m, int p) { return (uint32_t)__builtin_amdgcn_sbfe((int)m, p, 1); }

// one 32-position block's table by the backward recurrence
// f[p] = 1 word + f[p + cnt(p)]; a successor past the block is entry
// p + cnt - 32 of the NEXT block's table fn (identity for a thread's last
// block: the offset into the next thread's range).  All indices are static
// (the recurrence is unrolled), so f stays in registers; the successor is
// picked with three bitfield selects on the class bits.  TAIL: positions >=
// live are past n (the chain has ended there).
template <bool TAIL>
__device__ __forceinline__ void g4_dp(const G4Cls &c, uint32_t live, const uint32_t fn[15], uint32_t f[G4_SEG])
{
#pragma unroll
    for (int p = G4_SEG - 1; p >= 0; --p) {
        const uint32_t s3 = p + 3 < (int)G4_SEG ? f[(p + 3) % G4_SEG] : fn[(p + 3 - (int)G4_SEG) % 15];
        const uint32_t s4 = p + 4 < (int)G4_SEG ? f[(p + 4) % G4_SEG] : fn[(p + 4 - (int)G4_SEG) % 15];
        const uint32_t s7 = p + 7 < (int)G4_SEG ? f[(p + 7) % G4_SEG] : fn[(p + 7 - (int)G4_SEG) % 15];
        const uint32_t s15 = p + 15 < (int)G4_SEG ? f[(p + 15) % G4_SEG] : fn[(p + 15 - (int)G4_SEG) % 15];
        const uint32_t mlo = bitmask(c.lo, p), mhi = bitmask(c.hi, p);
        // mode 3: s3, 2: s4, 1: s7, 0: s15
        const uint32_t nx = (mhi & ((mlo & s3) | (~mlo & s4))) | (~mhi & ((mlo & s7) | (~mlo & s15)));
        if (TAIL)
            f[p] = (uint32_t)p < live ? nx + 16u : G4_DEAD;
        else
            f[p] = nx + 16u;
    }
}

// ---- one-pass pack ----------------------------------------------------------
constexpr unsigned G1_THREADS = 1024;
constexpr unsigned G1_WAVES = G1_THREADS / 64;            // 16
constexpr uint32_t G1_BLK = 3;                            // 32-position blocks per thread
constexpr uint32_t G1_RANGE = G4_SEG * G1_BLK;            // 96 positions per thread
constexpr uint32_t G1_TILE_MAX = G1_THREADS * G1_RANGE;   // 98,304 positions per block and round
constexpr uint32_t G1_GMAX = 256;                         // blocks of the persistent grid (<= one per CU)
constexpr uint32_t G1_MIN_TILE = 16384;                   // small buckets: fewer, larger tiles
constexpr uint64_t G1_TIMEOUT_TICKS = 1ull << 27;         // s_memrealtime (100 MHz): ~1.3 s, then status 4

// workspace: the header on a line of its own, then the granules (two round
// parities x G1_GMAX tiles x 16 entries x {entry, tag}), then (lab builds)
// the phase stamps
struct G1Hdr {
    uint64_t seq;           // tags used so far: round r of a launch tags seq + r + 1
    uint32_t done;          // blocks of the running launch that have finished (block 0 re-arms it)
    uint32_t tmo;           // nonzero: a block of the running launch timed out (block 0 re-arms it)
    uint64_t test_delay;    // tests only (tests/test_gpu_greedy4.py): block 0 starts this many ticks late
    uint64_t pad[29];
};
static_assert(sizeof(G1Hdr) == 256, "header size");
constexpr uint32_t G1_NSTAMP = 8;
constexpr uint64_t G1_WS_BYTES = sizeof(G1Hdr) + 2ull * G1_GMAX * 16 * 8 + (GC_G4_STAMPS ? G1_GMAX * G1_NSTAMP * 8 : 0);

// lab builds only: s_memrealtime (100 MHz) at a block's phase boundaries
#define G1_STAMP(i)                                                                                      \
    do {                                                                                                 \
        if (GC_G4_STAMPS && r == 0 && t == 0)                                                            \
            gran[2ull * G1_GMAX * 16 + (uint64_t)b * G1_NSTAMP + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)

struct G1Smem {
    alignas(16) uint32_t v[G1_TILE_MAX / 4 + 6];  // the tile's values as bytes + 16-byte halo (+ 8 bytes the word reads may touch)
    union {
        struct {
            uint32_t pl[G1_WAVES][63][8];         // per wave: the left children of its tree (u16 x 16 a row)
            union {
                uint32_t tr[G1_WAVES][32][8];     // per wave: right children of the level in flight
                uint32_t t0[G1_GMAX][16];         // the round's tile tables
            } u;
            uint32_t g4[G1_GMAX / 4][16];         // compositions of 4 / 16 / 64 tiles
            uint32_t g16[G1_GMAX / 16][16];
            uint32_t g64[G1_GMAX / 64][16];
            uint32_t x[32][16];                   // the tree of the 16 wave roots (nodes 1..31)
        } k;
        uint16_t wl[G1_WAVES / 2][64 * G1_RANGE / 3 + 4];  // emission, a big tile: half the waves' lists at a time
        uint16_t wlb[1];                          // emission: the block's word list (G1_WLCAP entries)
    };
    uint64_t wbase[G1_WAVES];                     // each wave's first word (absolute)
    uint32_t wcnt[G1_WAVES];                      // each wave's words
    uint32_t woff[G1_WAVES];                      // each wave's first word within the tile
    uint64_t base_b;                              // the block's word base within the round
    uint32_t s_b, s_end, tw, tile_words;
    uint32_t stage[G1_WAVES / 4];                 // STAGE: per quarter, its waves whose first batch is in (4 a round)
};
// entries of the block's word list: the tree storage, free by then
constexpr uint32_t G1_WLCAP = (uint32_t)(sizeof(((G1Smem *)nullptr)->k) / 2);

// the waves of a workgroup run one LDS tree each: order a wave's LDS stores
// before its later loads of other lanes' rows (LDS executes a wave's
// instructions in order; this keeps the compiler from moving them)
__device__ __forceinline__ void wave_lds_sync()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t g1_apply(uint32_t x, uint32_t &s)  // table entry -> words, new state
{
    s = x & 15u;
    return x >> 4;
}

// The hand-off of the round's tile tables: MI355X_MICROARCH.md's data-tagged
// granules (cdna_hip_programming.md Guideline 16, R2): every table entry is
// one 8-byte {entry, tag} granule written by ONE sc1 store; readers re-read
// with sc1 loads until every tag matches.  No flag, no counter, no fence.
// Tags are unique per (launch, round) (G1Hdr::seq), so nothing is re-armed.
// GC_G4_STRICT: the memory model's own message passing instead — the entry
// and tag as a release store of the whole granule, acquire loads — for builds
// that must not rely on the observed untorn sc1 granule.
__device__ __forceinline__ void g1_store_granule(uint64_t *p, uint64_t v)
{
#if GC_G4_STRICT
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
#else
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

__device__ __forceinline__ uint64_t g1_load_granule(const uint64_t *p)
{
#if GC_G4_STRICT
    return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
#else
    return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

template <uint32_t V>
struct G1Count {
    static constexpr uint32_t value = V;
};

// The bytes of wave w's ranges (positions 96 * 64 w .. + 6144, and the 16
// after them: the next range's head) into LDS by that wave alone, so a wave
// starts its recurrence as soon as its own data is in, while the other waves'
// loads are still in flight (the block-wide load and its barrier: 42.9 us per
// pack at 23.5 M; per wave: 42.1 us, profiles/r05zn_g4_shapes.csv).  Returns this lane's OR of the values read
// (the range check: > 255 means a value outside [0, 255]); the caller ORs it
// over the block at its next barrier.  Two batches of up to 13 / 12 int4
// loads per lane, all of a batch issued before any is used.
// STAGE: the tile is loaded by quarters (waves 4k .. 4k + 3, one per SIMD).
// Quarter k issues its loads once quarter k - 1's first batches are in (an LDS
// count per quarter and round), so the quarters' data arrives one after
// another and quarter k's recurrence runs while quarters > k still load;
// unstaged, every wave's loads went out at once and all finished together,
// near the end of the 13 us load.  Each quarter keeps ~100 KB in flight per
// CU (its second batches + the next quarter's first), above what the CU's
// share of HBM needs.  Groups of 2 or 8 waves, or the hand-on after a wave's
// last batch, or batches of 9 / 8 / 8 were slower (41.0 / 40.2 / 40.5 /
// 39.1-39.5 against 38.4-38.5 us; issue priorities by quarter (s_setprio)
// instead of the count: 40.8, no change).  The wait is bounded: it orders
// the loads and nothing else depends on it.
template <bool ALIGNED, bool STAGE>
__device__ __forceinline__ uint32_t g1_load_wave(G1Smem &sm, const int32_t *__restrict__ src, uint64_t n,
                                                 uint64_t start, uint32_t C, unsigned w, unsigned lane,
                                                 uint32_t target)
{
    typedef int i4v __attribute__((ext_vector_type(4)));
    constexpr uint32_t WQ = G1_RANGE / 4 * 64;  // dwords of a wave's ranges (1536)
    const uint32_t QT = C / 4, qb = WQ * w;
    uint32_t bad = 0;
    const uint32_t quarter = w / 4;
    auto signal = [&] {  // this wave's first batch is in: the next quarter may issue
        if (STAGE && lane == 0)
            __hip_atomic_fetch_add(&sm.stage[quarter], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    if (STAGE && quarter > 0) {  // a performance hint only: bounded, so a late quarter never waits forever
        for (uint32_t it = 0; it < 4096; ++it) {
            const uint32_t c = __hip_atomic_load(&sm.stage[quarter - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (__builtin_amdgcn_readfirstlane(c) >= target)
                break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (qb >= QT) {
        signal();
        return 0;  // no positions in this wave (wave-uniform)
    }
    const uint32_t qe = min(qb + WQ, QT) + 4u;  // + the 16-position halo
    auto batch = [&](uint32_t j0, auto NJ) {
        constexpr uint32_t J = decltype(NJ)::value;
        int4 v[J];
        const uint32_t q0 = qb + 64u * j0;
        const bool full = ALIGNED && q0 + 64u * J <= qe && start + 4ull * (q0 + 64u * J) <= n;
        if (full) {  // uniform: every load in bounds
#pragma unroll
            for (uint32_t j = 0; j < J; ++j) {
                const i4v r = __builtin_nontemporal_load(reinterpret_cast<const i4v *>(src + start) + q0 + 64u * j + lane);
                v[j] = make_int4(r.x, r.y, r.z, r.w);
            }
        } else {
#pragma unroll
            for (uint32_t j = 0; j < J; ++j) {
                const uint32_t q = q0 + 64u * j + lane;
                const uint64_t g = start + 4ull * q;
                int4 r = make_int4(0, 0, 0, 0);
                if (q < qe) {
                    if (ALIGNED && g + 4 <= n)
                        r = *reinterpret_cast<const int4 *>(src + g);
                    else if (g < n) {
                        r.x = src[g];
                        r.y = g + 1 < n ? src[g + 1] : 0;
                        r.z = g + 2 < n ? src[g + 2] : 0;
                        r.w = g + 3 < n ? src[g + 3] : 0;
                    }
                }
                v[j] = r;
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < J; ++j) {
            const uint32_t q = q0 + 64u * j + lane;
            if (q < qe) {
                bad |= (uint32_t)v[j].x | (uint32_t)v[j].y | (uint32_t)v[j].z | (uint32_t)v[j].w;
                sm.v[q] = __builtin_amdgcn_perm(__builtin_amdgcn_perm(v[j].w, v[j].z, 0x0c0c0400u),
                                                __builtin_amdgcn_perm(v[j].y, v[j].x, 0x0c0c0400u), 0x05040100u);
            }
        }
    };
    static_assert(64 * (13 + 12) >= WQ + 4, "two batches cover a wave's ranges and the halo");
    batch(0, G1Count<13>{});
    signal();
    if (qb + 64u * 13 < qe)  // wave-uniform
        batch(13, G1Count<12>{});
    wave_lds_sync();  // the wave's lanes read each other's bytes
    return bad;
}

// pack one word of mode `mode` from the bytes at tile offset a (zero past n).
// Per mode a SWAR form over the 16 bytes from a; `pres` (bit m: some lane of
// the wave packs a mode-m word, wave-uniform) skips the forms no lane needs.
//   mode 0 (15 x 2 bits): per dword (x * 0x40100401) >> 24 = b0 b1 b2 b3 as
//          2-bit fields, b0 on top (no two product terms share a bit);
//   mode 1 (7 x 4 bits):  per dword (x << 4 | x >> 8) holds b0b1 / b2b3 in
//          bytes 0 / 2, one perm joins them;
//   mode 2 (4 x 7 bits):  byte-swap, then 8 -> 7 -> 14-bit field merges;
//   mode 3 (3 x 8 bits):  one perm.
__device__ __forceinline__ uint32_t g1_word(const G1Smem &sm, uint32_t a, uint32_t mode, uint32_t pres)
{
    // three aligned 8-byte reads cover bytes a .. a + 15 (64 banks for 8-byte
    // reads: consecutive lanes' words stay conflict-free; 4-byte reads use 32)
    typedef uint32_t u2v __attribute__((ext_vector_type(2)));
    typedef __attribute__((address_space(3))) const volatile u2v lds_u2v;  // whole ds_read_b64s
    lds_u2v *d = (lds_u2v *)(&sm.v[(a >> 2) & ~1u]);
    const u2v p0 = d[0], p1 = d[1], p2 = d[2];
    const bool odd = (a >> 2) & 1u;
    const uint32_t sh = a & 3u;
    const uint32_t u0 = odd ? p0.y : p0.x, u1 = odd ? p1.x : p0.y, u2 = odd ? p1.y : p1.x, u3 = odd ? p2.x : p1.y,
                   u4 = odd ? p2.y : p2.x;
    const uint32_t x0 = __builtin_amdgcn_alignbyte(u1, u0, sh);
    uint32_t code = 0;
    if (pres & 3u) {
        const uint32_t x1 = __builtin_amdgcn_alignbyte(u2, u1, sh);
        if (pres & 1u) {
            const uint32_t x2 = __builtin_amdgcn_alignbyte(u3, u2, sh);
            const uint32_t x3 = __builtin_amdgcn_alignbyte(u4, u3, sh) & 0x00ffffffu;  // b15 is not in the word
            constexpr uint32_t M = 0x40100401u;
            const uint32_t c0 = ((x0 * M) >> 24 << 22) | ((x1 * M) >> 24 << 14) | ((x2 * M) >> 24 << 6) |
                                ((x3 * M) >> 26);
            code = mode == 0 ? c0 : code;
        }
        if (pres & 2u) {
            const uint32_t x1m = x1 & 0x00ffffffu;  // b7 is not in the word
            const uint32_t y0 = (x0 << 4) | (x0 >> 8), y1 = (x1m << 4) | (x1m >> 8);
            const uint32_t h0 = __builtin_amdgcn_perm(y0, y0, 0x0c0c0002u), h1 = __builtin_amdgcn_perm(y1, y1, 0x0c0c0002u);
            const uint32_t c1 = 0x40000000u | (h0 << 14) | (h1 >> 2);
            code = mode == 1 ? c1 : code;
        }
    }
    if (pres & 4u) {
        const uint32_t r = __builtin_amdgcn_perm(x0, x0, 0x00010203u);  // b0 << 24 | b1 << 16 | b2 << 8 | b3
        const uint32_t uu = (r & 0x007f007fu) | ((r >> 1) & 0x3f803f80u);
        const uint32_t v = (uu & 0x3fffu) | ((uu >> 2) & 0x0fffc000u);
        const uint32_t c2 = 0x80000000u | (v << 2);
        code = mode == 2 ? c2 : code;
    }
    if (pres & 8u) {
        const uint32_t c3 = 0xc0000000u | (__builtin_amdgcn_perm(x0, x0, 0x0c000102u) << 6);
        code = mode == 3 ? c3 : code;
    }
    return code;
}

__device__ __forceinline__ uint32_t g1_modes_present(uint32_t mode, bool active)
{
    return (__builtin_amdgcn_ballot_w64(active && mode == 0) ? 1u : 0u) |
           (__builtin_amdgcn_ballot_w64(active && mode == 1) ? 2u : 0u) |
           (__builtin_amdgcn_ballot_w64(active && mode == 2) ? 4u : 0u) |
           (__builtin_amdgcn_ballot_w64(active && mode == 3) ? 8u : 0u);
}

// Persistent pack.  Grid: G <= one block per CU (the LDS image admits one);
// every block runs all R rounds.  A block waits only for blocks of its own
// launch; one not yet resident gets a CU once another kernel's blocks leave.
// A wait longer than G1_TIMEOUT_TICKS ends the call with status 4.
template <bool ALIGNED, bool STAGE>
__global__ __launch_bounds__(G1_THREADS) void k_g4p_one(const int32_t *__restrict__ src, uint64_t n, uint32_t C,
                                                        uint32_t R, int32_t *__restrict__ out, uint64_t cap,
                                                        uint64_t *__restrict__ nwords, uint32_t *__restrict__ status,
                                                        G1Hdr *__restrict__ hdr, uint64_t *__restrict__ gran)
{
    __shared__ G1Smem sm;
    const unsigned tid = threadIdx.x;
    const uint32_t b = blockIdx.x, G = gridDim.x;
    if (b == 0) {  // the late-block test hook (0 in every product workspace)
        const uint64_t d = hdr->test_delay;
        if (d) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() - t0 < d)
                __builtin_amdgcn_s_sleep(127);
        }
    }
    // every block reads seq before its round-0 granules exist; block 0 moves
    // it on only after it has read every block's round-0 granules
    const uint64_t seq = __hip_atomic_load(&hdr->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t carry_s = 0, bad_all = 0, nospc = 0, tmo = 0;
    uint64_t carry_base = 0;
    if (STAGE) {
        if (tid < G1_WAVES / 4)
            sm.stage[tid] = 0;
        __syncthreads();
    }
    for (uint32_t r = 0; r < R; ++r) {
        // the thread index re-made opaque each round, so the many per-thread
        // LDS and global offsets are not hoisted out of the round loop (they
        // would hold ~60 VGPRs across the whole body)
        unsigned t;
        asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(tid));
        const unsigned lane = t & 63u, w = t >> 6;
        const uint64_t tile_start = ((uint64_t)r * G + b) * C;
        const uint32_t tag = (uint32_t)(seq + r + 1);
        G1_STAMP(0);
        // 1. this wave's bytes (the range check is ORed over the block below)
        const uint32_t badw = g1_load_wave<ALIGNED, STAGE>(sm, src, n, tile_start, C, w, lane, 4u * (r + 1));
        G1_STAMP(1);
        // 2. this thread's table over its 96 positions (identity past the tile)
        const bool in_tile = G1_RANGE * t < C;
        const uint64_t r0 = tile_start + G1_RANGE * t;
        const uint32_t live = r0 >= n ? 0u : (uint32_t)std::min<uint64_t>(G1_RANGE, n - r0);
        G4Cls cls[G1_BLK];
        uint32_t h[8];
        if (in_tile) {
            {  // 7 x 16-byte LDS reads (2-way bank conflicts at this 96-byte stride)
                uint32_t wv[G1_RANGE / 4 + 4];
#pragma unroll
                for (uint32_t j = 0; j < G1_RANGE / 4 + 4; j += 4) {  // volatile: kept whole (split into
                    // ds_read2_b32 pairs they were 8-way conflicts on 32 banks at this stride)
                    typedef uint32_t u4v __attribute__((ext_vector_type(4)));
                    typedef __attribute__((address_space(3))) const volatile u4v lds_u4v;
                    const u4v r = *(lds_u4v *)(&sm.v[G1_RANGE / 4 * t + j]);
                    wv[j] = r.x;
                    wv[j + 1] = r.y;
                    wv[j + 2] = r.z;
                    wv[j + 3] = r.w;
                }
                g4_classes3(wv, cls);
            }
            uint32_t fn[15];
#pragma unroll
            for (uint32_t q = 0; q < 15; ++q)
                fn[q] = q;
#pragma unroll
            for (int k = G1_BLK - 1; k >= 0; --k) {  // the blocks back to front, each one's table chained on
                uint32_t f[G4_SEG];
                g4_dp<false>(cls[k], G4_SEG, fn, f);  // n is handled below, for the one thread that holds it
#pragma unroll
                for (uint32_t q = 0; q < 15; ++q)
                    fn[q] = f[q];
            }
#pragma unroll
            for (uint32_t e = 0; e < 7; ++e)
                h[e] = fn[2 * e] | (fn[2 * e + 1] << 16);
            h[7] = fn[14] | (G4_DEAD << 16);
        } else {
#pragma unroll
            for (uint32_t k = 0; k < G1_BLK; ++k)
                cls[k] = G4Cls{0, 0};
#pragma unroll
            for (uint32_t e = 0; e < 8; ++e)
                h[e] = (2 * e) | ((2 * e + 1) << 16);
        }
        // the thread whose range holds position n: its chains end there, so
        // every entry is DEAD with the words that start before n.  Entry e is
        // walked by lane e of its wave (the class bits read from its lane);
        // ranges past it keep their tables, which a DEAD state passes through.
        if (n >= tile_start && n < tile_start + C) {  // block-uniform: the tile that holds n
            const uint32_t ts = (uint32_t)((n - tile_start) / G1_RANGE), nlive = (uint32_t)(n - tile_start) - G1_RANGE * ts;
            if (w == (ts >> 6)) {  // wave-uniform
                const int sl = (int)(ts & 63u);
                G4Cls sc[G1_BLK];
#pragma unroll
                for (uint32_t k = 0; k < G1_BLK; ++k)
                    sc[k] = G4Cls{(uint32_t)__builtin_amdgcn_readlane((int)cls[k].lo, sl),
                                  (uint32_t)__builtin_amdgcn_readlane((int)cls[k].hi, sl)};
                uint32_t pos = lane, words = 0;
                if (lane < 15) {
                    while (pos < nlive) {
                        const uint32_t k = pos >> 5;  // masks, not a select (that became a scratch array)
                        const uint32_t m0 = 0u - (k == 0), m1 = 0u - (k == 1), m2 = 0u - (k == 2);
                        const G4Cls c{(sc[0].lo & m0) | (sc[1].lo & m1) | (sc[2].lo & m2),
                                      (sc[0].hi & m0) | (sc[1].hi & m1) | (sc[2].hi & m2)};
                        pos += g4_cnt(g4_mode(c, pos & 31u));
                        ++words;
                    }
                }
                const uint32_t ent = G4_DEAD | (words << 4);
                uint32_t hs[8];
#pragma unroll
                for (uint32_t e = 0; e < 7; ++e)
                    hs[e] = (uint32_t)__builtin_amdgcn_readlane((int)ent, 2 * e) |
                            ((uint32_t)__builtin_amdgcn_readlane((int)ent, 2 * e + 1) << 16);
                hs[7] = (uint32_t)__builtin_amdgcn_readlane((int)ent, 14) | (G4_DEAD << 16);
                if (lane == (unsigned)sl) {
#pragma unroll
                    for (uint32_t e = 0; e < 8; ++e)
                        h[e] = hs[e];
                }
            }
        }
#if GC_G4_STAMPS
        __syncthreads();
        G1_STAMP(2);
#endif
        // 3. the wave's tree: node 64 + lane = this thread's table; even
        // nodes (left children) kept in pl[w][node / 2 - 1], odd ones only
        // while their level is composed (tr[w][index among the level's odd])
        {
            uint32_t *row = (lane & 1u) ? sm.k.u.tr[w][lane >> 1] : sm.k.pl[w][31 + (lane >> 1)];
            reinterpret_cast<uint4 *>(row)[0] = make_uint4(h[0], h[1], h[2], h[3]);
            reinterpret_cast<uint4 *>(row)[1] = make_uint4(h[4], h[5], h[6], h[7]);
        }
        wave_lds_sync();
#pragma unroll
        for (uint32_t m = 32; m >= 1; m >>= 1) {  // parents [m, 2m); a task = (parent, entry pair)
            constexpr uint32_t RMAX = 4;
            uint32_t res[RMAX];
#pragma unroll
            for (uint32_t rr = 0; rr < RMAX; ++rr) {
                const uint32_t task = lane + 64 * rr;
                if (task < 8 * m) {
                    const uint32_t p = m + (task >> 3), pr = task & 7u;
                    const uint32_t xx = sm.k.pl[w][p - 1][pr];
                    const uint16_t *rt = reinterpret_cast<const uint16_t *>(sm.k.u.tr[w][p - m]);
                    const uint32_t x0 = xx & 0xffffu, x1 = xx >> 16;
                    res[rr] = ((x0 & ~15u) + rt[x0 & 15u]) | (((x1 & ~15u) + rt[x1 & 15u]) << 16);
                }
            }
            wave_lds_sync();
#pragma unroll
            for (uint32_t rr = 0; rr < RMAX; ++rr) {
                const uint32_t task = lane + 64 * rr;
                if (task < 8 * m) {
                    const uint32_t p = m + (task >> 3), pr = task & 7u;
                    if (m == 1) {  // the wave root -> leaf 16 + w of the block's tree (u32 entries)
                        sm.k.x[16 + w][2 * pr] = res[rr] & 0xffffu;
                        sm.k.x[16 + w][2 * pr + 1] = res[rr] >> 16;
                    } else if ((p & 1u) == 0) {
                        sm.k.pl[w][p / 2 - 1][pr] = res[rr];
                    } else {
                        sm.k.u.tr[w][(p - 1) / 2 - m / 2][pr] = res[rr];
                    }
                }
            }
            wave_lds_sync();
        }
        const uint32_t bad = __syncthreads_or(badw > 255u);
        // 4. the block's tree over the wave roots (wave 0) -> x[1], published
        if (w == 0) {
#pragma unroll
            for (uint32_t m = 8; m >= 1; m >>= 1) {
                uint32_t res[2];
#pragma unroll
                for (uint32_t rr = 0; rr < 2; ++rr) {
                    const uint32_t task = lane + 64 * rr;
                    if (task < 16 * m) {
                        const uint32_t p = m + (task >> 4), e = task & 15u;
                        const uint32_t xv = sm.k.x[2 * p][e];
                        res[rr] = (xv & ~15u) + sm.k.x[2 * p + 1][xv & 15u];
                    }
                }
                wave_lds_sync();
#pragma unroll
                for (uint32_t rr = 0; rr < 2; ++rr) {
                    const uint32_t task = lane + 64 * rr;
                    if (task < 16 * m)
                        sm.k.x[m + (task >> 4)][task & 15u] = res[rr];
                }
                wave_lds_sync();
            }
            if (lane < 16)  // bit 31 of each entry: this tile holds a value outside [0, 255]
                g1_store_granule(&gran[((uint64_t)(r & 1u) * G1_GMAX + b) * 16 + lane],
                                 (uint64_t)(sm.k.x[1][lane] | (bad << 31)) | ((uint64_t)tag << 32));
        }
        G1_STAMP(3);
        // 5. every tile's table: thread t re-reads granules t, t + 1024, ...
        // (tile i, entry e = index / 16, index % 16) until every tag matches
        uint32_t rbad = 0;
        {
            const uint64_t *gr = gran + (uint64_t)(r & 1u) * G1_GMAX * 16;
            constexpr uint32_t NG = G1_GMAX * 16 / G1_THREADS;  // 4
            uint64_t g[NG];
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                bool ok = true;
#pragma unroll
                for (uint32_t j = 0; j < NG; ++j) {
                    const uint32_t i = t + j * G1_THREADS;
                    if (i < 16 * G && !tmo) {
                        g[j] = g1_load_granule(&gr[i]);
                        ok &= (uint32_t)(g[j] >> 32) == tag;
                    }
                }
                if (__builtin_amdgcn_ballot_w64(!ok) == 0)  // wave-uniform exit
                    break;
                __builtin_amdgcn_s_sleep(2);
                if (__builtin_amdgcn_s_memrealtime() - t0 > G1_TIMEOUT_TICKS) {
                    tmo = 1;
                    break;
                }
            }
#pragma unroll
            for (uint32_t j = 0; j < NG; ++j) {
                const uint32_t i = t + j * G1_THREADS;
                uint32_t a = i & 15u;  // identity past the grid
                if (i < 16 * G && !tmo) {
                    rbad |= (uint32_t)g[j] >> 31;
                    a = (uint32_t)g[j] & 0x7fffffffu;
                }
                sm.k.u.t0[i >> 4][i & 15u] = a;
            }
        }
        rbad = __syncthreads_or(rbad);
        tmo = __syncthreads_or(tmo);
        G1_STAMP(4);
        if (r == 0 && b == 0 && t == 0)  // every block has read seq: the next launch tags on from here
            __hip_atomic_store(&hdr->seq, seq + R, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        {  // compositions of 4 tiles (thread (k, e), k < 64)
            const uint32_t k = t >> 4, e = t & 15u;
            uint32_t c = sm.k.u.t0[4 * k][e];
#pragma unroll
            for (uint32_t j = 1; j < 4; ++j)
                c = (c & ~15u) + sm.k.u.t0[4 * k + j][c & 15u];
            sm.k.g4[k][e] = c;
        }
        __syncthreads();
        if (t < 256) {
            const uint32_t k = t >> 4, e = t & 15u;
            uint32_t c = sm.k.g4[4 * k][e];
#pragma unroll
            for (uint32_t j = 1; j < 4; ++j)
                c = (c & ~15u) + sm.k.g4[4 * k + j][c & 15u];
            sm.k.g16[k][e] = c;
        }
        __syncthreads();
        if (t < 64) {
            const uint32_t k = t >> 4, e = t & 15u;
            uint32_t c = sm.k.g16[4 * k][e];
#pragma unroll
            for (uint32_t j = 1; j < 4; ++j)
                c = (c & ~15u) + sm.k.g16[4 * k + j][c & 15u];
            sm.k.g64[k][e] = c;
        }
        __syncthreads();
        if (t == 0) {  // the block's entry and word base; the round's exit and total
            uint32_t s = carry_s, base = 0;
            const uint32_t i3 = b >> 6, i2 = (b >> 4) & 3u, i1 = (b >> 2) & 3u, i0 = b & 3u;
            for (uint32_t j = 0; j < i3; ++j)
                base += g1_apply(sm.k.g64[j][s], s);
            for (uint32_t j = 0; j < i2; ++j)
                base += g1_apply(sm.k.g16[4 * i3 + j][s], s);
            for (uint32_t j = 0; j < i1; ++j)
                base += g1_apply(sm.k.g4[16 * i3 + 4 * i2 + j][s], s);
            for (uint32_t j = 0; j < i0; ++j)
                base += g1_apply(sm.k.u.t0[64 * i3 + 16 * i2 + 4 * i1 + j][s], s);
            sm.s_b = s;
            sm.base_b = base;
            sm.tile_words = sm.k.x[1][s] >> 4;
            uint32_t se = carry_s, tw = 0;
            for (uint32_t j = 0; j < G1_GMAX / 64; ++j)
                tw += g1_apply(sm.k.g64[j][se], se);
            sm.s_end = se;
            sm.tw = tw;
        }
        __syncthreads();
        bad_all |= rbad;
        const uint64_t round_end = carry_base + sm.tw;
        if (round_end > cap)
            nospc = 1;
        const bool emit = !bad_all && !nospc && !tmo;
        // 6. this thread's entry and word base: down the block's tree, then the wave's
        uint32_t s = sm.s_b;
        uint64_t base = carry_base + sm.base_b;
        if (emit) {
            uint32_t node = 1;
#pragma unroll
            for (int d = 3; d >= 0; --d) {
                const uint32_t bit = (w >> d) & 1u;
                if (bit)
                    base += g1_apply(sm.k.x[2 * node][s], s);
                node = 2 * node + bit;
            }
            if (lane == 0) {
                sm.wbase[w] = base;
                sm.woff[w] = (uint32_t)(base - carry_base - sm.base_b);
            }
            const uint32_t xw = sm.k.x[16 + w][s];  // the wave's words from its entry
            if (lane == 0)
                sm.wcnt[w] = xw >> 4;
            node = 1;
#pragma unroll
            for (int d = 5; d >= 0; --d) {
                const uint32_t bit = (lane >> d) & 1u;
                if (bit)
                    base += g1_apply(reinterpret_cast<const uint16_t *>(sm.k.pl[w][node - 1])[s], s);
                node = 2 * node + bit;
            }
        }
        G1_STAMP(5);
        // 7. the words: each thread lists its word starts (position in its
        // wave's range | mode << 14) from its class bits, then every lane of
        // the block packs listed words, consecutive lanes consecutive words,
        // from the LDS bytes.  A tile of more than G1_WLCAP words (values
        // mostly >= 128) lists half its waves at a time.
        if (emit) {
            __syncthreads();  // the trees are no longer read
            const uint32_t tw_tile = sm.tile_words;
            if (tw_tile <= G1_WLCAP) {
                if (in_tile) {
                    uint32_t pos = s, j = sm.woff[w] + (uint32_t)(base - sm.wbase[w]);  // DEAD (15) past n
#pragma unroll
                    for (uint32_t k = 0; k < G1_BLK; ++k) {  // block by block: the class bits indexed statically
                        const uint32_t end = std::min<uint32_t>(live, G4_SEG * (k + 1));
                        while (pos < end) {
                            const uint32_t mode = g4_mode(cls[k], pos & 31u);
                            sm.wlb[j++] = (uint16_t)((G1_RANGE * lane + pos) | (mode << 14));
                            pos += g4_cnt(mode);
                        }
                    }
                }
                __syncthreads();
                const uint64_t ob = carry_base + sm.base_b;
                for (uint32_t k0 = 0; k0 < tw_tile; k0 += G1_THREADS) {
                    const uint32_t k = k0 + t;
                    const bool act = k < tw_tile;
                    const uint32_t ent = act ? sm.wlb[k] : 0u;
                    uint32_t wv = 0;  // the last wave whose first word is <= k
#pragma unroll
                    for (uint32_t st = G1_WAVES / 2; st >= 1; st >>= 1)
                        wv += sm.woff[wv + st] <= k ? st : 0u;
                    const uint32_t mode = ent >> 14;
                    const uint32_t code = g1_word(sm, 64 * G1_RANGE * wv + (ent & 0x3fffu), mode,
                                                  g1_modes_present(mode, act));
                    if (act)
                        out[ob + k] = (int32_t)code;
                }
            } else {
#pragma unroll 1
                for (uint32_t half = 0; half < 2; ++half) {
                    if (half)
                        __syncthreads();  // the first half's lists are packed
                    if ((w >> 3) == half && in_tile) {
                        uint16_t *wl = sm.wl[w & 7u];
                        uint32_t pos = s, j = (uint32_t)(base - sm.wbase[w]);
#pragma unroll
                        for (uint32_t k = 0; k < G1_BLK; ++k) {
                            const uint32_t end = std::min<uint32_t>(live, G4_SEG * (k + 1));
                            while (pos < end) {
                                const uint32_t mode = g4_mode(cls[k], pos & 31u);
                                wl[j++] = (uint16_t)((G1_RANGE * lane + pos) | (mode << 14));
                                pos += g4_cnt(mode);
                            }
                        }
                    }
                    __syncthreads();
                    const uint32_t L = w & 7u, wv = 8 * half + L;  // two waves per list
                    const uint32_t cnt = sm.wcnt[wv];
                    const uint64_t ob = sm.wbase[wv];
                    const uint16_t *wl = sm.wl[L];
                    for (uint32_t k0 = (w >> 3) * 64; k0 < cnt; k0 += 128) {
                        const uint32_t k = k0 + lane;
                        const bool act = k < cnt;
                        const uint32_t ent = act ? wl[k] : 0u;
                        const uint32_t mode = ent >> 14;
                        const uint32_t code = g1_word(sm, 64 * G1_RANGE * wv + (ent & 0x3fffu), mode,
                                                      g1_modes_present(mode, act));
                        if (act)
                            out[ob + k] = (int32_t)code;
                    }
                }
            }
        }
        carry_s = sm.s_end;
        carry_base = round_end;
        __syncthreads();  // the next round rewrites the LDS image and the trees
        G1_STAMP(6);
    }
    // The status: the range and capacity flags are the same in every block
    // (from the shared tables), a timeout is per block (block 0
    // alone reported its own, so a block that timed out and wrote none of its
    // words went unseen).  Every block ORs its timeout into hdr->tmo, then
    // counts itself done; block 0 waits (bounded) for all G, reports, and
    // re-arms both for the next launch.  A block that never finishes within the
    // bound is a timeout too (the workspace must then be zeroed again).
    if (tid == 0) {
        if (tmo)
            __hip_atomic_fetch_or(&hdr->tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&hdr->done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (b == 0 && tid == 0) {
        uint32_t late = 0;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(&hdr->done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < G) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > G1_TIMEOUT_TICKS) {
                late = 1;
                break;
            }
        }
        const uint32_t any_tmo = __hip_atomic_load(&hdr->tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | late;
        __hip_atomic_store(&hdr->tmo, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&hdr->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *nwords = carry_base;
        *status = (bad_all ? G4_STATUS_RANGE : 0u) | (nospc ? G4_STATUS_NOSPC : 0u) |
                  ((tmo | any_tmo) ? G4_STATUS_TIMEOUT : 0u);
    }
}

// n == 0: the result pair only
__global__ void k_g4p_empty(uint64_t *nwords, uint32_t *status)
{
    *nwords = 0;
    *status = 0;
}

// ---- unpack ---------------------------------------------------------------
constexpr uint32_t G4U_PER_THREAD = 4;
constexpr uint32_t G4U_BLOCK_WORDS = G4_THREADS * G4U_PER_THREAD;  // 2048 words -> <= 30720 values

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
// up to this many unpack blocks (8 M words) each emit block sums the block
// totals itself (k_g4u_emit_nb: <= 8 loads per thread from L2) instead of a
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

// the block's tot staged values (bytes, obuf) to dst as int32, consecutive
// lanes consecutive values (4-byte stores: the 16-byte forms, nontemporal or
// not, and direct stores without the LDS staging measured slower)
__device__ __forceinline__ void g4u_store_values(const uint8_t *obuf, uint32_t tot, int32_t *__restrict__ dst,
                                                 uint32_t t)
{
    for (uint32_t k = t; k < tot; k += G4_THREADS)
        dst[k] = (int32_t)obuf[k];
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
    g4u_store_values(obuf, tot, out + bbase[blockIdx.x], threadIdx.x);
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
    g4u_store_values(obuf, tot, out + base, t);
}

// unpack workspace layout (bytes, 256-aligned pieces)
struct G4Ws {
    uint32_t *bsum;
    uint64_t *bbase;
};

static inline uint64_t al256(uint64_t b) { return (b + 255) & ~255ull; }

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

// compute units of the stream's device (cached per device): the persistent
// pack's grid is at most one block per CU
static uint32_t g1_cus(hipStream_t st)
{
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipStreamGetDevice(st, &dev) != hipSuccess && hipGetDevice(&dev) != hipSuccess)
        dev = 0;
    if (dev < 0 || dev >= 64)
        dev = 0;
    int c = cache[dev].load(std::memory_order_relaxed);
    if (c <= 0) {
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
            c = 1;
        cache[dev].store(c, std::memory_order_relaxed);
    }
    return (uint32_t)c;
}

// the staged tile load (k_g4p_one<…, STAGE>): 38.4-38.5 against 40.5 us per
// xi pack at 23.5 M, 32.8 against 34.8 us for the sign bits
// (profiles/r05zp_g4_stage.log).  GC_G4_STAGE=0 selects the unstaged form (A/B)
static bool greedy4_stage()
{
    static const bool on = [] {
        const char *e = getenv("GC_G4_STAGE");
        return !(e && atol(e) == 0);
    }();
    return on;
}

// the pack's geometry for n positions on `cus` CUs: G blocks, R rounds, C
// positions per tile (a multiple of 96, <= G1_TILE_MAX), G * R * C >= n
struct G1Geom {
    uint32_t G, R, C;
};

static G1Geom g1_geom(uint64_t n, uint32_t cus)
{
    G1Geom g{};
    const uint64_t gmax = std::min<uint64_t>(std::min<uint32_t>(cus, G1_GMAX), (n + G1_MIN_TILE - 1) / G1_MIN_TILE);
    g.G = (uint32_t)std::max<uint64_t>(1, gmax);
    const uint64_t per_round = (uint64_t)g.G * G1_TILE_MAX;
    g.R = (uint32_t)std::max<uint64_t>(1, (n + per_round - 1) / per_round);
    const uint64_t per_tile = (n + (uint64_t)g.G * g.R - 1) / ((uint64_t)g.G * g.R);
    g.C = (uint32_t)std::max<uint64_t>(G1_RANGE, (per_tile + G1_RANGE - 1) / G1_RANGE * G1_RANGE);
    return g;
}

}  // namespace gc

using namespace gc;

extern "C" {

size_t gc_greedy4_workspace_size(uint64_t n)
{
    (void)n;
    return (size_t)G1_WS_BYTES;
}

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
    if (n == 0) {
        hipLaunchKernelGGL(k_g4p_empty, dim3(1), dim3(1), 0, st, nwords, status);
        return launch_status("gc_greedy4_pack_device");
    }
    const G1Geom g = g1_geom(n, g1_cus(st));
    G1Hdr *hdr = reinterpret_cast<G1Hdr *>(workspace);
    uint64_t *gran = reinterpret_cast<uint64_t *>(reinterpret_cast<char *>(workspace) + sizeof(G1Hdr));
    const bool al = aligned16(src), stg = greedy4_stage();
    auto kern = al ? (stg ? k_g4p_one<true, true> : k_g4p_one<true, false>)
                   : (stg ? k_g4p_one<false, true> : k_g4p_one<false, false>);
    hipLaunchKernelGGL(kern, dim3(g.G), dim3(G1_THREADS), 0, st, src, n, g.C, g.R, out, cap, nwords, status, hdr,
                       gran);
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
    hipLaunchKernelGGL(k_g4p_empty, dim3(1), dim3(1), 0, st, count, status);
    if (nwords == 0)
        return launch_status("gc_greedy4_unpack_device");
    hipLaunchKernelGGL(k_g4u_sums, dim3((unsigned)nb), dim3(G4_THREADS), 0, st, words, nwords, w.bsum);
    hipLaunchKernelGGL(k_g4u_scan, dim3(1), dim3(G4U_SCAN_THREADS), 0, st, w.bsum, nb, w.bbase, count, cap, status);
    hipLaunchKernelGGL(k_g4u_emit, dim3((unsigned)nb), dim3(G4_THREADS), 0, st, words, nwords, w.bbase, out, status);
    return launch_status("gc_greedy4_unpack_device");
}

}  // extern "C"
