// mt_jump.hip — the torch CPU-generator stream (MT19937, seed.py:6-11 /
// compressors.py:310 torch.bernoulli) generated in parallel on gfx950.
//
// MT19937 is serial: draw t+1 needs the state after draw t.  The parallel
// stream cuts the `count` draws into G = ceil(count / J) generators of J =
// GC_MT_JUMP_DRAWS (= 624 x 420) consecutive draws.  Generator g starts from
// the 624-word window at raw position g*J of the caller's state frame (so every
// window is aligned to the 624-word twist blocks of the serial generator, and
// the last generator's final window IS torch's state array), with the caller's
// read index.  Its window comes from the jump-ahead of mt_poly.cpp:
//     x_{gJ-1+j} = XOR_{k : a_k = 1} x_{k+j},   a = x^(gJ-1) mod P,  j = 1..624
// J is GC_MT_JUMP_DRAWS, or any multiple of 624 through the _j entry points
// (the package picks one per count so that the generators spread over the CUs).
// Three launches, all on the caller's stream, no host synchronisation:
//   k_mt_seq    one workgroup: the first 20561 raw words x_0.. of the stream
//               (32 twists of the state) into the workspace; window 0 = the
//               state itself, plus the read index
//   k_mt_jump   16 workgroups per generator g >= 1, each over 1/16 of the
//               19937 coefficient bits with four shifted copies of its slice
//               of x_0..x_20560 in LDS; per SET bit a thread reads four
//               stream words (one aligned ds_read_b128) into its four window
//               words; k_mt_gen XORs the 16 partial windows
//   k_mt_gen    one 3-wave workgroup per generator: its window in LDS; one
//               wave twists (column-owned, in registers; double-buffered
//               blocks) while two temper the previous block and store the
//               draws coalesced; the last generator writes the state back
// Bit-exact with the serial stream (tests/test_gpu_parity.py vs the oracle's
// MT19937 and the reference's torch-mode goldens).
#include <algorithm>
#include <type_traits>

#include "gc_device.h"
#include "gc_host.h"
#include "qsgd_encode.h"

namespace gc {

constexpr uint32_t kMtN = 624;
constexpr uint32_t kMtM = 397;
constexpr uint32_t kMtSeq = 19937 + kMtN;              // x_0 .. x_20560 (k + j <= 19936 + 624)
constexpr uint32_t kMtSeqWs = 33 * kMtN;              // 33 twist blocks cover kMtSeq

static_assert(kMtSeqWs >= kMtSeq, "sequence blocks");

// workspace (uint32): [0] read index, [64 ..) sequence, window 0, then the
// jump partials of generators 1 .. G-1
constexpr uint64_t kWsSeq = 64;
constexpr uint64_t kWsWin = kWsSeq + kMtSeqWs;

__device__ __forceinline__ uint32_t mtj_temper(uint32_t y)
{
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

__device__ __forceinline__ uint32_t mtj_mix(uint32_t a, uint32_t b, uint32_t c)
{
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// column m (< H = 227) of the twist block after `o`, written into `nw`
// (another buffer): nw[m] = mix(o[m], o[m+1], o[m+397]), nw[m+H] =
// mix(o[m+H], o[m+H+1], nw[m]) and, for m < 170, nw[m+2H] = mix(o[m+2H],
// o[m+2H+1], nw[m+H]) with nw[0] in place of o[624] for word 623 (recomputed
// from o there).  Each word's in-block dependency is the column's previous
// word, so a column is three register steps after one batch of loads, and the
// 227 columns are independent: one per lane of the twisting waves.
__device__ __forceinline__ void twist_column(const uint32_t *o, uint32_t *nw, uint32_t m)
{
    constexpr uint32_t H = kMtN - kMtM;  // 227
    if (m >= H)
        return;
    const uint32_t a0 = o[m], a1 = o[m + 1], a2 = o[m + kMtM], b0 = o[m + H], b1 = o[m + H + 1];
    const uint32_t k = m + 2 * H;
    const uint32_t c0 = o[min(k, kMtN - 1)], c1 = o[min(k + 1, kMtN - 1)];
    const uint32_t A = mtj_mix(a0, a1, a2);
    const uint32_t B = mtj_mix(b0, b1, A);
    nw[m] = A;
    nw[m + H] = B;
    if (k < kMtN - 1)
        nw[k] = mtj_mix(c0, c1, B);
    else if (k == kMtN - 1)
        nw[k] = mtj_mix(c0, mtj_mix(o[0], o[1], o[kMtM]), B);
}

// x_0 .. x_{kMtSeqWs-1} of the caller's state frame; window 0 and the read index.
// One workgroup: the block after b is twisted column by column (twist_column,
// one column per lane of the first 227 threads) from one LDS buffer into the
// other, and all 256 threads store it.  One barrier per block, waiting on LDS
// traffic only: __syncthreads would also drain the global stores in flight
// (seven of those per block took this chain-critical kernel to 20 us, 38 us
// beside the pipeline's other kernels).
__global__ __launch_bounds__(256) void k_mt_seq(const uint32_t *__restrict__ state, uint32_t *__restrict__ ws)
{
    __shared__ uint32_t buf[2][kMtN];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < kMtN; i += 256) {
        const uint32_t v = state[i];
        buf[0][i] = v;
        ws[kWsSeq + i] = v;
        ws[kWsWin + i] = v;  // generator 0 starts from the state itself
    }
    if (tid == 0)
        ws[0] = state[kMtN];
    __syncthreads();
    for (uint32_t b = 1; b < kMtSeqWs / kMtN; ++b) {
        // block b from block b-1 (the other buffer); the stores of block b-1
        // read this buffer before the previous barrier (lgkmcnt(0) there)
        twist_column(buf[(b - 1) & 1u], buf[b & 1u], tid);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        for (uint32_t i = tid; i < kMtN; i += 256)
            ws[kWsSeq + (uint64_t)b * kMtN + i] = buf[b & 1u][i];
    }
}

// window of generator g >= 1: x_{gJ-1+j} = XOR over the set coefficient bits k
// of table[g-1] of x_{k+j}, j = 1..624, split over kMtJumpSplit blocks by
// coefficient range (block s: bits [s*1248, (s+1)*1248)) whose partial windows
// k_mt_gen XORs.  Only SET bits cost work (about half of them):
//   - the block expands its 39 coefficient words into a list of set-bit
//     positions in LDS (popcount prefix over the words);
//   - thread q owns the four window words j = 4q+1 .. 4q+4; for set bit k it
//     needs x_{k+j} .. x_{k+j+3}, an aligned ds_read_b128 from the copy of the
//     stream slice shifted by k mod 4 (four copies in LDS; lanes read
//     consecutive 16 B: no bank conflicts);
//   - two set bits fold into each window word with one v_xor3.
// LDS traffic is the bound: 16 B per (set bit, thread).  (The earlier forms —
// one word per thread with a uniform mask per bit, then a sliding b128 window
// with a mask per bit — were VALU-bound at 506 and 207 us for 1e8 draws.)
constexpr uint32_t kMtJumpSplit = 16;                            // blocks per generator
constexpr uint32_t kMtJumpWords = kMtN / kMtJumpSplit;           // 39 coefficient words per block
constexpr uint32_t kMtJumpBits = kMtJumpWords * 32;              // 1248
constexpr uint32_t kMtJumpThreads = 192;                         // 3 waves; thread q < 156 owns words 4q..4q+3
constexpr uint32_t kMtJumpOwners = kMtN / 4;                     // 156
constexpr uint32_t kMtJumpQuads = (kMtJumpBits / 4 + kMtJumpThreads + 1 + 7) & ~7u;  // per copy: a + q < 504
static_assert(kMtJumpWords * kMtJumpSplit == kMtN, "coefficient split");
static_assert((kMtJumpBits - 1) / 4 + kMtJumpThreads - 1 < kMtJumpQuads, "copy length");

// workspace: partial windows [split][gens - 1][624] after window 0
constexpr uint64_t kWsPart = kWsWin + kMtN;

__global__ __launch_bounds__(kMtJumpThreads) void k_mt_jump(const uint32_t *__restrict__ table, uint32_t *__restrict__ ws,
                                                           uint32_t jumps, const uint32_t *__restrict__ end_coef,
                                                           uint32_t nend)
{
    __shared__ uint4 cp4[4 * kMtJumpQuads];  // copy r: word u = x_{k0 + u + r + 1}
    __shared__ alignas(16) uint32_t pos[kMtJumpBits + 8];  // byte offset of set bit kk in its copy: ((kk&3)*Q + (kk>>2)) * 16
    __shared__ uint32_t cnt[kMtJumpWords + 1];
    uint32_t *cp = reinterpret_cast<uint32_t *>(cp4);
    const uint32_t gi = blockIdx.x / kMtJumpSplit, sp = blockIdx.x % kMtJumpSplit;
    const uint32_t k0 = sp * kMtJumpBits, tid = threadIdx.x;
    // the last nend slots are end windows (k_mt_end): coefficients end_coef[k]
    const uint32_t *__restrict__ coef =
        (gi + nend >= jumps ? end_coef + (uint64_t)(gi + nend - jumps) * kMtN : table + (uint64_t)gi * kMtN) +
        sp * kMtJumpWords;
    uint32_t c = 0;
    if (tid < kMtJumpWords) {
        c = coef[tid];
        cnt[tid + 1] = __builtin_popcount(c);
    }
    for (uint32_t v = tid; v < 4 * kMtJumpQuads + 3; v += kMtJumpThreads) {
        const uint32_t xi = k0 + v + 1;
        const uint32_t x = xi < kMtSeqWs ? ws[kWsSeq + xi] : 0u;
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r)
            if (v >= r && v - r < 4 * kMtJumpQuads)
                cp[r * 4 * kMtJumpQuads + v - r] = x;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t t = 0;
        cnt[0] = 0;
        for (uint32_t w = 1; w <= kMtJumpWords; ++w)
            cnt[w] = t += cnt[w];
    }
    __syncthreads();
    if (tid < kMtJumpWords) {
        uint32_t o = cnt[tid];
        while (c) {
            const uint32_t kk = tid * 32 + __builtin_ctz(c);
            c &= c - 1;
            pos[o++] = ((kk & 3u) * kMtJumpQuads + (kk >> 2)) * 16u;
        }
    }
    __syncthreads();
    if (tid >= kMtJumpOwners)
        return;  // no barrier below
    const uint32_t n = cnt[kMtJumpWords];
    const char *base = reinterpret_cast<const char *>(cp4) + 16u * tid;
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    auto ld = [&](uint32_t off) { return *reinterpret_cast<const uint4 *>(base + off); };
    auto fold2 = [&](const uint4 &u, const uint4 &v) {  // v_xor3 (truth table 0x96)
        a0 = __builtin_amdgcn_bitop3_b32(a0, u.x, v.x, 0x96);
        a1 = __builtin_amdgcn_bitop3_b32(a1, u.y, v.y, 0x96);
        a2 = __builtin_amdgcn_bitop3_b32(a2, u.z, v.z, 0x96);
        a3 = __builtin_amdgcn_bitop3_b32(a3, u.w, v.w, 0x96);
    };
    uint32_t i = 0;
    const uint4 *pos4 = reinterpret_cast<const uint4 *>(pos);
    uint4 q0 = pos4[0], q1 = pos4[1];  // the next batch's positions, loaded one batch ahead
    for (; i + 8 <= n; i += 8) {
        const uint4 p0 = q0, p1 = q1;
        q0 = pos4[i / 4 + 2];  // in bounds: pos has kMtJumpBits + 8 entries
        q1 = pos4[i / 4 + 3];
        const uint4 u0 = ld(p0.x), u1 = ld(p0.y), u2 = ld(p0.z), u3 = ld(p0.w);
        const uint4 u4 = ld(p1.x), u5 = ld(p1.y), u6 = ld(p1.z), u7 = ld(p1.w);
        fold2(u0, u1);
        fold2(u2, u3);
        fold2(u4, u5);
        fold2(u6, u7);
        // keep the prefetch where it is: the positions arrived before u0..u7 (DS returns in order)
        asm volatile("" : "+v"(q0.x), "+v"(q0.y), "+v"(q0.z), "+v"(q0.w), "+v"(q1.x), "+v"(q1.y), "+v"(q1.z), "+v"(q1.w));
    }
    for (; i + 2 <= n; i += 2)
        fold2(ld(pos[i]), ld(pos[i + 1]));
    if (i < n)
        fold2(ld(pos[i]), make_uint4(0u, 0u, 0u, 0u));
    *reinterpret_cast<uint4 *>(ws + kWsPart + ((uint64_t)sp * jumps + gi) * kMtN + 4u * tid) = make_uint4(a0, a1, a2, a3);
}

// one workgroup of kMtTwistWaves + kMtTemperWaves waves per generator: draws
// [gJ, min((g+1)J, count)) into out.  The twisting waves (one column per lane)
// build block t+1 in the other buffer while the tempering waves temper block t
// and store it (one barrier per block): the serial chain is one column's three
// register steps per block; the tempering and the HBM stores ride beside it.
// MODE 0: out = the draws (uint32).  MODE 1 / 2: draw i is consumed at once by
// element i of x, as torch.bernoulli consumes it (compressors.py:299-316), and
// out = q = sign(x)*xi as int8 / int32: the draws never reach HBM.
constexpr uint32_t kMtTwistWaves = 4;  // 256 lanes >= the 227 columns
constexpr uint32_t kMtTemperWaves = 4;
constexpr uint32_t kMtTemperThreads = 64 * kMtTemperWaves;
constexpr uint32_t kMtGenThreads = 64 * kMtTwistWaves + kMtTemperThreads;
constexpr uint32_t kMtRounds = (kMtN + kMtTemperThreads - 1) / kMtTemperThreads;  // elements per tempering thread

constexpr uint32_t kMtPre = 4;  // blocks of x in flight per tempering thread (quantize modes)

// the per-block hand-off between the twisting and the tempering waves: only the
// LDS traffic has to be complete (__syncthreads would also drain every global
// load and store in flight: the draws' stores and the x prefetch)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// RN(|x| / norm) as the reference computes it: Markstein's one-correction
// quotient where it is exact (the encode's per-tile check made
// per element), else the IEEE division
__device__ __forceinline__ float mt_quot(float v, const DivNorm &dv)
{
    const float a = fabsf(v);
    const uint32_t b = __float_as_uint(a);
    return (dv.fast && b - 1u >= dv.lo1 && b <= dv.hi) ? div_fast(a, dv) : a / dv.norm;
}

template <int MODE>
__device__ __forceinline__ void mt_store_q(void *out, uint64_t e, float v, uint32_t r, const DivNorm &dv, float s)
{
    const uint32_t q = enc_lane(v, mt_quot(v, dv), s, 0, r);
    if constexpr (MODE == 1)
        reinterpret_cast<int8_t *>(out)[e] = (int8_t)q;
    else
        reinterpret_cast<int32_t *>(out)[e] = (int32_t)q;
}

template <int MODE>
__device__ __forceinline__ void mt_emit(void *out, uint64_t e, uint32_t r, const float *__restrict__ x,
                                        const DivNorm &dv, float s)
{
    if constexpr (MODE == 0)
        reinterpret_cast<uint32_t *>(out)[e] = r;
    else
        mt_store_q<MODE>(out, e, x[e], r, dv, s);
}

// x of the block starting at element `at` into ring row `row` (768 floats:
// element i of the block at row[i]) as tempering thread ct consumes it, with
// global_load_lds_dword: the data goes straight to LDS (lane l of a wave to
// M0 + 4 l), no registers wait for it.  Indices are clamped into [0, end), so
// every thread issues exactly kMtRounds loads per call and the waves' memory
// counter counts nothing else (they issue no other global memory operation in
// the loop): s_waitcnt vmcnt((kMtPre - 1) * kMtRounds) before reading a row
// is exact.  The row's previous contents must have been read (lgkmcnt(0)).
__device__ __forceinline__ void mt_load_row(float *row, const float *__restrict__ x, uint64_t at, uint64_t end,
                                            uint32_t ct)
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (uint32_t r = 0; r < kMtRounds; ++r) {
        const float *p = x + min(at + min(ct + kMtTemperThreads * r, kMtN - 1), end - 1);
        const uint32_t lds = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)(row + kMtTemperThreads * r + (ct & ~63u)));
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dword %1, off" ::"s"(lds), "v"(p) : "memory");
    }
}
static_assert(kMtPre == 4 && kMtRounds == 3, "mt_wait_row's count");
__device__ __forceinline__ void mt_wait_row() { asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); }

// where the split-plane modes (4, 5) put the draws of element e: call k =
// e / per_end goes to region slot(k) = (ring0 + k) % ring of `bytes` bytes
// (ring 0: slot k), the call's HI plane then its LO plane (gc_device.h
// split_hpad).  A workgroup's blocks cross at most one call boundary each
// (per_end >= 624): the two regions in play are tracked per block.
struct SplitOut {
    uint8_t *base;
    uint64_t per_end, bytes;
    uint32_t ring, ring0;
};

// draws stored non-temporally (GC_MT_NT=0: plain stores, A/B)
static uint32_t mt_nt_stores()
{
    static const uint32_t on = [] {
        const char *e = getenv("GC_MT_NT");
        return (uint32_t)!(e && atol(e) == 0);
    }();
    return on;
}

// one draw word to HBM, non-temporal when NT
template <bool NT>
__device__ __forceinline__ void mt_st(uint32_t *p, uint32_t v)
{
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

template <int MODE, bool NT = false>
__global__ __launch_bounds__(kMtGenThreads) void k_mt_gen(uint32_t *__restrict__ ws, uint64_t gens, uint64_t jumps,
                                                         uint64_t J, uint64_t count,
                                                         void *__restrict__ out, uint32_t *__restrict__ state,
                                                         const float *__restrict__ x, const float *__restrict__ normp,
                                                         float s, uint64_t g0, SplitOut so)
{
    __shared__ __attribute__((aligned(16))) uint32_t buf[2][kMtN];
    const uint32_t tid = threadIdx.x, wave = tid >> 6;
    const uint64_t g = g0 + blockIdx.x;
    if (g == 0)
        for (uint32_t i = tid; i < kMtN; i += kMtGenThreads)
            buf[0][i] = ws[kWsWin + i];
    else
        for (uint32_t i = tid; i < kMtN; i += kMtGenThreads) {
            uint32_t v = 0;
#pragma unroll
            for (uint32_t sp = 0; sp < kMtJumpSplit; ++sp)
                v ^= ws[kWsPart + (sp * jumps + g - 1) * kMtN + i];
            buf[0][i] = v;
        }
    const uint32_t ptr0 = ws[0];
    __syncthreads();
    const uint64_t pos0 = g * J, end = min(pos0 + J, count);  // J % 624 == 0: windows stay block-aligned
    const uint32_t head = ptr0 < kMtN ? (uint32_t)min((uint64_t)(kMtN - ptr0), end - pos0) : 0u;  // rest of block 0
    const uint64_t rest = end - pos0 - head;
    const uint32_t twists = (uint32_t)((rest + kMtN - 1) / kMtN);
    const uint32_t ct = tid - 64u * kMtTwistWaves;  // tempering thread 0 .. kMtTemperThreads-1
    // The twisting wave and the tempering waves run separate loops with the
    // same number of barriers (twists + 1): each loop is straight-line code
    // for the compiler's memory-counter tracking, so the tempering waves'
    // prefetched x loads stay in flight across blocks.
    typedef typename std::conditional<MODE == 2, int32_t, int8_t>::type QT;
    constexpr bool QUANT = MODE == 1 || MODE == 2;  // the quantize modes (0: draws, 3: 24-bit packed draws)
    __shared__ QT qbuf[QUANT ? 2 : 1][QUANT ? kMtN : 1];  // q of block t in qbuf[t & 1], stored by the twisting waves
    __shared__ float xring[QUANT ? kMtPre : 1][QUANT ? kMtTemperThreads * kMtRounds : 1];  // x, kMtPre blocks ahead
    if (wave < kMtTwistWaves) {
        // block t's q (t >= 1) lands in qbuf[t & 1] during iteration t and is
        // stored to HBM by these waves during iteration t + 1: the global stores
        // never sit in the same wave as the tempering waves' x prefetch
        auto store_q = [&](uint32_t t) {
            const uint64_t at = t ? pos0 + head + (uint64_t)(t - 1) * kMtN : pos0;
            const uint32_t take = t ? (uint32_t)min((uint64_t)kMtN, end - at) : head;
            QT *o = reinterpret_cast<QT *>(out) + at;
            for (uint32_t i = tid; i < take; i += 64u * kMtTwistWaves)
                o[i] = qbuf[t & 1u][i];
        };
        for (uint32_t t = 0; t < twists; ++t) {
            twist_column(buf[t & 1u], buf[(t + 1) & 1u], tid);
            if (QUANT && t > 0)
                store_q(t - 1);
            lds_barrier();
        }
        if (QUANT && twists > 0)
            store_q(twists - 1);
        lds_barrier();
        if (QUANT)
            store_q(twists);
    } else if constexpr (MODE == 0) {
        for (uint32_t i = ct; i < head; i += kMtTemperThreads)
            mt_st<NT>(reinterpret_cast<uint32_t *>(out) + (pos0 + i), mtj_temper(buf[0][ptr0 + i]));
        lds_barrier();
        for (uint32_t t = 1; t <= twists; ++t) {
            const uint32_t *cur = buf[t & 1u];
            const uint64_t at = pos0 + head + (uint64_t)(t - 1) * kMtN;
            const uint32_t take = (uint32_t)min((uint64_t)kMtN, end - at);
            if (take == kMtN) {
#pragma unroll
                for (uint32_t r = 0; r < kMtRounds; ++r) {
                    const uint32_t i = ct + kMtTemperThreads * r;
                    if (i < kMtN)
                        mt_st<NT>(reinterpret_cast<uint32_t *>(out) + (at + i), mtj_temper(cur[i]));
                }
            } else {
                for (uint32_t i = ct; i < take; i += kMtTemperThreads)
                    mt_st<NT>(reinterpret_cast<uint32_t *>(out) + (at + i), mtj_temper(cur[i]));
            }
            lds_barrier();
        }
    } else if constexpr (MODE == 4 || MODE == 5) {
        // split planes (GC_RNG_SPLIT8 / SPLIT16), one draw per tempering thread
        // and round like MODE 0 (all 256 lanes busy; a wave's 1- / 2-byte
        // stores are contiguous): the top HB of the draw's low 24 bits to the
        // HI plane, the rest to the LO plane of its call's region
        constexpr uint32_t HB = MODE == 4 ? 8u : 16u;
        const uint64_t hpad = split_hpad(so.per_end, HB);
        uint64_t kc = pos0 / so.per_end;         // call of the current block's first draw
        uint64_t bnd = (kc + 1) * so.per_end;    // first draw of the next call
        // the regions of calls kc and kc + 1, moved on at a call boundary (the
        // ring slot is stepped, not divided, per block: uniform but on the
        // tempering waves' per-block path)
        uint64_t slot = so.ring ? (so.ring0 + kc) % so.ring : kc;
        auto next_slot = [&](uint64_t sl) { return so.ring ? (sl + 1 == so.ring ? 0 : sl + 1) : sl + 1; };
        uint8_t *rcur = so.base + slot * so.bytes, *rnxt = so.base + next_slot(slot) * so.bytes;
        auto region = [&](uint64_t k) { return k == kc ? rcur : rnxt; };  // k is kc or kc + 1
        auto emit1 = [&](uint64_t e, uint32_t raw, uint8_t *rc, uint8_t *rn) {
            const uint32_t y = mtj_temper(raw);
            const bool nx = e >= bnd;
            uint8_t *r = nx ? rn : rc;
            const uint64_t loc = e - (nx ? bnd : bnd - so.per_end);
            if constexpr (HB == 8) {
                r[loc] = (uint8_t)(y >> 16);
                reinterpret_cast<uint16_t *>(r + hpad)[loc] = (uint16_t)y;
            } else {
                reinterpret_cast<uint16_t *>(r)[loc] = (uint16_t)(y >> 8);
                r[hpad + loc] = (uint8_t)y;
            }
        };
        // whole quads (read index and per_end multiples of 4: every quad's four
        // draws sit in one call, 8- / 4-byte aligned): thread ct tempers draws
        // 4q .. 4q+3 and stores one HI word pair / word and one LO word / pair
        // The plane pointers of a block are uniform: quads j = 4q < cut go to
        // call kc's region, the rest (a block that crosses a call boundary) to
        // call kc + 1's; each quad adds its own offset and picks one of the two
        // bases, and the byte shuffles are v_perm_b32 (VALU per quad about that
        // of the packed24 mode)
        constexpr uint32_t HS = HB / 8, LS = (24u - HB) / 8;  // bytes per draw in each plane
        struct Bases {
            uint8_t *hc, *lc, *hn, *ln;
            uint32_t cut;
        };
        auto bases = [&](uint64_t at0) {
            Bases B;
            uint8_t *r0 = region(kc);
            const uint64_t off0 = at0 - (bnd - so.per_end);  // element offset of at0 in call kc
            B.hc = r0 + HS * off0;
            B.lc = r0 + hpad + LS * off0;
            const uint64_t toend = bnd - at0;                // this block's draws still in call kc
            if (toend < kMtN) {
                uint8_t *r1 = region(kc + 1);
                B.cut = (uint32_t)toend;
                B.hn = r1 - HS * toend;                      // + HS * j for j >= cut: call kc + 1
                B.ln = r1 + hpad - LS * toend;
            } else {
                B.cut = kMtN;
                B.hn = B.hc;
                B.ln = B.lc;
            }
            return B;
        };
        auto emit4 = [&](uint32_t j, const uint32_t *src, const Bases &B) {
            const uint4 w = *reinterpret_cast<const uint4 *>(src);  // 16-byte aligned: ptr0 % 4 == 0
            const uint32_t a = mtj_temper(w.x), b = mtj_temper(w.y), c = mtj_temper(w.z), d = mtj_temper(w.w);
            const bool nx = j >= B.cut;
            uint8_t *h = (nx ? B.hn : B.hc) + HS * j;
            uint8_t *l = (nx ? B.ln : B.lc) + LS * j;
            uint32_t *h32 = reinterpret_cast<uint32_t *>(h), *l32 = reinterpret_cast<uint32_t *>(l);
            if constexpr (HB == 8) {  // HI: bytes 2 of a, b, c, d; LO: bytes 0-1 of each
                const uint32_t x = __builtin_amdgcn_perm(b, a, 0x0C0C0602u), y = __builtin_amdgcn_perm(d, c, 0x0C0C0602u);
                mt_st<NT>(h32, __builtin_amdgcn_perm(y, x, 0x05040100u));
                mt_st<NT>(l32, __builtin_amdgcn_perm(b, a, 0x05040100u));
                mt_st<NT>(l32 + 1, __builtin_amdgcn_perm(d, c, 0x05040100u));
            } else {  // HI: bytes 1-2 of each; LO: byte 0 of each
                mt_st<NT>(h32, __builtin_amdgcn_perm(b, a, 0x06050201u));
                mt_st<NT>(h32 + 1, __builtin_amdgcn_perm(d, c, 0x06050201u));
                const uint32_t x = __builtin_amdgcn_perm(b, a, 0x0C0C0400u), y = __builtin_amdgcn_perm(d, c, 0x0C0C0400u);
                mt_st<NT>(l32, __builtin_amdgcn_perm(y, x, 0x05040100u));
            }
        };
        const bool quads = (ptr0 & 3u) == 0 && (so.per_end & 3u) == 0;  // uniform
        if (quads) {
            const Bases B = bases(pos0);
            for (uint32_t q = ct; 4 * q < head; q += kMtTemperThreads)
                emit4(4 * q, &buf[0][ptr0 + 4 * q], B);
        } else {
            uint8_t *rc = region(kc), *rn = region(kc + 1);
            for (uint32_t i = ct; i < head; i += kMtTemperThreads)
                emit1(pos0 + i, buf[0][ptr0 + i], rc, rn);
        }
        lds_barrier();
        for (uint32_t t = 1; t <= twists; ++t) {
            const uint32_t *cur = buf[t & 1u];
            const uint64_t at = pos0 + head + (uint64_t)(t - 1) * kMtN;
            const uint32_t take = (uint32_t)min((uint64_t)kMtN, end - at);
            if (at >= bnd) {  // uniform: the block starts in the next call
                ++kc;
                bnd += so.per_end;
                slot = next_slot(slot);
                rcur = rnxt;
                rnxt = so.base + next_slot(slot) * so.bytes;
            }
            if (quads) {
                const Bases B = bases(at);
                for (uint32_t q = ct; 4 * q < take; q += kMtTemperThreads)
                    emit4(4 * q, cur + 4 * q, B);
            } else {
                uint8_t *rc = region(kc), *rn = region(kc + 1);
#pragma unroll
                for (uint32_t r = 0; r < kMtRounds; ++r) {
                    const uint32_t i = ct + kMtTemperThreads * r;
                    if (i < take)
                        emit1(at + i, cur[i], rc, rn);
                }
            }
            lds_barrier();
        }
    } else if constexpr (MODE == 3) {
        // 24-bit packed draws (GC_RNG_STREAM24): thread ct tempers draws
        // 4q .. 4q+3 of a block and stores their low 24 bits as 3 words.  The
        // caller's read index and count are multiples of 4 (host-checked), so
        // head, every block start `at` and every `take` are too
        uint32_t *o = reinterpret_cast<uint32_t *>(out);
        auto emit4 = [&](uint64_t e, const uint32_t *src) {
            const uint4 w = *reinterpret_cast<const uint4 *>(src);  // 16-byte aligned: ptr0 % 4 == 0
            const uint32_t a = mtj_temper(w.x), b = mtj_temper(w.y), c = mtj_temper(w.z), d = mtj_temper(w.w);
            uint3 p;
            p.x = (a & 0xFFFFFFu) | (b << 24);
            p.y = ((b >> 8) & 0xFFFFu) | (c << 16);
            p.z = ((c >> 16) & 0xFFu) | (d << 8);
            uint32_t *o3 = o + (e >> 2) * 3;
            mt_st<NT>(o3, p.x);
            mt_st<NT>(o3 + 1, p.y);
            mt_st<NT>(o3 + 2, p.z);
        };
        for (uint32_t q = ct; 4 * q < head; q += kMtTemperThreads)
            emit4(pos0 + 4 * q, &buf[0][ptr0 + 4 * q]);
        lds_barrier();
        for (uint32_t t = 1; t <= twists; ++t) {
            const uint32_t *cur = buf[t & 1u];
            const uint64_t at = pos0 + head + (uint64_t)(t - 1) * kMtN;
            const uint32_t take = (uint32_t)min((uint64_t)kMtN, end - at);
            for (uint32_t q = ct; 4 * q < take; q += kMtTemperThreads)
                emit4(at + 4 * q, cur + 4 * q);
            lds_barrier();
        }
    } else {
        // quantize modes: x of block t is fetched kMtPre blocks ahead into an
        // LDS ring by global_load_lds (mt_load_row), and these waves issue no
        // other global memory operation in the loop (their q goes to qbuf, the
        // twisting waves store it), so each wait is an exact count
        const DivNorm dv = make_div(*normp);
        const uint64_t body = pos0 + head;  // element of block 1's first draw
        for (uint32_t i = ct; i < head; i += kMtTemperThreads) {
            const float v = x[pos0 + i];
            qbuf[0][i] = (QT)enc_lane(v, mt_quot(v, dv), s, 0, mtj_temper(buf[0][ptr0 + i]));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the head's loads: the ring's counts start from zero
#pragma unroll
        for (uint32_t d = 0; d < kMtPre; ++d)
            mt_load_row(xring[d], x, body + (uint64_t)d * kMtN, end, ct);
        lds_barrier();
        for (uint32_t t0 = 1; t0 <= twists; t0 += kMtPre) {
#pragma unroll
            for (uint32_t d = 0; d < kMtPre; ++d) {
                const uint32_t t = t0 + d;
                if (t > twists)
                    break;  // uniform over the tempering waves
                const uint32_t *cur = buf[t & 1u];
                const uint64_t at = body + (uint64_t)(t - 1) * kMtN;
                mt_wait_row();
#pragma unroll
                for (uint32_t r = 0; r < kMtRounds; ++r) {
                    const uint32_t i = ct + kMtTemperThreads * r;
                    const uint32_t ic = min(i, kMtN - 1);  // past 623: recomputes word 623 (same x, same draw)
                    const float v = xring[d][i];
                    qbuf[t & 1u][ic] = (QT)enc_lane(v, mt_quot(v, dv), s, 0, mtj_temper(cur[ic]));
                }
                mt_load_row(xring[d], x, at + (uint64_t)kMtPre * kMtN, end, ct);
                lds_barrier();
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-bound load outlives the workgroup
    }
    __syncthreads();
    if (state && g == gens - 1) {  // the advanced state: the last block (aligned to the twist blocks) + read index
        for (uint32_t i = tid; i < kMtN; i += kMtGenThreads)
            state[i] = buf[twists & 1u][i];
        if (tid == 0)
            state[kMtN] = twists ? (uint32_t)(rest - (uint64_t)(twists - 1) * kMtN) : ptr0 + head;
    }
}

// the state after `count` draws without generating them: raw block B =
// floor((idx + count - 1) / 624) of the caller's frame (block 0 = the state
// itself) is the window at raw position 624 B, jumped by k_mt_jump's end slot
// (coefficients x^(624 B - 1) mod P); the read index becomes idx + count - 624 B
// (in 1 .. 624).  Written over the caller's state in place (k_mt_seq has
// already copied it into the workspace), so the next call's sequence can start
// while this call's generators still run.
__global__ __launch_bounds__(256) void k_mt_end(uint32_t *__restrict__ ws, uint32_t jumps, uint64_t count,
                                                uint64_t end_block, uint32_t *__restrict__ state)
{
    const uint32_t ptr0 = ws[0];
    for (uint32_t i = threadIdx.x; i < kMtN; i += 256) {
        uint32_t v;
        if (end_block == 0) {
            v = ws[kWsWin + i];
        } else {
            v = 0;
#pragma unroll
            for (uint32_t sp = 0; sp < kMtJumpSplit; ++sp)
                v ^= ws[kWsPart + ((uint64_t)sp * jumps + jumps - 1) * kMtN + i];
        }
        state[i] = v;
    }
    if (threadIdx.x == 0)  // a caller whose end_block does not match idx gets an impossible index (> 624)
        state[kMtN] = (uint32_t)(ptr0 + count - kMtN * end_block);
}

// nend end states of one run (gc_mt19937_generate_multi_j): end k is the state
// after (k + 1) * per_end draws, from the jump slot jumps - nend + k (raw
// block B_k = floor((idx + (k + 1) per_end - 1) / 624) >= 1, read index
// idx + (k + 1) per_end - 624 B_k), into ends[k * kMtEndStride ..]; the last
// one also over the caller's state (the next run chains from it)
constexpr uint32_t kMtEndStride = kMtN + 2;  // 624 words + read index, 8-byte rows
__global__ __launch_bounds__(256) void k_mt_end_multi(const uint32_t *__restrict__ ws, uint32_t jumps, uint32_t nend,
                                                      uint64_t per_end, uint32_t *__restrict__ state,
                                                      uint32_t *__restrict__ ends)
{
    const uint32_t k = blockIdx.x;
    const uint32_t ptr0 = ws[0];
    const uint64_t pos = (uint64_t)ptr0 + (k + 1) * per_end;
    const uint64_t block = (pos - 1) / kMtN;
    const uint32_t slot = jumps - nend + k;
    uint32_t *e = ends + (uint64_t)k * kMtEndStride;
    for (uint32_t i = threadIdx.x; i < kMtN; i += 256) {
        uint32_t v = 0;
#pragma unroll
        for (uint32_t sp = 0; sp < kMtJumpSplit; ++sp)
            v ^= ws[kWsPart + ((uint64_t)sp * jumps + slot) * kMtN + i];
        e[i] = v;
        if (k == nend - 1)
            state[i] = v;
    }
    if (threadIdx.x == 0) {
        e[kMtN] = (uint32_t)(pos - kMtN * block);
        if (k == nend - 1)
            state[kMtN] = (uint32_t)(pos - kMtN * block);
    }
}

}  // namespace gc

using namespace gc;

extern "C" {

size_t gc_mt19937_workspace_size_j(uint64_t count, uint64_t J)
{
    const uint64_t gens = count && J ? (count + J - 1) / J : 1;
    return 4 * (kWsPart + kMtJumpSplit * gens * kMtN);  // gens - 1 generator windows + the end window
}

size_t gc_mt19937_workspace_size(uint64_t count) { return gc_mt19937_workspace_size_j(count, GC_MT_JUMP_DRAWS); }

// seq -> jump -> gen<MODE> for `count` draws of state_dev, generators of J draws
// (phase bit 1: seq + jump, bit 2: gen; the two halves of one run must be
// enqueued in order on one stream with the same arguments)
// SPLIT (gc_mt19937_generate_split_j): phase 1 also jumps to the end state and
// writes it over state_dev (k_mt_end); the generators then leave the state alone
static int mt_run(const char *what, int mode, uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens,
                  uint64_t J, void *out, uint64_t count, void *workspace, gc_stream_t stream, const float *x,
                  const float *norm, float s, int phase = 3, bool split = false, const uint32_t *end_coef = nullptr,
                  uint64_t end_block = 0)
{
    GC_REQUIRE(state_dev && workspace, "%s: null state/workspace", what);
    GC_REQUIRE(count == 0 || out || !(phase & 2), "%s: null out", what);
    GC_REQUIRE(J > 0 && J % kMtN == 0, "%s: J = %llu is not a positive multiple of 624", what, (unsigned long long)J);
    if (count == 0)
        return GC_OK;
    const uint64_t gens = (count + J - 1) / J;
    GC_REQUIRE(gens - 1 <= table_gens && (gens == 1 || table_dev),
               "%s: jump table holds %llu generators, %llu draws need %llu", what, (unsigned long long)table_gens,
               (unsigned long long)count, (unsigned long long)(gens - 1));
    GC_REQUIRE(gens <= 0x7fffffffull / kMtJumpSplit, "%s: count too large", what);
    const bool has_end = split && end_block > 0;
    GC_REQUIRE(!has_end || end_coef, "%s: null end coefficients", what);
    const uint32_t jumps = (uint32_t)(gens - 1 + (has_end ? 1 : 0));
    hipStream_t st = as_stream(stream);
    uint32_t *ws = reinterpret_cast<uint32_t *>(workspace);
    if (phase & 1) {
        hipLaunchKernelGGL(k_mt_seq, dim3(1), dim3(256), 0, st, state_dev, ws);
        if (jumps > 0)
            hipLaunchKernelGGL(k_mt_jump, dim3((unsigned)(jumps * kMtJumpSplit)), dim3(kMtJumpThreads), 0, st,
                               table_dev, ws, jumps, has_end ? end_coef : nullptr, has_end ? 1u : 0u);
        if (split)
            hipLaunchKernelGGL(k_mt_end, dim3(1), dim3(256), 0, st, ws, jumps, count, end_block, state_dev);
    }
    if (!(phase & 2))
        return launch_status(what);
    uint32_t *gstate = split ? nullptr : state_dev;
    if (mode == 0)
        hipLaunchKernelGGL(k_mt_gen<0>, dim3((unsigned)gens), dim3(kMtGenThreads), 0, st, ws, gens, (uint64_t)jumps,
                           J, count, out, gstate, x, norm, s, (uint64_t)0, SplitOut{});
    else if (mode == 1)
        hipLaunchKernelGGL(k_mt_gen<1>, dim3((unsigned)gens), dim3(kMtGenThreads), 0, st, ws, gens, (uint64_t)jumps,
                           J, count, out, gstate, x, norm, s, (uint64_t)0, SplitOut{});
    else if (mode == 2)
        hipLaunchKernelGGL(k_mt_gen<2>, dim3((unsigned)gens), dim3(kMtGenThreads), 0, st, ws, gens, (uint64_t)jumps,
                           J, count, out, gstate, x, norm, s, (uint64_t)0, SplitOut{});
    else
        hipLaunchKernelGGL(k_mt_gen<3>, dim3((unsigned)gens), dim3(kMtGenThreads), 0, st, ws, gens, (uint64_t)jumps,
                           J, count, out, gstate, x, norm, s, (uint64_t)0, SplitOut{});
    return launch_status(what);
}

int gc_mt19937_generate_jumped_j(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint64_t J,
                                 uint32_t *out, uint64_t count, void *workspace, gc_stream_t stream)
{
    return mt_run("gc_mt19937_generate_jumped", 0, state_dev, table_dev, table_gens, J, out, count, workspace, stream,
                  nullptr, nullptr, 0.0f);
}

int gc_mt19937_generate_phase_j(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint64_t J,
                                uint32_t *out, uint64_t count, void *workspace, int phase, gc_stream_t stream)
{
    GC_REQUIRE(phase >= 1 && phase <= 3, "gc_mt19937_generate_phase_j: phase must be 1, 2 or 3");
    return mt_run("gc_mt19937_generate_phase_j", 0, state_dev, table_dev, table_gens, J, out, count, workspace, stream,
                  nullptr, nullptr, 0.0f, phase);
}

int gc_mt19937_generate_split_j(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint64_t J,
                                const uint32_t *end_coef, uint64_t end_block, uint32_t *out, uint64_t count,
                                void *workspace, int phase, gc_stream_t stream)
{
    GC_REQUIRE(phase >= 1 && phase <= 3, "gc_mt19937_generate_split_j: phase must be 1, 2 or 3");
    GC_REQUIRE(count > 0, "gc_mt19937_generate_split_j: count must be positive");
    return mt_run("gc_mt19937_generate_split_j", 0, state_dev, table_dev, table_gens, J, out, count, workspace, stream,
                  nullptr, nullptr, 0.0f, phase, true, end_coef, end_block);
}

int gc_mt19937_generate_split24_j(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint64_t J,
                                  const uint32_t *end_coef, uint64_t end_block, uint32_t *out, uint64_t count,
                                  uint64_t idx, void *workspace, int phase, gc_stream_t stream)
{
    const char *what = "gc_mt19937_generate_split24_j";
    GC_REQUIRE(phase >= 1 && phase <= 3, "%s: phase must be 1, 2 or 3", what);
    GC_REQUIRE(count > 0 && count % 4 == 0 && idx % 4 == 0 && idx <= kMtN,
               "%s: count (%llu) and the read index (%llu) must be multiples of 4", what, (unsigned long long)count,
               (unsigned long long)idx);
    GC_REQUIRE(!out || ((uintptr_t)out & 3u) == 0, "%s: out must be 4-byte aligned", what);
    return mt_run(what, 3, state_dev, table_dev, table_gens, J, out, count, workspace, stream, nullptr, nullptr, 0.0f,
                  phase, true, end_coef, end_block);
}

size_t gc_mt19937_workspace_size_multi_j(uint64_t count, uint64_t J, uint32_t nend)
{
    const uint64_t gens = count && J ? (count + J - 1) / J : 1;
    return 4 * (kWsPart + kMtJumpSplit * (gens - 1 + nend) * kMtN);
}

}  // extern "C"

// the multi-call run of gc_mt19937_generate_multi_j / _multi24_j: MODE 0
// plain draws, 3 the 24-bit packed draws
static int mt_multi(const char *what, int mode, uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens,
                    uint64_t J, const uint32_t *end_coefs, uint32_t nend, uint64_t per_end, uint32_t *ends_out,
                    uint32_t *out, void *workspace, int phase, gc_stream_t stream, SplitOut so = SplitOut{},
                    uint64_t g_first = 0, uint64_t g_count = ~0ull)
{
    GC_REQUIRE(phase >= 1 && phase <= 3, "%s: phase must be 1, 2 or 3", what);
    GC_REQUIRE(state_dev && workspace && end_coefs && ends_out, "%s: null state / workspace / ends", what);
    GC_REQUIRE(nend >= 1 && nend <= 64 && per_end >= kMtN, "%s: nend must be 1..64 and per_end >= 624", what);
    GC_REQUIRE(J > 0 && J % kMtN == 0, "%s: J = %llu is not a positive multiple of 624", what, (unsigned long long)J);
    const uint64_t count = per_end * nend;
    GC_REQUIRE(count < (1ull << 40), "%s: count too large", what);
    GC_REQUIRE(!(phase & 2) || out, "%s: null out", what);
    GC_REQUIRE(!(phase & 2) || ((uintptr_t)out & 3u) == 0, "%s: out must be 4-byte aligned", what);
    const uint64_t gens = (count + J - 1) / J;
    GC_REQUIRE(gens - 1 <= table_gens && (gens == 1 || table_dev),
               "%s: jump table holds %llu generators, %llu draws need %llu", what, (unsigned long long)table_gens,
               (unsigned long long)count, (unsigned long long)(gens - 1));
    GC_REQUIRE(gens - 1 + nend <= 0x7fffffffull / kMtJumpSplit, "%s: count too large", what);
    const uint32_t jumps = (uint32_t)(gens - 1 + nend);
    hipStream_t st = as_stream(stream);
    uint32_t *ws = reinterpret_cast<uint32_t *>(workspace);
    if (phase & 1) {
        hipLaunchKernelGGL(k_mt_seq, dim3(1), dim3(256), 0, st, state_dev, ws);
        hipLaunchKernelGGL(k_mt_jump, dim3((unsigned)(jumps * kMtJumpSplit)), dim3(kMtJumpThreads), 0, st, table_dev,
                           ws, jumps, end_coefs, nend);
        hipLaunchKernelGGL(k_mt_end_multi, dim3(nend), dim3(256), 0, st, ws, jumps, nend, per_end, state_dev,
                           ends_out);
    }
    if (phase & 2) {
        // generators g_first .. g_first + g_count - 1 (clamped to the run)
        const uint64_t g1 = std::min(gens, g_first + std::min(g_count, gens));
        if (g_first >= g1)
            return launch_status(what);
        const dim3 grid((unsigned)(g1 - g_first));
#define GC_MTG1(M_, NT_)                                                                                             \
    hipLaunchKernelGGL((k_mt_gen<M_, NT_>), grid, dim3(kMtGenThreads), 0, st, ws, gens, (uint64_t)jumps, J, count,   \
                       (void *)out, (uint32_t *)nullptr, (const float *)nullptr, (const float *)nullptr, 0.0f, g_first, \
                       so)
#define GC_MTG(M_)                                                                                                   \
    do {                                                                                                             \
        if (mt_nt_stores())                                                                                          \
            GC_MTG1(M_, true);                                                                                       \
        else                                                                                                         \
            GC_MTG1(M_, false);                                                                                      \
    } while (0)
        if (mode == 3)
            GC_MTG(3);
        else if (mode == 4)
            GC_MTG(4);
        else if (mode == 5)
            GC_MTG(5);
        else
            GC_MTG(0);
#undef GC_MTG
#undef GC_MTG1
    }
    return launch_status(what);
}

extern "C" {

int gc_mt19937_generate_multi_j(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint64_t J,
                                const uint32_t *end_coefs, uint32_t nend, uint64_t per_end, uint32_t *ends_out,
                                uint32_t *out, void *workspace, int phase, gc_stream_t stream)
{
    return mt_multi("gc_mt19937_generate_multi_j", 0, state_dev, table_dev, table_gens, J, end_coefs, nend, per_end,
                    ends_out, out, workspace, phase, stream);
}

int gc_mt19937_generate_multi24_j(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint64_t J,
                                  const uint32_t *end_coefs, uint32_t nend, uint64_t per_end, uint64_t idx,
                                  uint32_t *ends_out, uint32_t *out, void *workspace, int phase, gc_stream_t stream)
{
    const char *what = "gc_mt19937_generate_multi24_j";
    GC_REQUIRE(per_end % 4 == 0 && idx % 4 == 0 && idx <= kMtN,
               "%s: per_end (%llu) and the read index (%llu) must be multiples of 4", what,
               (unsigned long long)per_end, (unsigned long long)idx);
    return mt_multi(what, 3, state_dev, table_dev, table_gens, J, end_coefs, nend, per_end, ends_out, out, workspace,
                    phase, stream);
}

uint64_t gc_rng_split_bytes(uint64_t n, uint32_t hi_bits)
{
    return (hi_bits == 8 || hi_bits == 16) ? split_bytes(n, hi_bits) : 0;
}

int gc_mt19937_generate_multi_split_j(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint64_t J,
                                      const uint32_t *end_coefs, uint32_t nend, uint64_t per_end, uint64_t idx,
                                      uint32_t hi_bits, uint32_t *ends_out, void *out, uint32_t ring, uint32_t ring0,
                                      uint64_t g_first, uint64_t g_count, void *workspace, int phase,
                                      gc_stream_t stream)
{
    const char *what = "gc_mt19937_generate_multi_split_j";
    GC_REQUIRE(hi_bits == 8 || hi_bits == 16, "%s: hi_bits must be 8 or 16", what);
    GC_REQUIRE(idx <= kMtN, "%s: read index %llu above 624", what, (unsigned long long)idx);
    GC_REQUIRE(!(phase & 2) || ((uintptr_t)out & 15u) == 0, "%s: out must be 16-byte aligned", what);
    GC_REQUIRE(ring == 0 || ring >= 2, "%s: a ring holds 0 (none) or at least 2 regions", what);
    GC_REQUIRE(ring == 0 || ring0 < ring, "%s: ring0 must be below ring", what);
    SplitOut so;
    so.base = reinterpret_cast<uint8_t *>(out);
    so.per_end = per_end;
    so.bytes = split_bytes(per_end, hi_bits);
    so.ring = ring;
    so.ring0 = ring0;
    return mt_multi(what, hi_bits == 8 ? 4 : 5, state_dev, table_dev, table_gens, J, end_coefs, nend, per_end,
                    ends_out, reinterpret_cast<uint32_t *>(out), workspace, phase, stream, so, g_first, g_count);
}

int gc_mt19937_generate_jumped(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint32_t *out,
                               uint64_t count, void *workspace, gc_stream_t stream)
{
    return gc_mt19937_generate_jumped_j(state_dev, table_dev, table_gens, GC_MT_JUMP_DRAWS, out, count, workspace,
                                        stream);
}

int gc_qsgd_quantize_mt19937(const float *x, uint64_t n, const float *norm, uint32_t bits, uint32_t *state_dev,
                             const uint32_t *table_dev, uint64_t table_gens, uint64_t J, void *q, uint32_t q_dtype,
                             void *workspace, gc_stream_t stream)
{
    GC_REQUIRE(bits >= 1 && bits <= 8, "gc_qsgd_quantize_mt19937: bits must be 1..8");
    GC_REQUIRE(q_dtype == GC_I32 || (q_dtype == GC_I8 && bits <= 7),
               "gc_qsgd_quantize_mt19937: q_dtype must be GC_I8 (bits <= 7) or GC_I32");
    GC_REQUIRE(n == 0 || (x && norm), "gc_qsgd_quantize_mt19937: null x/norm");
    return mt_run("gc_qsgd_quantize_mt19937", q_dtype == GC_I8 ? 1 : 2, state_dev, table_dev, table_gens, J, q, n,
                  workspace, stream, x, norm, (float)((1u << bits) - 1u));
}

}  // extern "C"
