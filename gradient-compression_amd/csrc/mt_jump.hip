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
#include "gc_device.h"
#include "gc_host.h"

namespace gc {

constexpr uint32_t kMtN = 624;
constexpr uint32_t kMtM = 397;
constexpr uint32_t kMtJ = GC_MT_JUMP_DRAWS;
constexpr uint32_t kMtSeq = 19937 + kMtN;              // x_0 .. x_20560 (k + j <= 19936 + 624)
constexpr uint32_t kMtSeqWs = 33 * kMtN;              // 33 twist blocks cover kMtSeq

static_assert(kMtJ % kMtN == 0, "generator windows stay aligned to the twist blocks");
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

// the twist block after `o` into `nw` (another buffer) by one wave.  With
// H = 227: nw[k] = mix(o[k], o[k+1], o[k+397]) for k < H, mix(o[k], o[k+1],
// nw[k-H]) for k < 623, and nw[623] = mix(o[623], nw[0], nw[396]).  Lane
// column m (< H) owns nw[m], nw[m+H], nw[m+2H]: each word's in-block
// dependency is the word before it in the SAME lane, so the three phases run
// in registers (only nw[0] crosses lanes: a readlane) after one batch of
// old-block loads.
__device__ __forceinline__ void twist_into(const uint32_t *o, uint32_t *nw, uint32_t lane)
{
    constexpr uint32_t H = kMtN - kMtM;  // 227
    uint32_t oa[4], ob[4], oc[4], pb[4], qb[4], pc[4], qc[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t m = min(lane + 64u * r, H - 1);
        oa[r] = o[m];
        ob[r] = o[m + 1];
        oc[r] = o[m + kMtM];
        pb[r] = o[m + H];
        qb[r] = o[m + H + 1];
        pc[r] = o[min(m + 2 * H, kMtN - 1)];
        qc[r] = o[min(m + 2 * H + 1, kMtN - 1)];
    }
    uint32_t A[4], B[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        A[r] = mtj_mix(oa[r], ob[r], oc[r]);
        B[r] = mtj_mix(pb[r], qb[r], A[r]);
    }
    const uint32_t nw0 = __builtin_amdgcn_readlane(A[0], 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t m = lane + 64u * r;
        if (m < H) {
            nw[m] = A[r];
            nw[m + H] = B[r];
            if (m + 2 * H < kMtN)
                nw[m + 2 * H] = mtj_mix(pc[r], m + 2 * H == kMtN - 1 ? nw0 : qc[r], B[r]);
        }
    }
}

// x_0 .. x_{kMtSeqWs-1} of the caller's state frame; window 0 and the read index
__global__ __launch_bounds__(256) void k_mt_seq(const uint32_t *__restrict__ state, uint32_t *__restrict__ ws)
{
    __shared__ uint32_t s[kMtN];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < kMtN; i += 256) {
        s[i] = state[i];
        ws[kWsSeq + i] = state[i];
        ws[kWsWin + i] = state[i];  // generator 0 starts from the state itself
    }
    if (tid == 0)
        ws[0] = state[kMtN];
    __syncthreads();
    for (uint32_t b = 1; b < kMtSeqWs / kMtN; ++b) {
        // block-wide twist: the three phases with barriers
        uint32_t v = 0;
        constexpr uint32_t H = kMtN - kMtM;
        if (tid < H)
            v = mtj_mix(s[tid], s[tid + 1], s[tid + kMtM]);
        __syncthreads();
        if (tid < H)
            s[tid] = v;
        __syncthreads();
        if (tid < H)
            v = mtj_mix(s[H + tid], s[H + tid + 1], s[tid]);
        __syncthreads();
        if (tid < H)
            s[H + tid] = v;
        __syncthreads();
        const uint32_t k = 2 * H + tid;
        if (k < kMtN - 1)
            v = mtj_mix(s[k], s[k + 1], s[k - H]);
        else if (k == kMtN - 1)
            v = mtj_mix(s[k], s[0], s[k - H]);
        __syncthreads();
        if (k < kMtN)
            s[k] = v;
        __syncthreads();
        for (uint32_t i = tid; i < kMtN; i += 256)
            ws[kWsSeq + (uint64_t)b * kMtN + i] = s[i];
        __syncthreads();
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
                                                           uint32_t jumps)
{
    __shared__ uint4 cp4[4 * kMtJumpQuads];  // copy r: word u = x_{k0 + u + r + 1}
    __shared__ alignas(16) uint32_t pos[kMtJumpBits + 8];  // byte offset of set bit kk in its copy: ((kk&3)*Q + (kk>>2)) * 16
    __shared__ uint32_t cnt[kMtJumpWords + 1];
    uint32_t *cp = reinterpret_cast<uint32_t *>(cp4);
    const uint32_t gi = blockIdx.x / kMtJumpSplit, sp = blockIdx.x % kMtJumpSplit;
    const uint32_t k0 = sp * kMtJumpBits, tid = threadIdx.x;
    const uint32_t *__restrict__ coef = table + (uint64_t)gi * kMtN + sp * kMtJumpWords;
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

// one workgroup of three waves per generator: draws [gJ, min((g+1)J, count))
// into out.  Wave 0 twists block t+1 into the other buffer while waves 1-2
// temper block t and store it (one barrier per block): the serial chain is the
// twist alone, the tempering and the HBM stores ride beside it.
constexpr uint32_t kMtGenThreads = 192;

__global__ __launch_bounds__(kMtGenThreads) void k_mt_gen(uint32_t *__restrict__ ws, uint64_t gens, uint64_t count,
                                                         uint32_t *__restrict__ out, uint32_t *__restrict__ state)
{
    __shared__ uint32_t buf[2][kMtN];
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    const uint64_t g = blockIdx.x;
    if (g == 0)
        for (uint32_t i = tid; i < kMtN; i += kMtGenThreads)
            buf[0][i] = ws[kWsWin + i];
    else
        for (uint32_t i = tid; i < kMtN; i += kMtGenThreads) {
            uint32_t v = 0;
#pragma unroll
            for (uint32_t sp = 0; sp < kMtJumpSplit; ++sp)
                v ^= ws[kWsPart + (sp * (gens - 1) + g - 1) * kMtN + i];
            buf[0][i] = v;
        }
    const uint32_t ptr0 = ws[0];
    __syncthreads();
    const uint64_t pos0 = g * kMtJ, end = min(pos0 + kMtJ, count);
    const uint32_t head = ptr0 < kMtN ? (uint32_t)min((uint64_t)(kMtN - ptr0), end - pos0) : 0u;  // rest of block 0
    const uint64_t rest = end - pos0 - head;
    const uint32_t twists = (uint32_t)((rest + kMtN - 1) / kMtN);
    const uint32_t ct = tid - 64u;  // consumer thread 0..127
    for (uint32_t t = 0; t <= twists; ++t) {
        const uint32_t *cur = buf[t & 1u];
        if (wave == 0) {
            if (t < twists)
                twist_into(cur, buf[(t + 1) & 1u], lane);
        } else if (t == 0) {
            for (uint32_t i = ct; i < head; i += 128)
                out[pos0 + i] = mtj_temper(cur[ptr0 + i]);
        } else {
            const uint64_t at = pos0 + head + (uint64_t)(t - 1) * kMtN;
            uint32_t *o = out + at;
            const uint32_t take = (uint32_t)min((uint64_t)kMtN, end - at);
            if (take == kMtN) {
#pragma unroll
                for (uint32_t r = 0; r < 5; ++r) {
                    const uint32_t i = ct + 128u * r;
                    if (r < 4 || i < kMtN)
                        o[i] = mtj_temper(cur[i]);
                }
            } else {
                for (uint32_t i = ct; i < take; i += 128)
                    o[i] = mtj_temper(cur[i]);
            }
        }
        __syncthreads();
    }
    if (g == gens - 1) {  // the advanced state: the last block (aligned to the twist blocks) + read index
        for (uint32_t i = tid; i < kMtN; i += kMtGenThreads)
            state[i] = buf[twists & 1u][i];
        if (tid == 0)
            state[kMtN] = twists ? (uint32_t)(rest - (uint64_t)(twists - 1) * kMtN) : ptr0 + head;
    }
}

}  // namespace gc

using namespace gc;

extern "C" {

size_t gc_mt19937_workspace_size(uint64_t count)
{
    const uint64_t gens = count ? (count + kMtJ - 1) / kMtJ : 1;
    return 4 * (kWsPart + kMtJumpSplit * (gens - 1) * kMtN);
}

int gc_mt19937_generate_jumped(uint32_t *state_dev, const uint32_t *table_dev, uint64_t table_gens, uint32_t *out,
                               uint64_t count, void *workspace, gc_stream_t stream)
{
    GC_REQUIRE(state_dev && workspace, "gc_mt19937_generate_jumped: null state/workspace");
    GC_REQUIRE(count == 0 || out, "gc_mt19937_generate_jumped: null out");
    if (count == 0)
        return GC_OK;
    const uint64_t gens = (count + kMtJ - 1) / kMtJ;
    GC_REQUIRE(gens - 1 <= table_gens && (gens == 1 || table_dev),
               "gc_mt19937_generate_jumped: jump table holds %llu generators, %llu draws need %llu",
               (unsigned long long)table_gens, (unsigned long long)count, (unsigned long long)(gens - 1));
    GC_REQUIRE(gens <= 0x7fffffffull / kMtJumpSplit, "gc_mt19937_generate_jumped: count too large");
    hipStream_t st = as_stream(stream);
    uint32_t *ws = reinterpret_cast<uint32_t *>(workspace);
    hipLaunchKernelGGL(k_mt_seq, dim3(1), dim3(256), 0, st, state_dev, ws);
    if (gens > 1)
        hipLaunchKernelGGL(k_mt_jump, dim3((unsigned)((gens - 1) * kMtJumpSplit)), dim3(kMtJumpThreads), 0, st, table_dev,
                           ws, (uint32_t)(gens - 1));
    hipLaunchKernelGGL(k_mt_gen, dim3((unsigned)gens), dim3(kMtGenThreads), 0, st, ws, gens, count, out, state_dev);
    return launch_status("gc_mt19937_generate_jumped");
}

}  // extern "C"
