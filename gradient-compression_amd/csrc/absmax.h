// absmax.h — the max-norm scan (reducer.py:516 buffer.abs().max()) shared by
// qsgd.hip (product), segments.hip (fused flatten) and tools/encode_lab.hip.
//
// uint max over |x| bit patterns (exact, order-free, NaN wins like
// torch.max), wave64 shuffle tree, wave partials in LDS, one partial per
// block.  Without a workspace: one atomicMax per block into *norm (zeroed by
// a preceding hipMemsetAsync).  With a workspace: no memset launch — every
// block stores its partial (sc1) and takes a ticket of its group (block b in
// group b mod 16, one XCD's blocks; agent-scope atomic add); the block that
// draws its group's last ticket takes a top-level ticket, and the block that
// draws the last of those reduces the partials (sc1 loads), writes *norm and
// re-arms the tickets.  Two levels because same-address atomics serialise
// (~88/us, MI355X_MICROARCH.md 'dequeue'): 256 blocks on one ticket held the
// kernel's end ~2.9 us behind its last load (17.2 against 14.4 us for the
// plain read of the ResNet50 bucket, profiles/r05j lab_ms); 16 + 16 adds on
// 17 lines take ~0.4 us.
//
// The hand-off is fence-free and rests on a gfx950 hardware property, not on
// the HIP memory model: every partial is stored sc1 (write-through past the
// XCD L2) and drained (s_waitcnt vmcnt(0)) before its block's relaxed
// agent-scope ticket add, and the last block reads the partials with sc1
// loads (L1 bypassed) only after its add returned — row 1 of the sc1 hand-off
// table of MI355X_MICROARCH.md ("measured on gfx950 / ROCm 7.2, not an
// architectural guarantee").  The release / acquire form the model asks for
// costs a buffer_wbl2 per block (~1.7 us each, same guide) and a buffer_inv in
// the last block; it measured 2x slower than the memset it removes
// (include/gcodec.h states the assumption).  GC_STRICT_HANDOFF=1 builds that
// form instead (make strict -> lib/libgcodec_strict.so; plain partial stores,
// an agent release fence before the ticket, an agent acquire in the last
// block, plain loads), so the hardware assumption can be switched off;
// tests/test_gpu_strict_handoff.py checks the two builds agree.  Launchers cap
// the grid at kAbsmaxMaxBlocks = 1024 partials.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gc_device.h"

#ifndef GC_STRICT_HANDOFF
#define GC_STRICT_HANDOFF 0
#endif

namespace gc {

constexpr unsigned kAbsmaxThreads = 1024;  // product block size
constexpr unsigned kAbsmaxMaxBlocks = 1024;  // block partials in the workspace
// workspace (uint32 words): [0] top-level ticket, [kWsGroup (g + 1)] the
// ticket of group g (each on a 128-byte line of its own), [kWsPart + b] block
// partials
constexpr unsigned kAbsmaxGroups = 16;
constexpr unsigned kWsGroup = 32;
constexpr unsigned kWsPart = kWsGroup * (kAbsmaxGroups + 1);
constexpr unsigned kAbsmaxWsWords = kWsPart + kAbsmaxMaxBlocks;

__device__ __forceinline__ uint32_t absbits(float v) { return __float_as_uint(v) & 0x7fffffffu; }

__device__ __forceinline__ uint32_t absbits4(float4 a)
{
    return max(max(absbits(a.x), absbits(a.y)), max(absbits(a.z), absbits(a.w)));
}

__device__ __forceinline__ void sc1_store(uint32_t *p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t sc1_load(const uint32_t *p)
{
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// block max of m (valid in thread 0)
template <unsigned BT>
__device__ __forceinline__ uint32_t block_max(uint32_t m, uint32_t *part)
{
    m = wave_max_u32(m);
    __syncthreads();
    if ((threadIdx.x & 63) == 0)
        part[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0)
        for (unsigned w = 1; w < BT / 64; ++w)
            m = max(m, part[w]);
    return m;
}

// the block partials' hand-off: sc1 stores / loads, or (GC_STRICT_HANDOFF)
// plain ones ordered by the release / acquire fences around the ticket
__device__ __forceinline__ void part_store(uint32_t *p, uint32_t v)
{
#if GC_STRICT_HANDOFF
    *p = v;
#else
    sc1_store(p, v);
#endif
}
__device__ __forceinline__ uint32_t part_load(const uint32_t *p)
{
#if GC_STRICT_HANDOFF
    return *p;
#else
    return sc1_load(p);
#endif
}

// max over `count` handed-off partials by the whole block (valid in thread 0)
template <unsigned BT>
__device__ __forceinline__ uint32_t block_max_sc1(const uint32_t *p, uint32_t count, uint32_t *part)
{
    uint32_t v = 0;
    for (uint32_t i = threadIdx.x; i < count; i += BT)
        v = max(v, part_load(&p[i]));
    return block_max<BT>(v, part);
}

// G: ticket groups (1 = every block on one group ticket: the single-level
// chain, kept for the A/B in tools/lab_ms.hip)
template <bool WS, unsigned BT = kAbsmaxThreads, unsigned G = kAbsmaxGroups>
__device__ __forceinline__ void absmax_finish(uint32_t m, uint32_t *__restrict__ out, uint32_t *__restrict__ ws)
{
    __shared__ uint32_t part[BT / 64];
    __shared__ int last;
    m = block_max<BT>(m, part);
    if constexpr (!WS) {
        if (threadIdx.x == 0 && m)
            atomicMax(out, m);
        return;
    } else {
        const uint32_t nb = gridDim.x;  // <= kAbsmaxMaxBlocks (launchers)
        if (threadIdx.x == 0) {
            // sc1 store, drained, then the agent-scope tickets: the fence-free
            // hand-off of MI355X_MICROARCH.md (row 1 of the sc1 table), chained
            // through the group's last block (its top-level add is issued only
            // after its group add returned, i.e. after every add of the group)
            static_assert(G >= 1 && G <= kAbsmaxGroups, "ticket groups");
            const uint32_t g = blockIdx.x % G;
            const uint32_t ng = min(nb, G), cnt = (nb - g + G - 1) / G;
            part_store(&ws[kWsPart + blockIdx.x], m);
#if GC_STRICT_HANDOFF
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bool l = false;
            if (__hip_atomic_fetch_add(&ws[kWsGroup * (g + 1)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                cnt - 1) {
#if GC_STRICT_HANDOFF
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");  // the group's partials on to the top level
#endif
                l = __hip_atomic_fetch_add(&ws[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
            }
#if GC_STRICT_HANDOFF
            if (l) {  // the acquire, then (barrier below) every wave's plain loads
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
#endif
            last = l;
        }
        __syncthreads();  // the other waves load only after the last add returned
        if (!last)
            return;
        const uint32_t r = block_max_sc1<BT>(&ws[kWsPart], nb, part);
        if (threadIdx.x == 0)
            *out = r;
        if (threadIdx.x <= G)  // re-arm: every ticket has reached its count
            sc1_store(&ws[kWsGroup * threadIdx.x], 0u);
    }
}

// MODE 0: float4 dense, 1: scalar dense, 2: gather.  U float4 loads in flight
// per thread; NT: nontemporal loads (streamed once).  (Round 5 measured a
// reverse walk meant to leave x's front in the Infinity Cache for the encode:
// no gain, DESIGN_HISTORY §5.1.)
template <int MODE, bool WS, unsigned BT = kAbsmaxThreads, int U = 4, bool NT = false, unsigned G = kAbsmaxGroups>
__global__ __launch_bounds__(BT) void k_absmax(const float *__restrict__ x, const int64_t *__restrict__ idx,
                                               uint64_t n, uint32_t *__restrict__ out, uint32_t *__restrict__ ws)
{
    uint32_t m = 0;
    const uint64_t stride = (uint64_t)gridDim.x * BT;
    uint64_t t = (uint64_t)blockIdx.x * BT + threadIdx.x;
    if constexpr (MODE == 0) {
        const float4 *x4 = reinterpret_cast<const float4 *>(x);
        const uint64_t n4 = n >> 2;
        for (; t + (U - 1) * stride < n4; t += U * stride) {
            float4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                v[u] = NT ? ld_nt(x4 + t + u * stride) : x4[t + u * stride];
#pragma unroll
            for (int u = 0; u < U; ++u)
                m = max(m, absbits4(v[u]));
        }
        for (; t < n4; t += stride)
            m = max(m, absbits4(x4[t]));
        if (blockIdx.x == 0 && threadIdx.x < (n & 3))
            m = max(m, absbits(x[(n4 << 2) + threadIdx.x]));
    } else {
        for (; t < n; t += stride)
            m = max(m, absbits(MODE == 2 ? x[idx[t]] : x[t]));
    }
    absmax_finish<WS, BT, G>(m, out, ws);
}

}  // namespace gc
