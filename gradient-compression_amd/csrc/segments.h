// segments.h — device side of the gc_segments table (include/gcodec.h) and the
// block-level finish of the max-norm scan, shared by k_absmax (qsgd.hip) and
// the fused flatten+absmax (segments.hip).
//
// A gc_segments table describes the reference's TensorBuffer (reducer.py:46-68)
// without materialising it: flat element e lives in tensor s at
// seg[s].ptr[e - seg[s].start].  chunk_seg[e >> shift] is a lower bound on s
// (the first segment holding the chunk's first element), so a lookup is two
// dependent loads (chunk index -> 32-byte record) plus a forward walk over
// the segments that begin inside the chunk — no binary search.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gc_device.h"

namespace gc {

struct SegRec {  // = gc_seg
    uint64_t start, end;
    float *ptr;
    uint64_t reserved;
};

struct SegArg {
    const SegRec *seg;
    const uint32_t *chunk_seg;
    uint64_t count;
    uint32_t shift;
};

struct SegPos {
    uint64_t s;
    SegRec r;
};

__device__ __forceinline__ SegRec seg_rec(const SegArg &sg, uint64_t s) { return sg.seg[s]; }

// the segment holding flat element i (< n)
__device__ __forceinline__ SegPos seg_find(const SegArg &sg, uint64_t i)
{
    SegPos p;
    p.s = sg.chunk_seg[i >> sg.shift];
    p.r = seg_rec(sg, p.s);
    while (i >= p.r.end)  // terminates: i < seg[count-1].end
        p.r = seg_rec(sg, ++p.s);
    return p;
}

__device__ __forceinline__ float seg_pick(const float4 &v, int j) { return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w; }

// flat elements i0 .. i0+3 (those < n) -> their tensors
__device__ __forceinline__ void seg_store4(const SegArg &sg, uint64_t i0, uint64_t n, float4 v)
{
    SegPos p = seg_find(sg, i0);
    if (i0 + 4 <= p.r.end) {
        float *d = p.r.ptr + (i0 - p.r.start);
        if ((reinterpret_cast<uintptr_t>(d) & 15u) == 0) {
            *reinterpret_cast<float4 *>(d) = v;
        } else {
            d[0] = v.x;
            d[1] = v.y;
            d[2] = v.z;
            d[3] = v.w;
        }
        return;
    }
    for (int j = 0; j < 4; ++j) {  // the group straddles a tensor boundary (or the end)
        const uint64_t i = i0 + j;
        if (i >= n)
            return;
        while (i >= p.r.end)
            p.r = seg_rec(sg, ++p.s);
        p.r.ptr[i - p.r.start] = seg_pick(v, j);
    }
}

// ---------------------------------------------------------------------------
// max-norm block finish (see k_absmax in qsgd.hip for the protocol)
// ---------------------------------------------------------------------------
constexpr unsigned kAbsmaxThreads = 1024;
constexpr unsigned kAbsmaxMaxBlocks = 256;

__device__ __forceinline__ uint32_t absbits(float v) { return __float_as_uint(v) & 0x7fffffffu; }

__device__ __forceinline__ uint32_t absbits4(float4 a)
{
    return max(max(absbits(a.x), absbits(a.y)), max(absbits(a.z), absbits(a.w)));
}

template <bool WS>
__device__ __forceinline__ void absmax_finish(uint32_t m, uint32_t *__restrict__ out, uint32_t *__restrict__ ws)
{
    m = wave_max_u32(m);
    __shared__ uint32_t part[kAbsmaxThreads / 64];
    __shared__ int last;
    if ((threadIdx.x & 63) == 0)
        part[threadIdx.x >> 6] = m;
    __syncthreads();
    if constexpr (!WS) {
        if (threadIdx.x == 0) {
            for (unsigned w = 1; w < kAbsmaxThreads / 64; ++w)
                m = max(m, part[w]);
            if (m)
                atomicMax(out, m);
        }
        return;
    } else {
        uint32_t *ticket = ws;
        uint32_t *partials = ws + 16;  // own cache line
        if (threadIdx.x == 0) {
            for (unsigned w = 1; w < kAbsmaxThreads / 64; ++w)
                m = max(m, part[w]);
            // sc1 store, drained, then the agent-scope ticket: the fence-free
            // hand-off of MI355X_MICROARCH.md (row 1 of the sc1 table) — every
            // store and every load of the partials is sc1, hipMalloc memory
            __hip_atomic_store(&partials[blockIdx.x], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t tk = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = tk == gridDim.x - 1;
        }
        __syncthreads();  // the other waves load only after the last add returned
        if (!last)
            return;
        uint32_t v = 0;
        for (uint32_t i = threadIdx.x; i < gridDim.x; i += kAbsmaxThreads)
            v = max(v, __hip_atomic_load(&partials[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        v = wave_max_u32(v);
        __syncthreads();
        if ((threadIdx.x & 63) == 0)
            part[threadIdx.x >> 6] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t r = part[0];
            for (unsigned w = 1; w < kAbsmaxThreads / 64; ++w)
                r = max(r, part[w]);
            *out = r;
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace gc
