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

#include "absmax.h"
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
            st_nt4(d, v);
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

}  // namespace gc
