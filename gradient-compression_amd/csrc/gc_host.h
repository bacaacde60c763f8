// gc_host.h — host-side helpers shared by the libgcodec translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gcodec.h"

namespace gc {

constexpr unsigned kBlockHost = 256;  // threads per block of every streaming kernel

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int launch_status(const char *what);  // hipGetLastError -> GC_OK | GC_EHIP

inline hipStream_t as_stream(gc_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
inline bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// grid for a grid-stride streaming kernel over `items` work items
unsigned grid_for(uint64_t items, unsigned max_blocks = 0);

// validate a caller-provided lane layout against its own (n, range, world, offset)
int check_lanes(const gc_lanes *l, uint64_t n, const char *what);
int check_bits(uint32_t bits, const char *what);
int check_levels(const gc_levels *lv, const char *what);

struct SegArg;  // segments.h
// validate a gc_segments for a bucket of n elements and make its kernel argument
int seg_arg(const gc_segments *segs, uint64_t n, SegArg *out, const char *what);

}  // namespace gc

#define GC_REQUIRE(cond, ...)                      \
    do {                                           \
        if (!(cond))                               \
            return ::gc::fail(GC_EINVAL, __VA_ARGS__); \
    } while (0)
