// capi.cpp — library-level C ABI: version, errors, device check, layouts.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <string>

#include "gc_host.h"

#ifndef GC_VERSION_STRING
#define GC_VERSION_STRING "gcodec 0.1.0 (gfx950)"
#endif

namespace gc {

static thread_local std::string g_last_error;

int fail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

int launch_status(const char *what)
{
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(GC_EHIP, "%s: %s", what, hipGetErrorString(e));
    return GC_OK;
}

unsigned grid_for(uint64_t items, unsigned max_blocks)
{
    // 256 CUs x 8 resident 256-thread blocks; grid-stride beyond that
    if (max_blocks == 0)
        max_blocks = 256u * 8u;
    uint64_t b = (items + kBlockHost - 1) / kBlockHost;
    if (b == 0)
        b = 1;
    return (unsigned)(b < max_blocks ? b : max_blocks);
}

int check_bits(uint32_t bits, const char *what)
{
    if (bits < 1 || bits > 24)
        return fail(GC_EINVAL, "%s: quantization bits %u outside [1, 24]", what, bits);
    return GC_OK;
}

int check_levels(const gc_levels *lv, const char *what)
{
    if (!lv || lv->count < 1 || lv->count > GC_MAX_LEVELS)
        return fail(GC_EINVAL, "%s: level count must be in [1, %d]", what, GC_MAX_LEVELS);
    for (uint32_t i = 0; i < lv->count; ++i) {
        if (lv->bits[i] < 1 || lv->bits[i] > 24)
            return fail(GC_EINVAL, "%s: level %u bits %u outside [1, 24]", what, i, lv->bits[i]);
        if (i && lv->bits[i] < lv->bits[i - 1])
            return fail(GC_EINVAL, "%s: levels must be sorted ascending (compressors.py:768)", what);
    }
    return GC_OK;
}

int check_lanes(const gc_lanes *l, uint64_t n, const char *what)
{
    if (!l)
        return fail(GC_EINVAL, "%s: null lane layout", what);
    gc_lanes ref;
    int rc = gc_lane_layout(l->n, l->range, l->world, l->offset, &ref);
    if (rc != GC_OK)
        return rc;
    // plane_words may exceed the minimal layout's (the multi-scale layouts couple
    // the mask and q plane sizes, gc_ms_layout) but keeps its alignment
    const uint64_t align = l->plane_words >= 65536 ? 64 : 4;
    if (ref.bits != l->bits || ref.per_word != l->per_word || l->plane_words < ref.plane_words ||
        l->plane_words % align)
        return fail(GC_EINVAL, "%s: lane layout inconsistent with (n, range, world)", what);
    if (l->n != n)
        return fail(GC_EINVAL, "%s: lane layout is for n=%llu, call has n=%llu", what,
                    (unsigned long long)l->n, (unsigned long long)n);
    return GC_OK;
}

}  // namespace gc

extern "C" {

const char *gc_version(void) { return GC_VERSION_STRING; }
const char *gc_last_error(void) { return gc::g_last_error.c_str(); }
int gc_abi_version(void) { return GC_ABI_VERSION; }

int gc_device_check(int device)
{
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess)
        return gc::fail(GC_ENODEV, "no HIP device %d: %s", device, hipGetErrorString(e));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return gc::fail(GC_ENODEV, "device %d is %s, libgcodec is built for gfx950", device, prop.gcnArchName);
    return GC_OK;
}

int gc_lane_layout(uint64_t n, uint64_t range, uint32_t world, uint32_t offset, gc_lanes *out)
{
    GC_REQUIRE(out, "gc_lane_layout: null out");
    GC_REQUIRE(world >= 1, "gc_lane_layout: world must be >= 1");
    GC_REQUIRE(range >= 1, "gc_lane_layout: range must be >= 1");
    GC_REQUIRE(offset <= range, "gc_lane_layout: offset above range");
    GC_REQUIRE(range < (1ull << 32) && (range * world) < (1ull << 32),
               "gc_lane_layout: world*range = %llu does not fit a 32-bit lane",
               (unsigned long long)(range * world));
    uint64_t top = range * (uint64_t)world;
    uint32_t w = 0;
    while ((top >> w) != 0)
        ++w;
    uint32_t L = 32u / w;
    uint64_t m = (n + L - 1) / L;
    // planes start on 256-B boundaries for large streams (a wave's 1 KiB
    // float4 access never straddles a line shared with another XCD's L2);
    // 16 B (all the kernels need) for small ones (GRandK K ~ 1e4)
    m = m >= 65536 ? (m + 63) & ~(uint64_t)63 : (m + 3) & ~(uint64_t)3;
    out->n = n;
    out->plane_words = m;
    out->bits = w;
    out->per_word = L;
    out->offset = offset;
    out->world = world;
    out->range = range;
    return GC_OK;
}

int gc_qsgd_layout(uint64_t n, uint32_t bits, uint32_t world, gc_lanes *out)
{
    int rc = gc::check_bits(bits, "gc_qsgd_layout");
    if (rc)
        return rc;
    uint32_t s = (1u << bits) - 1u;
    return gc_lane_layout(n, 2ull * s, world, s, out);
}

// W = 1 multi-scale layouts are coupled: with r = floor(32 / Lq) (Lq = q lanes
// per word), the q plane size Mq is a multiple of 64 r and the mask plane size
// is Mm = Mq / r, so mask plane P = h + r k holds exactly the elements of q lane
// k of q words h Mm .. (h+1) Mm - 1.  A kernel that owns mask-word quad t then
// owns q-word quads t, t + Mm/4, ..., t + (r-1) Mm/4 whole: the one-pass W = 1
// encode (gc_ms_encode_w1) writes both streams without exchanging lanes between
// blocks.  Mask planes P >= r Lq stay empty (r Lq of the 32 used: 30 for the
// 2-bit lower level, a mask stream 6.7% above the minimum).
static int ms_q_lanes(uint64_t n, const gc_levels *levels, uint32_t world, gc_lanes *out, uint32_t *r)
{
    // |q| <= s_0 for two levels; <= s_0 + 1 for three or more (a rank whose own
    // mask is above the common one may round level m up by one).
    uint32_t qmax = (1u << levels->bits[0]) - 1u + (levels->count >= 3 ? 1u : 0u);
    int rc = gc_lane_layout(n, 2ull * qmax, world, qmax, out);
    if (rc || world != 1 || levels->count < 2)
        return rc;
    const uint32_t rr = 32u / out->per_word;
    const uint64_t q = 64ull * rr;
    out->plane_words = (((n + out->per_word - 1) / out->per_word) + q - 1) / q * q;
    *r = rr;
    return GC_OK;
}

int gc_ms_layout(uint64_t n, const gc_levels *levels, uint32_t world, gc_lanes *out)
{
    int rc = gc::check_levels(levels, "gc_ms_layout");
    if (rc)
        return rc;
    uint32_t r = 0;
    return ms_q_lanes(n, levels, world, out, &r);
}

int gc_ms_mask_layout(uint64_t n, const gc_levels *levels, uint32_t world, gc_lanes *out)
{
    int rc = gc::check_levels(levels, "gc_ms_mask_layout");
    if (rc)
        return rc;
    GC_REQUIRE(levels->count >= 2, "gc_ms_mask_layout: needs >= 2 levels");
    if ((rc = gc_lane_layout(n, 1, world, 0, out)))
        return rc;
    if (world == 1) {  // coupled to the q layout (above)
        gc_lanes ql;
        uint32_t r = 0;
        if ((rc = ms_q_lanes(n, levels, world, &ql, &r)))
            return rc;
        out->plane_words = ql.plane_words / r;
    }
    return GC_OK;
}

}  // extern "C"
