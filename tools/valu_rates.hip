// valu_rates.hip — issue rate of the VALU ops the encode's Philox and
// quantizer use, on gfx950 (measurement tool, not product code).
// 8 independent chains per thread, every op in inline asm so nothing folds.
// Reports wave-instructions per cycle per CU (at the measured clock) and the
// cost relative to v_add_u32.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e_), __LINE__);        \
            return 2;                                                                  \
        }                                                                              \
    } while (0)

constexpr int ITER = 4096;

#define CHAINS8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)

__global__ __launch_bounds__(256) void k_add(uint32_t *out, uint32_t s)
{
    uint32_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j;
    for (int i = 0; i < ITER; ++i) {
#define OP(j) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[j]) : "s"(s));
        CHAINS8(OP)
#undef OP
    }
    uint32_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= a[j];
    if (r == 0x12345u) out[0] = r;
}

__global__ __launch_bounds__(256) void k_bitop3(uint32_t *out, uint32_t s)
{
    uint32_t a[8], b = threadIdx.x * 3u;
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j;
    for (int i = 0; i < ITER; ++i) {
#define OP(j) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[j]) : "v"(b), "s"(s));
        CHAINS8(OP)
#undef OP
    }
    uint32_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= a[j];
    if (r == 0x12345u) out[0] = r;
}

__global__ __launch_bounds__(256) void k_mad64(uint32_t *out, uint32_t s)
{
    uint64_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j;
    for (int i = 0; i < ITER; ++i) {
#define OP(j) asm volatile("v_mad_u64_u32 %0, s[100:101], %1, %2, %0" : "+v"(a[j]) : "v"((uint32_t)a[j]), "s"(s) : "s100", "s101");
        CHAINS8(OP)
#undef OP
    }
    uint64_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= a[j];
    if (r == 0x12345u) out[0] = (uint32_t)r;
}

__global__ __launch_bounds__(256) void k_mulhi(uint32_t *out, uint32_t s)
{
    uint32_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j;
    for (int i = 0; i < ITER; ++i) {
#define OP(j) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[j]) : "s"(s));
        CHAINS8(OP)
#undef OP
    }
    uint32_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= a[j];
    if (r == 0x12345u) out[0] = r;
}

__global__ __launch_bounds__(256) void k_mullo(uint32_t *out, uint32_t s)
{
    uint32_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j;
    for (int i = 0; i < ITER; ++i) {
#define OP(j) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[j]) : "s"(s));
        CHAINS8(OP)
#undef OP
    }
    uint32_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= a[j];
    if (r == 0x12345u) out[0] = r;
}

__global__ __launch_bounds__(256) void k_mul24(uint32_t *out, uint32_t s)
{
    uint32_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j;
    for (int i = 0; i < ITER; ++i) {
#define OP(j) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[j]) : "s"(s));
        CHAINS8(OP)
#undef OP
    }
    uint32_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= a[j];
    if (r == 0x12345u) out[0] = r;
}

__global__ __launch_bounds__(256) void k_pkfma(uint32_t *out, uint32_t s)
{
    float2 a[8];
    for (int j = 0; j < 8; ++j) a[j] = make_float2(threadIdx.x + j, j);
    const float2 b = make_float2(1.0001f, 0.9999f);
    for (int i = 0; i < ITER; ++i) {
#define OP(j) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(b));
        CHAINS8(OP)
#undef OP
    }
    float r = 0;
    for (int j = 0; j < 8; ++j) r += a[j].x + a[j].y;
    if (r == 1234.5f) out[0] = 1;
}

__global__ __launch_bounds__(256) void k_fma(uint32_t *out, uint32_t s)
{
    float a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j;
    const float b = 1.0001f;
    for (int i = 0; i < ITER; ++i) {
#define OP(j) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(b));
        CHAINS8(OP)
#undef OP
    }
    float r = 0;
    for (int j = 0; j < 8; ++j) r += a[j];
    if (r == 1234.5f) out[0] = 1;
}

__global__ __launch_bounds__(256) void k_cvt(uint32_t *out, uint32_t s)
{
    uint32_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j;
    for (int i = 0; i < ITER; ++i) {
#define OP(j) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a[j]));
        CHAINS8(OP)
#undef OP
    }
    uint32_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= a[j];
    if (r == 0x12345u) out[0] = r;
}

template <class K>
static float run(K k, uint32_t *out, unsigned grid)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 12345u);
    hipDeviceSynchronize();
    hipEventRecord(a, 0);
    for (int r = 0; r < 5; ++r)
        hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 12345u);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main()
{
    uint32_t *out;
    CK(hipMalloc(&out, 64));
    int clk_khz = 0;
    CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
    const unsigned grid = 256 * 8;  // 8 blocks (32 waves) per CU
    const double waves = grid * 4.0, instr = waves * ITER * 8.0;
    struct {
        const char *name;
        float ms;
    } r[] = {
        {"v_add_u32", run(k_add, out, grid)},      {"v_bitop3_b32", run(k_bitop3, out, grid)},
        {"v_mad_u64_u32", run(k_mad64, out, grid)}, {"v_mul_hi_u32", run(k_mulhi, out, grid)},
        {"v_mul_lo_u32", run(k_mullo, out, grid)}, {"v_mul_u32_u24", run(k_mul24, out, grid)},
        {"v_fma_f32", run(k_fma, out, grid)},      {"v_pk_fma_f32", run(k_pkfma, out, grid)},
        {"v_cvt_f32_u32", run(k_cvt, out, grid)},
    };
    printf("clock attribute %d kHz; %u blocks x 256 threads, %d x 8 ops per thread\n", clk_khz, grid, ITER);
    for (auto &x : r) {
        const double per_cu_per_s = instr / 256.0 / (x.ms * 1e-3);
        printf("%-16s %8.3f ms  %6.3f wave-instr/cycle/CU (at %.2f GHz)  x%.2f vs add\n", x.name, x.ms,
               per_cu_per_s / (clk_khz * 1e3), clk_khz / 1e6, x.ms / r[0].ms);
    }
    return 0;
}
