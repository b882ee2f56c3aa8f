// Microbenchmark (development aid): SIMD issue cost of fp64 / misc VALU forms on gfx950, 8 independent
// chains per wave, 8 waves per SIMD (issue-bound).  ns per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int ITER = 2048;
#define K1(NAME, ASM)                                                                          \
    __global__ __launch_bounds__(64) void NAME(float* out, float a) {                          \
        float x[8];                                                                            \
        for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;                           \
        for (int it = 0; it < ITER; ++it) {                                                    \
            asm volatile(ASM : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a));       \
            asm volatile(ASM : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a));       \
        }                                                                                      \
        float s = 0;                                                                           \
        for (int i = 0; i < 8; ++i) s += x[i];                                                 \
        out[blockIdx.x * 64 + threadIdx.x] = s;                                                \
    }
__global__ __launch_bounds__(64) void d0(float* out, float a) {
    double x[8]; const double av = a;
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001 + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_add_f64 %0, %0, %4\n v_add_f64 %1, %1, %4\n v_add_f64 %2, %2, %4\n v_add_f64 %3, %3, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av) : "vcc");
        asm volatile("v_add_f64 %0, %0, %4\n v_add_f64 %1, %1, %4\n v_add_f64 %2, %2, %4\n v_add_f64 %3, %3, %4" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(av) : "vcc");
    }
    double s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s; }
__global__ __launch_bounds__(64) void d1(float* out, float a) {
    double x[8]; const double av = a;
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001 + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_mul_f64 %0, %0, %4\n v_mul_f64 %1, %1, %4\n v_mul_f64 %2, %2, %4\n v_mul_f64 %3, %3, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av) : "vcc");
        asm volatile("v_mul_f64 %0, %0, %4\n v_mul_f64 %1, %1, %4\n v_mul_f64 %2, %2, %4\n v_mul_f64 %3, %3, %4" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(av) : "vcc");
    }
    double s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s; }
__global__ __launch_bounds__(64) void d2(float* out, float a) {
    double x[8]; const double av = a;
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001 + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av) : "vcc");
        asm volatile("v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(av) : "vcc");
    }
    double s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s; }
__global__ __launch_bounds__(64) void d3(float* out, float a) {
    double x[8]; const double av = a;
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001 + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_fmac_f64 %0, %4, %4\n v_fmac_f64 %1, %4, %4\n v_fmac_f64 %2, %4, %4\n v_fmac_f64 %3, %4, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av) : "vcc");
        asm volatile("v_fmac_f64 %0, %4, %4\n v_fmac_f64 %1, %4, %4\n v_fmac_f64 %2, %4, %4\n v_fmac_f64 %3, %4, %4" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(av) : "vcc");
    }
    double s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s; }
__global__ __launch_bounds__(64) void d4(float* out, float a) {
    double x[8]; const double av = a;
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001 + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_min_f64 %0, %0, %4\n v_min_f64 %1, %1, %4\n v_min_f64 %2, %2, %4\n v_min_f64 %3, %3, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av) : "vcc");
        asm volatile("v_min_f64 %0, %0, %4\n v_min_f64 %1, %1, %4\n v_min_f64 %2, %2, %4\n v_min_f64 %3, %3, %4" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(av) : "vcc");
    }
    double s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s; }
__global__ __launch_bounds__(64) void d5(float* out, float a) {
    double x[8]; const double av = a;
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001 + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_max_f64 %0, |%0|, %4\n v_max_f64 %1, |%1|, %4\n v_max_f64 %2, |%2|, %4\n v_max_f64 %3, |%3|, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av) : "vcc");
        asm volatile("v_max_f64 %0, |%0|, %4\n v_max_f64 %1, |%1|, %4\n v_max_f64 %2, |%2|, %4\n v_max_f64 %3, |%3|, %4" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(av) : "vcc");
    }
    double s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s; }
__global__ __launch_bounds__(64) void d6(float* out, float a) {
    double x[8]; const double av = a;
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001 + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_mov_b64 %0, %4\n v_mov_b64 %1, %4\n v_mov_b64 %2, %4\n v_mov_b64 %3, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av) : "vcc");
        asm volatile("v_mov_b64 %0, %4\n v_mov_b64 %1, %4\n v_mov_b64 %2, %4\n v_mov_b64 %3, %4" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(av) : "vcc");
    }
    double s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s; }
__global__ __launch_bounds__(64) void d7(float* out, float a) {
    double x[8]; const double av = a;
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001 + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_ldexp_f64 %0, %0, 1\n v_ldexp_f64 %1, %1, 1\n v_ldexp_f64 %2, %2, 1\n v_ldexp_f64 %3, %3, 1" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av) : "vcc");
        asm volatile("v_ldexp_f64 %0, %0, 1\n v_ldexp_f64 %1, %1, 1\n v_ldexp_f64 %2, %2, 1\n v_ldexp_f64 %3, %3, 1" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(av) : "vcc");
    }
    double s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s; }
__global__ __launch_bounds__(64) void d8(float* out, float a) {
    double x[8]; const double av = a;
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001 + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av) : "vcc");
        asm volatile("v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(av) : "vcc");
    }
    double s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s; }
__global__ __launch_bounds__(64) void d9(float* out, float a) {
    double x[8]; const double av = a;
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001 + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_cmp_gt_f64 vcc, %0, %4\n v_cmp_gt_f64 vcc, %1, %4\n v_cmp_gt_f64 vcc, %2, %4\n v_cmp_gt_f64 vcc, %3, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av) : "vcc");
        asm volatile("v_cmp_gt_f64 vcc, %0, %4\n v_cmp_gt_f64 vcc, %1, %4\n v_cmp_gt_f64 vcc, %2, %4\n v_cmp_gt_f64 vcc, %3, %4" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(av) : "vcc");
    }
    double s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s; }
__global__ __launch_bounds__(64) void d10(float* out, float a) {
    double x[8]; const double av = a;
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001 + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_cmp_gt_i64 vcc, %0, %4\n v_cmp_gt_i64 vcc, %1, %4\n v_cmp_gt_i64 vcc, %2, %4\n v_cmp_gt_i64 vcc, %3, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av) : "vcc");
        asm volatile("v_cmp_gt_i64 vcc, %0, %4\n v_cmp_gt_i64 vcc, %1, %4\n v_cmp_gt_i64 vcc, %2, %4\n v_cmp_gt_i64 vcc, %3, %4" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(av) : "vcc");
    }
    double s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s; }
__global__ __launch_bounds__(64) void d11(float* out, float a) {
    double x[8]; const double av = a;
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001 + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_lshl_add_u64 %0, %0, 1, %4\n v_lshl_add_u64 %1, %1, 1, %4\n v_lshl_add_u64 %2, %2, 1, %4\n v_lshl_add_u64 %3, %3, 1, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av) : "vcc");
        asm volatile("v_lshl_add_u64 %0, %0, 1, %4\n v_lshl_add_u64 %1, %1, 1, %4\n v_lshl_add_u64 %2, %2, 1, %4\n v_lshl_add_u64 %3, %3, 1, %4" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(av) : "vcc");
    }
    double s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s; }
__global__ __launch_bounds__(64) void s0(float* out, float a) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_cndmask_b32_e64 %0, %0, %4, s[8:9]\n v_cndmask_b32_e64 %1, %1, %4, s[8:9]\n v_cndmask_b32_e64 %2, %2, %4, s[8:9]\n v_cndmask_b32_e64 %3, %3, %4, s[8:9]" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a) : "vcc", "s8", "s9");
        asm volatile("v_cndmask_b32_e64 %0, %0, %4, s[8:9]\n v_cndmask_b32_e64 %1, %1, %4, s[8:9]\n v_cndmask_b32_e64 %2, %2, %4, s[8:9]\n v_cndmask_b32_e64 %3, %3, %4, s[8:9]" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a) : "vcc", "s8", "s9");
    }
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s; }
__global__ __launch_bounds__(64) void s2(float* out, float a) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_mul_lo_u32 %0, %0, %4\n v_mul_lo_u32 %1, %1, %4\n v_mul_lo_u32 %2, %2, %4\n v_mul_lo_u32 %3, %3, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a) : "vcc", "s8", "s9");
        asm volatile("v_mul_lo_u32 %0, %0, %4\n v_mul_lo_u32 %1, %1, %4\n v_mul_lo_u32 %2, %2, %4\n v_mul_lo_u32 %3, %3, %4" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a) : "vcc", "s8", "s9");
    }
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s; }
__global__ __launch_bounds__(64) void s3(float* out, float a) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_exp_f32 %0, %0\n v_exp_f32 %1, %1\n v_exp_f32 %2, %2\n v_exp_f32 %3, %3" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a) : "vcc", "s8", "s9");
        asm volatile("v_exp_f32 %0, %0\n v_exp_f32 %1, %1\n v_exp_f32 %2, %2\n v_exp_f32 %3, %3" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a) : "vcc", "s8", "s9");
    }
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s; }
__global__ __launch_bounds__(64) void s4(float* out, float a) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_log_f32 %0, %0\n v_log_f32 %1, %1\n v_log_f32 %2, %2\n v_log_f32 %3, %3" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a) : "vcc", "s8", "s9");
        asm volatile("v_log_f32 %0, %0\n v_log_f32 %1, %1\n v_log_f32 %2, %2\n v_log_f32 %3, %3" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a) : "vcc", "s8", "s9");
    }
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s; }
__global__ __launch_bounds__(64) void s5(float* out, float a) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_add_co_u32 %0, vcc, %0, %4\n v_add_co_u32 %1, vcc, %1, %4\n v_add_co_u32 %2, vcc, %2, %4\n v_add_co_u32 %3, vcc, %3, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a) : "vcc", "s8", "s9");
        asm volatile("v_add_co_u32 %0, vcc, %0, %4\n v_add_co_u32 %1, vcc, %1, %4\n v_add_co_u32 %2, vcc, %2, %4\n v_add_co_u32 %3, vcc, %3, %4" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a) : "vcc", "s8", "s9");
    }
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s; }
__global__ __launch_bounds__(64) void s6(float* out, float a) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_addc_co_u32 %0, vcc, %0, %4, vcc\n v_addc_co_u32 %1, vcc, %1, %4, vcc\n v_addc_co_u32 %2, vcc, %2, %4, vcc\n v_addc_co_u32 %3, vcc, %3, %4, vcc" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a) : "vcc", "s8", "s9");
        asm volatile("v_addc_co_u32 %0, vcc, %0, %4, vcc\n v_addc_co_u32 %1, vcc, %1, %4, vcc\n v_addc_co_u32 %2, vcc, %2, %4, vcc\n v_addc_co_u32 %3, vcc, %3, %4, vcc" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a) : "vcc", "s8", "s9");
    }
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s; }
__global__ __launch_bounds__(64) void s7(float* out, float a) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_add3_u32 %0, %0, %4, %4\n v_add3_u32 %1, %1, %4, %4\n v_add3_u32 %2, %2, %4, %4\n v_add3_u32 %3, %3, %4, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a) : "vcc", "s8", "s9");
        asm volatile("v_add3_u32 %0, %0, %4, %4\n v_add3_u32 %1, %1, %4, %4\n v_add3_u32 %2, %2, %4, %4\n v_add3_u32 %3, %3, %4, %4" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a) : "vcc", "s8", "s9");
    }
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s; }
__global__ __launch_bounds__(64) void kcvt(float* out, float a) {
    double x[4]; float y[4];
    for (int i = 0; i < 4; ++i) y[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER * 2; ++it) {
        asm volatile("v_cvt_f64_f32 %0, %4\n v_cvt_f64_f32 %1, %5\n v_cvt_f64_f32 %2, %6\n v_cvt_f64_f32 %3, %7" : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]) : "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]));
        asm volatile("v_cvt_f32_f64 %0, %4\n v_cvt_f32_f64 %1, %5\n v_cvt_f32_f64 %2, %6\n v_cvt_f32_f64 %3, %7" : "=v"(y[0]), "=v"(y[1]), "=v"(y[2]), "=v"(y[3]) : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]));
    }
    out[blockIdx.x * 64 + threadIdx.x] = y[0] + y[1] + y[2] + y[3] + a; }
__global__ __launch_bounds__(64) void kbperm(float* out, float a) {
    int x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
    const int addr = ((threadIdx.x ^ 5) & 63) << 2;
    for (int it = 0; it < ITER; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_ds_bpermute(addr, x[i]);
    int s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s + a; }
template <class K>
float run(K kern, float* out, int blocks) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    kern<<<blocks, 64>>>(out, 1.0001f);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) kern<<<blocks, 64>>>(out, 1.0001f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    float* out;
    const int w = 8, blocks = 1024 * w;
    (void)hipMalloc(&out, blocks * 64 * sizeof(float));
    const double instr = ITER * 8.0 * w;
    struct { const char* n; void (*k)(float*, float); } ks[] = {{"v_add_f64", d0}, {"v_mul_f64", d1}, {"v_fma_f64", d2}, {"v_fmac_f64", d3}, {"v_min_f64", d4}, {"v_max_f64 abs", d5}, {"v_mov_b64", d6}, {"v_ldexp_f64", d7}, {"v_rcp_f64", d8}, {"v_cmp_gt_f64 (vcc)", d9}, {"v_cmp_gt_i64 (vcc)", d10}, {"v_lshl_add_u64", d11}, {"v_cndmask_b32_e64 (sgpr mask)", s0}, {"v_mul_lo_u32", s2}, {"v_exp_f32", s3}, {"v_log_f32", s4}, {"v_add_co_u32", s5}, {"v_addc_co_u32", s6}, {"v_add3_u32", s7}, {"v_cvt_f64_f32 / v_cvt_f32_f64 (alternating)", kcvt}, {"ds_bpermute_b32 (8 chains)", kbperm}};
    for (auto& k : ks) printf("%-44s %.3f ns per wave-instruction per SIMD\n", k.n, run(k.k, out, blocks) * 1e6 / instr);
    return 0;
}
