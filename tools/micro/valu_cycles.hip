// Calibration of the SQ VALU counters on gfx950 (development aid, tools/prof_r04.sh): kernels of
// one VALU form each (8 independent chains per wave, 8 waves per SIMD: issue-bound), timed here
// by HIP events and counted by rocprofv3 (SQ_INSTS_VALU, SQ_THREAD_CYCLES_VALU,
// SQ_ACTIVE_INST_VALU per dispatch).  Prints ns per wave-instruction per SIMD for each form, so
// the counters' cycles per instruction can be set against the measured issue cost.
//   hipcc --offload-arch=gfx950 -O3 -o valu_cycles tools/micro/valu_cycles.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 4096;
#define KF(NAME, T, INIT, ASM)                                                                      \
    __global__ __launch_bounds__(64) void NAME(float* out, float a) {                               \
        T x[8];                                                                                     \
        for (int i = 0; i < 8; ++i) x[i] = (T)(INIT);                                               \
        const T av = (T)a;                                                                          \
        for (int it = 0; it < ITER; ++it) {                                                         \
            asm volatile(ASM : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av));            \
            asm volatile(ASM : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(av));            \
        }                                                                                           \
        T s = 0;                                                                                    \
        for (int i = 0; i < 8; ++i) s += x[i];                                                      \
        out[blockIdx.x * 64 + threadIdx.x] = (float)s;                                              \
    }
#define X4(OP) OP(0) OP(1) OP(2) OP(3)
KF(k_add_f32, float, threadIdx.x * 0.001f + i,
   "v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %4\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4")
KF(k_fma_f32, float, threadIdx.x * 0.001f + i,
   "v_fma_f32 %0, %0, %4, %4\n v_fma_f32 %1, %1, %4, %4\n v_fma_f32 %2, %2, %4, %4\n v_fma_f32 %3, %3, %4, %4")
KF(k_xor_b32, float, threadIdx.x * 0.001f + i,
   "v_xor_b32 %0, %0, %4\n v_xor_b32 %1, %1, %4\n v_xor_b32 %2, %2, %4\n v_xor_b32 %3, %3, %4")
KF(k_dpp_add, float, threadIdx.x * 0.001f + i,
   "v_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
   " v_add_f32_dpp %1, %1, %1 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
   " v_add_f32_dpp %2, %2, %2 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
   " v_add_f32_dpp %3, %3, %3 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1")
KF(k_exp_f32, float, threadIdx.x * 0.0001f,
   "v_exp_f32 %0, %0\n v_exp_f32 %1, %1\n v_exp_f32 %2, %2\n v_exp_f32 %3, %3")
KF(k_add_f64, double, threadIdx.x * 0.001 + i,
   "v_add_f64 %0, %0, %4\n v_add_f64 %1, %1, %4\n v_add_f64 %2, %2, %4\n v_add_f64 %3, %3, %4")
KF(k_fma_f64, double, threadIdx.x * 0.001 + i,
   "v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4")
KF(k_mul_f64, double, threadIdx.x * 0.001 + i,
   "v_mul_f64 %0, %0, %4\n v_mul_f64 %1, %1, %4\n v_mul_f64 %2, %2, %4\n v_mul_f64 %3, %3, %4")
KF(k_mul_f32, float, threadIdx.x * 0.001f + i,
   "v_mul_f32 %0, %0, %4\n v_mul_f32 %1, %1, %4\n v_mul_f32 %2, %2, %4\n v_mul_f32 %3, %3, %4")
KF(k_bitop3, float, threadIdx.x * 0.001f + i,
   "v_bitop3_b32 %0, %0, %4, %4 bitop3:0x6c\n v_bitop3_b32 %1, %1, %4, %4 bitop3:0x6c\n"
   " v_bitop3_b32 %2, %2, %4, %4 bitop3:0x6c\n v_bitop3_b32 %3, %3, %4, %4 bitop3:0x6c")
KF(k_add_u32, float, threadIdx.x * 0.001f + i,
   "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4")
KF(k_min_f32, float, threadIdx.x * 0.001f + i,
   "v_min_f32 %0, %0, %4\n v_min_f32 %1, %1, %4\n v_min_f32 %2, %2, %4\n v_min_f32 %3, %3, %4")
// f32 -> f64 -> f32 round trips: 16 conversions per asm pair
__global__ __launch_bounds__(64) void k_cvt_f64(float* out, float a) {
    float x[8];
    double t[4];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i + a;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int h = 0; h < 8; h += 4)
            asm volatile(
                "v_cvt_f64_f32 %4, %0\n v_cvt_f32_f64 %0, %4\n v_cvt_f64_f32 %5, %1\n v_cvt_f32_f64 %1, %5\n"
                " v_cvt_f64_f32 %6, %2\n v_cvt_f32_f64 %2, %6\n v_cvt_f64_f32 %7, %3\n v_cvt_f32_f64 %3, %7"
                : "+v"(x[h]), "+v"(x[h + 1]), "+v"(x[h + 2]), "+v"(x[h + 3]), "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]),
                  "=&v"(t[3]));
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}
KF(k_movdpp, float, threadIdx.x * 0.001f + i,
   "v_mov_b32_dpp %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
   " v_mov_b32_dpp %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
   " v_mov_b32_dpp %2, %2 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
   " v_mov_b32_dpp %3, %3 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1")

typedef void (*Kern)(float*, float);

int main() {
    const struct {
        const char* name;
        Kern k;
    } ks[] = {{"v_add_f32", k_add_f32}, {"v_fma_f32", k_fma_f32}, {"v_xor_b32", k_xor_b32},
              {"v_add_f32_dpp", k_dpp_add}, {"v_exp_f32", k_exp_f32}, {"v_add_f64", k_add_f64},
              {"v_fma_f64", k_fma_f64}, {"v_mul_f64", k_mul_f64}, {"v_mul_f32", k_mul_f32},
              {"v_bitop3_b32", k_bitop3}, {"v_add_u32", k_add_u32}, {"v_min_f32", k_min_f32},
              {"v_cvt_f32_f64+f64_f32", k_cvt_f64}, {"v_mov_b32_dpp", k_movdpp}};
    const int blocks = 256 * 4 * 8;  // 8 waves per SIMD
    float* out;
    if (hipMalloc(&out, (size_t)blocks * 64 * sizeof(float)) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 60; ++w) {  // ~0.3 s of load first: the clock leaves its idle state
        for (const auto& k : ks) hipLaunchKernelGGL(k.k, dim3(blocks), dim3(64), 0, 0, out, 1.0001f);
    }
    (void)hipDeviceSynchronize();
    for (const auto& k : ks) {
        float ms = 1e30f;
        for (int r = 0; r < 5; ++r) {  // best of 5
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(64), 0, 0, out, 1.0001f);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float t = 0;
            (void)hipEventElapsedTime(&t, e0, e1);
            ms = t < ms ? t : ms;
        }
        const double instr_per_simd = (double)blocks / 1024.0 * ITER * (k.k == k_cvt_f64 ? 16 : 8);
        printf("%-16s %.3f ns per wave-instruction per SIMD (%.4f ms)\n", k.name, ms * 1e6 / instr_per_simd, ms);
    }
    (void)hipFree(out);
    return 0;
}
