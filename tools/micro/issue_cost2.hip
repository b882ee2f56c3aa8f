// Microbenchmark (development aid): SIMD issue cost of more VALU forms on gfx950, 8 independent
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
K1(k0, "v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %4\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4")
K1(k1, "v_add_f32_e64 %0, |%0|, %4\n v_add_f32_e64 %1, |%1|, %4\n v_add_f32_e64 %2, |%2|, %4\n v_add_f32_e64 %3, |%3|, %4")
K1(k2, "v_sub_f32 %0, %4, %0\n v_sub_f32 %1, %4, %1\n v_sub_f32 %2, %4, %2\n v_sub_f32 %3, %4, %3")
K1(k3, "v_mul_f32 %0, %0, %4\n v_mul_f32 %1, %1, %4\n v_mul_f32 %2, %2, %4\n v_mul_f32 %3, %3, %4")
K1(k4, "v_fmac_f32 %0, %4, %4\n v_fmac_f32 %1, %4, %4\n v_fmac_f32 %2, %4, %4\n v_fmac_f32 %3, %4, %4")
K1(k5, "v_fma_f32 %0, %0, %4, %4\n v_fma_f32 %1, %1, %4, %4\n v_fma_f32 %2, %2, %4, %4\n v_fma_f32 %3, %3, %4, %4")
K1(k6, "v_min_f32 %0, %0, %4\n v_min_f32 %1, %1, %4\n v_min_f32 %2, %2, %4\n v_min_f32 %3, %3, %4")
K1(k7, "v_max_f32_e64 %0, |%0|, %4\n v_max_f32_e64 %1, |%1|, %4\n v_max_f32_e64 %2, |%2|, %4\n v_max_f32_e64 %3, |%3|, %4")
K1(k8, "v_med3_f32 %0, -|%0|, %4, |%0|\n v_med3_f32 %1, -|%1|, %4, |%1|\n v_med3_f32 %2, -|%2|, %4, |%2|\n v_med3_f32 %3, -|%3|, %4, |%3|")
K1(k9, "v_mov_b32 %0, %4\n v_mov_b32 %1, %4\n v_mov_b32 %2, %4\n v_mov_b32 %3, %4")
K1(k10, "v_xor_b32 %0, %0, %4\n v_xor_b32 %1, %1, %4\n v_xor_b32 %2, %2, %4\n v_xor_b32 %3, %3, %4")
K1(k11, "v_and_b32 %0, %0, %4\n v_and_b32 %1, %1, %4\n v_and_b32 %2, %2, %4\n v_and_b32 %3, %3, %4")
K1(k12, "v_or_b32 %0, %0, %4\n v_or_b32 %1, %1, %4\n v_or_b32 %2, %2, %4\n v_or_b32 %3, %3, %4")
K1(k13, "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4")
K1(k14, "v_min_u32 %0, %0, %4\n v_min_u32 %1, %1, %4\n v_min_u32 %2, %2, %4\n v_min_u32 %3, %3, %4")
K1(k15, "v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n v_cndmask_b32 %2, %2, %4, vcc\n v_cndmask_b32 %3, %3, %4, vcc")
K1(k16, "v_bfi_b32 %0, %4, %0, %4\n v_bfi_b32 %1, %4, %1, %4\n v_bfi_b32 %2, %4, %2, %4\n v_bfi_b32 %3, %4, %3, %4")
K1(k17, "v_bfe_u32 %0, %0, 3, 1\n v_bfe_u32 %1, %1, 3, 1\n v_bfe_u32 %2, %2, 3, 1\n v_bfe_u32 %3, %3, 3, 1")
K1(k18, "v_lshl_or_b32 %0, %0, 1, %4\n v_lshl_or_b32 %1, %1, 1, %4\n v_lshl_or_b32 %2, %2, 1, %4\n v_lshl_or_b32 %3, %3, 1, %4")
K1(k19, "v_and_or_b32 %0, %0, %4, %4\n v_and_or_b32 %1, %1, %4, %4\n v_and_or_b32 %2, %2, %4, %4\n v_and_or_b32 %3, %3, %4, %4")
K1(k20, "v_xad_u32 %0, %0, %4, %4\n v_xad_u32 %1, %1, %4, %4\n v_xad_u32 %2, %2, %4, %4\n v_xad_u32 %3, %3, %4, %4")
K1(k21, "v_perm_b32 %0, %0, %4, %4\n v_perm_b32 %1, %1, %4, %4\n v_perm_b32 %2, %2, %4, %4\n v_perm_b32 %3, %3, %4, %4")
K1(k22, "v_ldexp_f32 %0, %0, 1\n v_ldexp_f32 %1, %1, 1\n v_ldexp_f32 %2, %2, 1\n v_ldexp_f32 %3, %3, 1")
K1(k23, "v_cvt_f32_u32 %0, %0\n v_cvt_f32_u32 %1, %1\n v_cvt_f32_u32 %2, %2\n v_cvt_f32_u32 %3, %3")
K1(k24, "v_mul_lo_u32 %0, %0, %4\n v_mul_lo_u32 %1, %1, %4\n v_mul_lo_u32 %2, %2, %4\n v_mul_lo_u32 %3, %3, %4")
typedef float f2 __attribute__((ext_vector_type(2)));
#define PK(NAME, OP) __global__ __launch_bounds__(64) void NAME(float* out, float a) { f2 x[4]; \
    for (int i = 0; i < 4; ++i) x[i] = f2{threadIdx.x * 0.001f + i, i * 0.5f}; const f2 av = {a, a}; \
    for (int it = 0; it < ITER; ++it) { \
        asm volatile(OP " %0, %0, %4\n " OP " %1, %1, %4\n " OP " %2, %2, %4\n " OP " %3, %3, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av)); \
        asm volatile(OP " %0, %0, %4\n " OP " %1, %1, %4\n " OP " %2, %2, %4\n " OP " %3, %3, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av)); } \
    out[blockIdx.x * 64 + threadIdx.x] = x[0].x + x[1].y + x[2].x + x[3].y; }
PK(kpkmul, "v_pk_mul_f32")
__global__ __launch_bounds__(64) void kpkfma(float* out, float a) { f2 x[4];
    for (int i = 0; i < 4; ++i) x[i] = f2{threadIdx.x * 0.001f + i, i * 0.5f}; const f2 av = {a, a};
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_pk_fma_f32 %0, %0, %4, %4\n v_pk_fma_f32 %1, %1, %4, %4\n v_pk_fma_f32 %2, %2, %4, %4\n v_pk_fma_f32 %3, %3, %4, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av));
        asm volatile("v_pk_fma_f32 %0, %0, %4, %4\n v_pk_fma_f32 %1, %1, %4, %4\n v_pk_fma_f32 %2, %2, %4, %4\n v_pk_fma_f32 %3, %3, %4, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av)); }
    out[blockIdx.x * 64 + threadIdx.x] = x[0].x + x[1].y + x[2].x + x[3].y; }
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
    struct { const char* n; void (*k)(float*, float); } ks[] = {{"v_add_f32 (vop2)", k0}, {"v_add_f32_e64 abs (vop3)", k1}, {"v_sub_f32", k2}, {"v_mul_f32", k3}, {"v_fmac_f32 (vop2)", k4}, {"v_fma_f32 (vop3)", k5}, {"v_min_f32 (vop2)", k6}, {"v_max_f32 abs (vop3)", k7}, {"v_med3_f32", k8}, {"v_mov_b32", k9}, {"v_xor_b32", k10}, {"v_and_b32", k11}, {"v_or_b32", k12}, {"v_add_u32", k13}, {"v_min_u32", k14}, {"v_cndmask_b32 (vcc)", k15}, {"v_bfi_b32", k16}, {"v_bfe_u32", k17}, {"v_lshl_or_b32", k18}, {"v_and_or_b32", k19}, {"v_xad_u32", k20}, {"v_perm_b32", k21}, {"v_ldexp_f32", k22}, {"v_cvt_f32_u32", k23}, {"v_mul_lo_u32", k24}, {"v_pk_mul_f32", kpkmul}, {"v_pk_fma_f32", kpkfma}};
    for (auto& k : ks) printf("%-32s %.3f ns per wave-instruction per SIMD\n", k.n, run(k.k, out, blocks) * 1e6 / instr);
    return 0;
}
