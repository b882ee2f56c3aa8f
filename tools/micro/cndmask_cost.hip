// Microbenchmark (development aid): v_cndmask_b32 with VCC vs an SGPR-pair mask, 8 waves per SIMD,
// 8 independent chains; the masks are written once before the loop (VCC by v_cmp) or inside it.
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int ITER = 2048;
#define BODY4(OP) OP(0) OP(1) OP(2) OP(3)
__global__ __launch_bounds__(64) void k_vcc(float* out, float a) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    asm volatile("v_cmp_gt_f32 vcc, %0, 0.5" ::"v"(x[1]) : "vcc");
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n v_cndmask_b32 %2, %2, %4, vcc\n v_cndmask_b32 %3, %3, %4, vcc" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a));
        asm volatile("v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n v_cndmask_b32 %2, %2, %4, vcc\n v_cndmask_b32 %3, %3, %4, vcc" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a));
    }
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}
__global__ __launch_bounds__(64) void k_sgpr(float* out, float a) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    asm volatile("v_cmp_gt_f32 s[8:9], %0, 0.5" ::"v"(x[1]) : "s8", "s9");
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_cndmask_b32_e64 %0, %0, %4, s[8:9]\n v_cndmask_b32_e64 %1, %1, %4, s[8:9]\n v_cndmask_b32_e64 %2, %2, %4, s[8:9]\n v_cndmask_b32_e64 %3, %3, %4, s[8:9]" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a) : "s8", "s9");
        asm volatile("v_cndmask_b32_e64 %0, %0, %4, s[8:9]\n v_cndmask_b32_e64 %1, %1, %4, s[8:9]\n v_cndmask_b32_e64 %2, %2, %4, s[8:9]\n v_cndmask_b32_e64 %3, %3, %4, s[8:9]" : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a) : "s8", "s9");
    }
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}
// realistic: compare then select, VCC form (v_cmp_e32 + v_cndmask_b32_e32), 4 independent pairs
__global__ __launch_bounds__(64) void k_cmpsel_vcc(float* out, float a) {
    float x[4];
    for (int i = 0; i < 4; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_cmp_gt_f32 vcc, %0, %4\n v_cndmask_b32 %0, %0, %4, vcc\n v_cmp_gt_f32 vcc, %1, %4\n v_cndmask_b32 %1, %1, %4, vcc\n"
                     "v_cmp_gt_f32 vcc, %2, %4\n v_cndmask_b32 %2, %2, %4, vcc\n v_cmp_gt_f32 vcc, %3, %4\n v_cndmask_b32 %3, %3, %4, vcc"
                     : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a) : "vcc");
    }
    out[blockIdx.x * 64 + threadIdx.x] = x[0] + x[1] + x[2] + x[3];
}
__global__ __launch_bounds__(64) void k_cmpsel_sgpr(float* out, float a) {
    float x[4];
    for (int i = 0; i < 4; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_cmp_gt_f32_e64 s[8:9], %0, %4\n v_cmp_gt_f32_e64 s[10:11], %1, %4\n v_cmp_gt_f32_e64 s[12:13], %2, %4\n v_cmp_gt_f32_e64 s[14:15], %3, %4\n"
                     "v_cndmask_b32_e64 %0, %0, %4, s[8:9]\n v_cndmask_b32_e64 %1, %1, %4, s[10:11]\n v_cndmask_b32_e64 %2, %2, %4, s[12:13]\n v_cndmask_b32_e64 %3, %3, %4, s[14:15]"
                     : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a) : "s8", "s9", "s10", "s11", "s12", "s13", "s14", "s15");
    }
    out[blockIdx.x * 64 + threadIdx.x] = x[0] + x[1] + x[2] + x[3];
}
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
    printf("v_cndmask_b32 vcc (mask set once)      %.3f ns\n", run(k_vcc, out, blocks) * 1e6 / instr);
    printf("v_cndmask_b32_e64 sgpr (mask set once) %.3f ns\n", run(k_sgpr, out, blocks) * 1e6 / instr);
    printf("v_cmp vcc + v_cndmask vcc (per pair)   %.3f ns per instruction\n", run(k_cmpsel_vcc, out, blocks) * 1e6 / instr);
    printf("v_cmp_e64 sgpr + v_cndmask_e64         %.3f ns per instruction\n", run(k_cmpsel_sgpr, out, blocks) * 1e6 / instr);
    return 0;
}
