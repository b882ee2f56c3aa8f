// Microbenchmark (development aid): 32x32 integer multiply forms on gfx950 (the Philox round of
// csrc/channel_kernel.hip): v_mul_lo_u32, v_mul_hi_u32, v_mad_u64_u32 (both halves at once).
// 8 waves per SIMD, 8 independent chains.  ns per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int ITER = 2048;
__global__ __launch_bounds__(64) void k_lo(float* out, unsigned m) {
    unsigned x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 77u + i;
    for (int it = 0; it < ITER; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[i]) : "v"(m));
    unsigned s = 0;
    for (int i = 0; i < 8; ++i) s ^= x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s;
}
__global__ __launch_bounds__(64) void k_hi(float* out, unsigned m) {
    unsigned x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 77u + i;
    for (int it = 0; it < ITER; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[i]) : "v"(m));
    unsigned s = 0;
    for (int i = 0; i < 8; ++i) s ^= x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s;
}
__global__ __launch_bounds__(64) void k_mad(float* out, unsigned m) {
    unsigned long long x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 77u + i;
    for (int it = 0; it < ITER; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            unsigned lo = (unsigned)x[i];
            asm volatile("v_mad_u64_u32 %0, s[8:9], %1, %2, 0" : "=v"(x[i]) : "v"(lo), "v"(m) : "s8", "s9");
        }
    unsigned long long s = 0;
    for (int i = 0; i < 8; ++i) s ^= x[i];
    out[blockIdx.x * 64 + threadIdx.x] = (float)s;
}
template <class K>
float run(K kern, float* out, int blocks) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    kern<<<blocks, 64>>>(out, 0xD2511F53u);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) kern<<<blocks, 64>>>(out, 0xD2511F53u);
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
    printf("v_mul_lo_u32   %.3f ns\n", run(k_lo, out, blocks) * 1e6 / instr);
    printf("v_mul_hi_u32   %.3f ns\n", run(k_hi, out, blocks) * 1e6 / instr);
    printf("v_mad_u64_u32  %.3f ns\n", run(k_mad, out, blocks) * 1e6 / instr);
    return 0;
}
