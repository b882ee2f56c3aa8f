// Microbenchmark (development aid): does an s_nop (the DPP read-after-VALU-write hazard fill) cost
// SIMD issue slots that other waves could have used?  Each wave runs CH independent chains of
// v_add_f32 (no hazard) or of s_nop 1 + v_add_f32_dpp (the lane-level pattern of sc_static.h),
// at 1..8 waves per SIMD (64-thread blocks, 256 CUs x 4 SIMDs).  Prints ns per VALU instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int ITER = 4096;

template <int CH>
__global__ __launch_bounds__(64) void k_add(float* out, float a) {
    float x[CH];
    for (int i = 0; i < CH; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it)
#pragma unroll
        for (int i = 0; i < CH; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
    float s = 0;
    for (int i = 0; i < CH; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}
template <int CH>
__global__ __launch_bounds__(64) void k_dpp(float* out, float a) {
    float x[CH];
    for (int i = 0; i < CH; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it)
#pragma unroll
        for (int i = 0; i < CH; ++i)
            asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1"
                         : "+v"(x[i]));
    float s = 0;
    for (int i = 0; i < CH; ++i) s += x[i] + a;
    out[blockIdx.x * 64 + threadIdx.x] = s;
}
template <int CH>
__global__ __launch_bounds__(64) void k_dpp_nonop(float* out, float a) {  // 2 chains interleaved: no nop needed
    float x[CH], y[CH];
    for (int i = 0; i < CH; ++i) x[i] = threadIdx.x * 0.001f + i, y[i] = x[i] * 0.5f;
    for (int it = 0; it < ITER / 2; ++it)
#pragma unroll
        for (int i = 0; i < CH; ++i)
            asm volatile("v_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                         "v_add_f32 %1, %1, %1\n\t"
                         "v_add_f32 %1, %1, %1\n\t"
                         "v_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                         : "+v"(x[i]), "+v"(y[i]));
    float s = 0;
    for (int i = 0; i < CH; ++i) s += x[i] + y[i] + a;
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <class K>
float run(K kern, float* out, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<<<blocks, 64>>>(out, 1.0001f);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) kern<<<blocks, 64>>>(out, 1.0001f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    float* out;
    hipMalloc(&out, 1024 * 8 * 64 * sizeof(float));
    for (int w = 1; w <= 8; w *= 2) {
        if (w == 8) w = 8;
        const int blocks = 1024 * w;
        const double instr = ITER * 1.0 * w;  // per chain per SIMD
        auto ns = [&](float ms, int ch) { return ms * 1e6 / (instr * ch); };
        printf("waves/SIMD %d: add x1 %.3f  add x2 %.3f  nop+dpp x1 %.3f  nop+dpp x2 %.3f  dpp+2add(no nop) x1 %.3f ns/VALU\n", w,
               ns(run(k_add<1>, out, blocks), 1), ns(run(k_add<2>, out, blocks), 2), ns(run(k_dpp<1>, out, blocks), 1),
               ns(run(k_dpp<2>, out, blocks), 2), ns(run(k_dpp_nonop<1>, out, blocks), 2));
    }
    for (int w = 3; w <= 6; w += 3) {
        const int blocks = 1024 * w;
        const double instr = ITER * 1.0 * w;
        auto ns = [&](float ms, int ch) { return ms * 1e6 / (instr * ch); };
        printf("waves/SIMD %d: add x1 %.3f  add x2 %.3f  nop+dpp x1 %.3f  nop+dpp x2 %.3f  dpp+2add(no nop) x1 %.3f ns/VALU\n", w,
               ns(run(k_add<1>, out, blocks), 1), ns(run(k_add<2>, out, blocks), 2), ns(run(k_dpp<1>, out, blocks), 1),
               ns(run(k_dpp<2>, out, blocks), 2), ns(run(k_dpp_nonop<1>, out, blocks), 2));
    }
    return 0;
}
