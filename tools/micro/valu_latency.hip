// Microbenchmark (development aid): dependent-chain VALU latency on gfx950 at 1..4 waves per SIMD
// (one 64-thread block per SIMD slot, 256 CUs x 4 SIMDs).  Chains: v_add_f32, v_bitop3_b32, and
// DPP mirror + v_add (the lane-level pattern of sc_static.h).
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int ITER = 8192;

__global__ __launch_bounds__(64) void k_add(float* out, float a) {
    float x = threadIdx.x * 0.001f;
    for (int it = 0; it < ITER; ++it) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(a));
    out[blockIdx.x * 64 + threadIdx.x] = x;
}
__global__ __launch_bounds__(64) void k_bitop3(float* out, float a) {
    unsigned x = threadIdx.x, m = __float_as_uint(a);
    for (int it = 0; it < ITER; ++it) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x6c" : "+v"(x) : "v"(m));
    out[blockIdx.x * 64 + threadIdx.x] = (float)x;
}
__global__ __launch_bounds__(64) void k_dpp(float* out, float a) {
    float x = threadIdx.x * 0.001f;
    for (int it = 0; it < ITER; ++it) {
        float y = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x141, 0xF, 0xF, true));
        x = x + y * a;
    }
    out[blockIdx.x * 64 + threadIdx.x] = x;
}

template <class K>
float run(K kern, float* out, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<<<blocks, 64>>>(out, 1.0001f);
    hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) kern<<<blocks, 64>>>(out, 1.0001f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 3;
}

int main() {
    float* out;
    hipMalloc(&out, 1024 * 8 * 64 * sizeof(float));
    for (int w = 1; w <= 4; ++w) {
        const int blocks = 1024 * w;
        const float ta = run(k_add, out, blocks), tb = run(k_bitop3, out, blocks), td = run(k_dpp, out, blocks);
        printf("%d waves/SIMD: add chain %.2f ns/instr/wave  bitop3 chain %.2f  dpp+fma chain %.2f ns/iter/wave"
               "  | per SIMD: add %.2f ns/instr\n",
               w, ta * 1e6 / ITER, tb * 1e6 / ITER, td * 1e6 / ITER, ta * 1e6 / ITER / w);
    }
    return 0;
}
