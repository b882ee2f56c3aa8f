// Microbenchmark (development aid): issue cost of f32 VALU forms on gfx950 -- v_fma_f32 vs
// v_pk_fma_f32 vs v_bitop3_b32 vs v_med3_f32 vs DPP mov -- with 8 independent chains per wave and
// enough waves to fill every SIMD.  Prints ns per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 4096;

__global__ __launch_bounds__(256) void k_fma(float* out, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "s"(b));
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_pkfma(float* out, float a, float b) {
    f2 x[4];
    for (int i = 0; i < 4; ++i) x[i] = f2{threadIdx.x * 0.001f + i, threadIdx.x * 0.002f - i};
    const f2 av = {a, a * 0.5f}, bv = {b, b * 2.f};
    for (int it = 0; it < ITER * 2; ++it)
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(av), "v"(bv));
    float s = 0;
    for (int i = 0; i < 4; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_bitop3(float* out, float a, float b) {
    unsigned x[8];
    const unsigned m = __float_as_uint(a), c = __float_as_uint(b);
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 77u + i;
    for (int it = 0; it < ITER; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_bitop3_b32(x[i], m, c, 0x6c);
    unsigned s = 0;
    for (int i = 0; i < 8; ++i) s ^= x[i];
    out[blockIdx.x * 256 + threadIdx.x] = (float)s;
}
__global__ __launch_bounds__(256) void k_med3(float* out, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_fmed3f(-__builtin_fabsf(x[i]), a, __builtin_fabsf(x[i]));
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_dpp(float* out, float a, float b) {
    int x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 3 + i;
    for (int it = 0; it < ITER; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_mov_dpp(x[i], 0x141, 0xF, 0xF, true) + 1;
    int s = 0;
    for (int i = 0; i < 8; ++i) s ^= x[i];
    out[blockIdx.x * 256 + threadIdx.x] = (float)s + a + b;
}

template <class K>
float run(K kern, float* out, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<<<blocks, 256>>>(out, 1.0001f, 0.5f);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) kern<<<blocks, 256>>>(out, 1.0001f, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    float* out;
    const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD
    hipMalloc(&out, blocks * 256 * sizeof(float));
    const double waves_per_simd = blocks * 4.0 / 1024.0, instr = ITER * 8.0;
    struct { const char* name; float ms; double per_wave_instr; } r[] = {
        {"v_fma_f32", run(k_fma, out, blocks), instr},
        {"v_pk_fma_f32 (2 fma each)", run(k_pkfma, out, blocks), instr},
        {"v_bitop3_b32", run(k_bitop3, out, blocks), instr},
        {"v_med3_f32 (abs/neg mods)", run(k_med3, out, blocks), instr},
        {"v_mov_b32_dpp + v_add", run(k_dpp, out, blocks), instr * 2},
    };
    for (auto& x : r)
        printf("%-28s %.3f ms  %.3f ns per wave-instruction per SIMD\n", x.name, x.ms,
               x.ms * 1e6 / (waves_per_simd * x.per_wave_instr));
    return 0;
}
