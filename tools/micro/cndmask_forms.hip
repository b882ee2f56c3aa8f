// Issue cost of the select forms on gfx950 (development aid).  valu_cycles.hip measures
// v_cndmask_b32_e32 (mask = VCC, implicit) at ~5x the VOP3 form with an SGPR-pair mask; the
// exact-f SC kernel issues ~1800 of the VOP2 form per wave.  Variants, 8 independent registers per
// wave, 8 waves per SIMD:
//   e32_vcc      v_cndmask_b32_e32 with VCC never written in the kernel
//   e32_vcc_set  the same after VCC is set by a v_cmp before the loop
//   e64_vcc      VOP3 form naming vcc as the mask
//   e64_sgpr     VOP3 form, mask in s[4:5] written by s_mov
//   e64_sgpr_v   VOP3 form, mask in an SGPR pair written by a v_cmp before the loop
//   cmp_sel      per select a v_cmp_gt_f32 writing VCC then the VOP2 select reading it
//   cmp_sel64    the same with the compare writing an SGPR pair and the VOP3 select
//   mix_e32      one VOP2 select per three v_add_f32
//   mix_e64      one VOP3 select per three v_add_f32
//   cmp_sel2     a v_cmp writing VCC, then two VOP2 selects reading it back to back (a min/max swap)
//   pair_mix     two VOP2 selects back to back between two v_add_f32, VCC not written
//   hipcc --offload-arch=gfx950 -O3 -o cndmask_forms tools/micro/cndmask_forms.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 4096;

#define LOOP(PRE, BODY_A, BODY_B, CLOB)                                                                       \
    float x[8];                                                                                              \
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;                                             \
    PRE;                                                                                                     \
    for (int it = 0; it < ITER; ++it) {                                                                      \
        asm volatile(BODY_A : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a) CLOB);                \
        asm volatile(BODY_B : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a) CLOB);                \
    }                                                                                                        \
    float s = 0;                                                                                             \
    for (int i = 0; i < 8; ++i) s += x[i];                                                                   \
    out[blockIdx.x * 64 + threadIdx.x] = s;

#define S4(F) F(0) "\n " F(1) "\n " F(2) "\n " F(3)
#define E32(r) "v_cndmask_b32_e32 %" #r ", %" #r ", %4, vcc"
#define E64V(r) "v_cndmask_b32_e64 %" #r ", %" #r ", %4, vcc"
#define CMPSEL(r) "v_cmp_gt_f32_e32 vcc, %" #r ", %4\n v_cndmask_b32_e32 %" #r ", %" #r ", %4, vcc"
#define CLOBV : "vcc"

__global__ __launch_bounds__(64) void k_e32_vcc(float* out, float a) { LOOP((void)0, S4(E32), S4(E32), CLOBV) }
__global__ __launch_bounds__(64) void k_e32_vcc_set(float* out, float a) {
    LOOP(asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1" ::"v"(x[0]), "v"(a) : "vcc"), S4(E32), S4(E32), CLOBV)
}
__global__ __launch_bounds__(64) void k_e64_vcc(float* out, float a) { LOOP((void)0, S4(E64V), S4(E64V), CLOBV) }
__global__ __launch_bounds__(64) void k_cmp_sel(float* out, float a) { LOOP((void)0, S4(CMPSEL), S4(CMPSEL), CLOBV) }

#define SG(NAME, PRE)                                                                                        \
    __global__ __launch_bounds__(64) void NAME(float* out, float a) {                                        \
        float x[8];                                                                                          \
        for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;                                         \
        unsigned long long m;                                                                                \
        PRE;                                                                                                 \
        for (int it = 0; it < ITER; ++it) {                                                                  \
            asm volatile("v_cndmask_b32_e64 %0, %0, %4, %5\n v_cndmask_b32_e64 %1, %1, %4, %5\n"             \
                         " v_cndmask_b32_e64 %2, %2, %4, %5\n v_cndmask_b32_e64 %3, %3, %4, %5"              \
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a), "s"(m));                 \
            asm volatile("v_cndmask_b32_e64 %0, %0, %4, %5\n v_cndmask_b32_e64 %1, %1, %4, %5\n"             \
                         " v_cndmask_b32_e64 %2, %2, %4, %5\n v_cndmask_b32_e64 %3, %3, %4, %5"              \
                         : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a), "s"(m));                 \
        }                                                                                                    \
        float s = 0;                                                                                         \
        for (int i = 0; i < 8; ++i) s += x[i];                                                               \
        out[blockIdx.x * 64 + threadIdx.x] = s;                                                              \
    }
SG(k_e64_sgpr, m = 0x5555555555555555ull)
SG(k_e64_sgpr_v, asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x[0]), "v"(a)))

__global__ __launch_bounds__(64) void k_cmp_sel64(float* out, float a) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int h = 0; h < 8; h += 4) {
            unsigned long long m0, m1, m2, m3;
            asm volatile("v_cmp_gt_f32_e64 %4, %0, %8\n v_cmp_gt_f32_e64 %5, %1, %8\n"
                         " v_cmp_gt_f32_e64 %6, %2, %8\n v_cmp_gt_f32_e64 %7, %3, %8\n"
                         " v_cndmask_b32_e64 %0, %0, %8, %4\n v_cndmask_b32_e64 %1, %1, %8, %5\n"
                         " v_cndmask_b32_e64 %2, %2, %8, %6\n v_cndmask_b32_e64 %3, %3, %8, %7"
                         : "+v"(x[h]), "+v"(x[h + 1]), "+v"(x[h + 2]), "+v"(x[h + 3]), "=&s"(m0), "=&s"(m1),
                           "=&s"(m2), "=&s"(m3)
                         : "v"(a));
        }
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

#define MIXA(SEL) SEL(0) "\n v_add_f32 %1, %1, %4\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4"
#define MIXB(SEL) "v_add_f32 %0, %0, %4\n " SEL(1) "\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4"
#define E64S(r) "v_cndmask_b32_e64 %" #r ", %" #r ", %4, %5"
__global__ __launch_bounds__(64) void k_mix_e32(float* out, float a) { LOOP((void)0, MIXA(E32), MIXB(E32), CLOBV) }
__global__ __launch_bounds__(64) void k_mix_e64(float* out, float a) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    const unsigned long long m = 0x5555555555555555ull;
    for (int it = 0; it < ITER; ++it) {
        asm volatile(MIXA(E64S) : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a), "s"(m));
        asm volatile(MIXB(E64S) : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a), "s"(m));
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

#define CMPSEL2A "v_cmp_gt_f32_e32 vcc, %0, %1\n v_cndmask_b32_e32 %0, %0, %4, vcc\n v_cndmask_b32_e32 %1, %1, %4, vcc\n" \
                 " v_cmp_gt_f32_e32 vcc, %2, %3\n v_cndmask_b32_e32 %2, %2, %4, vcc\n v_cndmask_b32_e32 %3, %3, %4, vcc"
#define PAIRMIX "v_add_f32 %0, %0, %4\n v_cndmask_b32_e32 %1, %1, %4, vcc\n v_cndmask_b32_e32 %2, %2, %4, vcc\n" \
                " v_add_f32 %3, %3, %4"
__global__ __launch_bounds__(64) void k_cmp_sel2(float* out, float a) { LOOP((void)0, CMPSEL2A, CMPSEL2A, CLOBV) }
__global__ __launch_bounds__(64) void k_pair_mix(float* out, float a) { LOOP((void)0, PAIRMIX, PAIRMIX, CLOBV) }

typedef void (*Kern)(float*, float);

int main() {
    const struct {
        const char* name;
        Kern k;
        int per_iter;  // instructions per wave per loop iteration
    } ks[] = {{"e32_vcc", k_e32_vcc, 8},     {"e32_vcc_set", k_e32_vcc_set, 8}, {"e64_vcc", k_e64_vcc, 8},
              {"e64_sgpr", k_e64_sgpr, 8},   {"e64_sgpr_v", k_e64_sgpr_v, 8},   {"cmp_sel", k_cmp_sel, 16},
              {"cmp_sel64", k_cmp_sel64, 16}, {"mix_e32", k_mix_e32, 8},        {"mix_e64", k_mix_e64, 8},
              {"cmp_sel2", k_cmp_sel2, 12},  {"pair_mix", k_pair_mix, 8}};
    const int blocks = 256 * 4 * 8;  // 8 waves per SIMD
    float* out;
    if (hipMalloc(&out, (size_t)blocks * 64 * sizeof(float)) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 60; ++w)
        for (const auto& k : ks) hipLaunchKernelGGL(k.k, dim3(blocks), dim3(64), 0, 0, out, 1.0001f);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    for (const auto& k : ks) {
        float ms = 1e30f;
        for (int r = 0; r < 5; ++r) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(64), 0, 0, out, 1.0001f);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float t = 0;
            (void)hipEventElapsedTime(&t, e0, e1);
            ms = t < ms ? t : ms;
        }
        const double instr_per_simd = (double)blocks / 1024.0 * ITER * k.per_iter;
        printf("%-12s %.3f ns per wave-instruction per SIMD (%.4f ms)\n", k.name, ms * 1e6 / instr_per_simd, ms);
    }
    (void)hipFree(out);
    return 0;
}
