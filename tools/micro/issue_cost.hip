// Microbenchmark (development aid): SIMD issue cost of single VALU forms on gfx950, 8 independent
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
#define R4(I) I(0) I(1) I(2) I(3)
K1(k_add, "v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %4\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4")
K1(k_bitop3, "v_bitop3_b32 %0, %0, %4, %4 bitop3:0x6c\n v_bitop3_b32 %1, %1, %4, %4 bitop3:0x6c\n v_bitop3_b32 %2, %2, %4, %4 bitop3:0x6c\n v_bitop3_b32 %3, %3, %4, %4 bitop3:0x6c")
K1(k_shl, "v_lshlrev_b32 %0, 3, %0\n v_lshlrev_b32 %1, 3, %1\n v_lshlrev_b32 %2, 3, %2\n v_lshlrev_b32 %3, 3, %3")
K1(k_alignbit, "v_alignbit_b32 %0, %0, %4, 31\n v_alignbit_b32 %1, %1, %4, 31\n v_alignbit_b32 %2, %2, %4, 31\n v_alignbit_b32 %3, %3, %4, 31")
K1(k_dpp_qp, "v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_f32_dpp %1, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_f32_dpp %2, %2, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_f32_dpp %3, %3, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1")
K1(k_dpp_rm, "v_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_f32_dpp %1, %1, %1 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_f32_dpp %2, %2, %2 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_f32_dpp %3, %3, %3 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1")
K1(k_movdpp, "v_mov_b32_dpp %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_mov_b32_dpp %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_mov_b32_dpp %2, %2 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_mov_b32_dpp %3, %3 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1")
K1(k_min3, "v_min3_f32 %0, |%0|, |%4|, %4\n v_min3_f32 %1, |%1|, |%4|, %4\n v_min3_f32 %2, |%2|, |%4|, %4\n v_min3_f32 %3, |%3|, |%4|, %4")
K1(k_addsat, "v_add_i32 %0, %0, -1 clamp\n v_add_i32 %1, %1, -1 clamp\n v_add_i32 %2, %2, -1 clamp\n v_add_i32 %3, %3, -1 clamp")
K1(k_cmp, "v_cmp_eq_f32 vcc, %0, %4\n v_cmp_eq_f32 vcc, %1, %4\n v_cmp_eq_f32 vcc, %2, %4\n v_cmp_eq_f32 vcc, %3, %4")
K1(k_swz, "v_permlane16_swap_b32 %0, %1\n v_permlane16_swap_b32 %2, %3\n v_permlane16_swap_b32 %0, %1\n v_permlane16_swap_b32 %2, %3")

__global__ __launch_bounds__(64) void k_shl64(float* out, float a) {
    unsigned long long x[4];
    for (int i = 0; i < 4; ++i) x[i] = threadIdx.x * 0x10001ull + i;
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_lshlrev_b64 %0, 1, %0\n v_lshlrev_b64 %1, 1, %1\n v_lshlrev_b64 %2, 1, %2\n v_lshlrev_b64 %3, 1, %3" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]));
        asm volatile("v_lshlrev_b64 %0, 1, %0\n v_lshlrev_b64 %1, 1, %1\n v_lshlrev_b64 %2, 1, %2\n v_lshlrev_b64 %3, 1, %3" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]));
    }
    out[blockIdx.x * 64 + threadIdx.x] = (float)(x[0] ^ x[1] ^ x[2] ^ x[3]) + a;
}
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(64) void k_pkadd(float* out, float a) {
    f2 x[4];
    for (int i = 0; i < 4; ++i) x[i] = f2{threadIdx.x * 0.001f + i, i * 0.5f};
    const f2 av = {a, a};
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av));
        asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(av));
    }
    out[blockIdx.x * 64 + threadIdx.x] = x[0].x + x[1].y + x[2].x + x[3].y;
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
    struct { const char* n; void (*k)(float*, float); } ks[] = {
        {"v_add_f32", k_add}, {"v_bitop3_b32", k_bitop3}, {"v_lshlrev_b32", k_shl}, {"v_alignbit_b32", k_alignbit},
        {"v_add_f32_dpp quad_perm", k_dpp_qp}, {"v_add_f32_dpp row_mirror", k_dpp_rm}, {"v_mov_b32_dpp row_half_mirror", k_movdpp},
        {"v_min3_f32 abs", k_min3}, {"v_add_i32 clamp", k_addsat}, {"v_cmp_eq_f32 (vcc)", k_cmp}, {"v_permlane16_swap_b32", k_swz},
        {"v_lshlrev_b64", k_shl64}, {"v_pk_add_f32", k_pkadd}};
    for (auto& k : ks) printf("%-32s %.3f ns per wave-instruction per SIMD\n", k.n, run(k.k, out, blocks) * 1e6 / instr);
    return 0;
}
