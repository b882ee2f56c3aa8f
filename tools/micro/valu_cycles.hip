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

// round 5: the forms of the SC bench kernel's instruction stream that the
// SQ class counters leave unclassified, each calibrated the same way
#define KA(NAME, FORM)                                                                    \
    KF(NAME, float, threadIdx.x * 0.001f + i,                                             \
       FORM(0) "\n " FORM(1) "\n " FORM(2) "\n " FORM(3))
#define F_MIN3(r) "v_min3_f32 %" #r ", |%" #r "|, |%4|, %4"
#define F_MED3(r) "v_med3_f32 %" #r ", -|%" #r "|, %4, |%" #r "|"
#define F_ALIGN(r) "v_alignbit_b32 %" #r ", %" #r ", %4, 7"
#define F_LSHL(r) "v_lshlrev_b32 %" #r ", 3, %" #r
#define F_LSHR(r) "v_lshrrev_b32 %" #r ", 3, %" #r
#define F_BFE(r) "v_bfe_u32 %" #r ", %" #r ", 3, 1"
#define F_AND(r) "v_and_b32 %" #r ", %" #r ", %4"
#define F_MOV(r) "v_mov_b32 %" #r ", %4"
#define F_CVTUB(r) "v_cvt_f32_ubyte0 %" #r ", %" #r
#define F_BCNT(r) "v_bcnt_u32_b32 %" #r ", %" #r ", 0"
#define F_XORDPP(r) "v_xor_b32_dpp %" #r ", %" #r ", %" #r " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1"
#define F_ANDDPP(r) "v_and_b32_dpp %" #r ", %" #r ", %" #r " quad_perm:[3,2,1,0] row_mask:0xf bank_mask:0xf bound_ctrl:1"
#define F_MINUDPP(r) "v_min_u32_dpp %" #r ", %" #r ", %" #r " row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1"
#define F_ADDUDPP(r) "v_add_u32_dpp %" #r ", %" #r ", %" #r " row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1"
#define F_CNDM(r) "v_cndmask_b32 %" #r ", %" #r ", %4, vcc"
#define F_CMPEQ(r) "v_cmp_eq_f32 vcc, 0, %" #r
KA(k_min3, F_MIN3)
KA(k_med3, F_MED3)
KA(k_alignbit, F_ALIGN)
KA(k_lshl, F_LSHL)
KA(k_lshr, F_LSHR)
KA(k_bfe, F_BFE)
KA(k_and, F_AND)
KA(k_mov, F_MOV)
KA(k_cvtub, F_CVTUB)
KA(k_bcnt, F_BCNT)
KA(k_xordpp, F_XORDPP)
KA(k_anddpp, F_ANDDPP)
KA(k_minudpp, F_MINUDPP)
KA(k_addudpp, F_ADDUDPP)
// the two forms that read or write VCC, with VCC declared clobbered
#define KV(NAME, FORM)                                                                                   \
    __global__ __launch_bounds__(64) void NAME(float* out, float a) {                                    \
        float x[8];                                                                                      \
        for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;                                     \
        for (int it = 0; it < ITER; ++it) {                                                              \
            asm volatile(FORM(0) "\n " FORM(1) "\n " FORM(2) "\n " FORM(3)                              \
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a) : "vcc");             \
            asm volatile(FORM(0) "\n " FORM(1) "\n " FORM(2) "\n " FORM(3)                              \
                         : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a) : "vcc");             \
        }                                                                                                \
        float s = 0;                                                                                     \
        for (int i = 0; i < 8; ++i) s += x[i];                                                           \
        out[blockIdx.x * 64 + threadIdx.x] = s;                                                          \
    }
KV(k_cndmask, F_CNDM)
// v_cndmask_b32_e64 with an SGPR-pair mask (the form the kernels' selects mostly take)
__global__ __launch_bounds__(64) void k_cndmask64(float* out, float a) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    const unsigned long long msk = 0x5555555555555555ull;  // a constant: materialised in an SGPR pair
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_cndmask_b32_e64 %0, %0, %4, %5\n v_cndmask_b32_e64 %1, %1, %4, %5\n"
                     " v_cndmask_b32_e64 %2, %2, %4, %5\n v_cndmask_b32_e64 %3, %3, %4, %5"
                     : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "v"(a), "s"(msk));
        asm volatile("v_cndmask_b32_e64 %0, %0, %4, %5\n v_cndmask_b32_e64 %1, %1, %4, %5\n"
                     " v_cndmask_b32_e64 %2, %2, %4, %5\n v_cndmask_b32_e64 %3, %3, %4, %5"
                     : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(a), "s"(msk));
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}
KV(k_cmpeq, F_CMPEQ)
// v_pk_add_f32 on 64-bit register pairs (two results per instruction)
__global__ __launch_bounds__(64) void k_pkadd(float* out, float a) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 x[8];
    for (int i = 0; i < 8; ++i) x[i] = f2{threadIdx.x * 0.001f + i, a};
    for (int it = 0; it < ITER; ++it) {
        asm volatile("v_pk_add_f32 %0, %0, %0\n v_pk_add_f32 %1, %1, %1\n v_pk_add_f32 %2, %2, %2\n v_pk_add_f32 %3, %3, %3"
                     : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]));
        asm volatile("v_pk_add_f32 %0, %0, %0\n v_pk_add_f32 %1, %1, %1\n v_pk_add_f32 %2, %2, %2\n v_pk_add_f32 %3, %3, %3"
                     : "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

typedef void (*Kern)(float*, float);

int main() {
    const struct {
        const char* name;
        Kern k;
    } ks[] = {{"v_add_f32", k_add_f32}, {"v_fma_f32", k_fma_f32}, {"v_xor_b32", k_xor_b32},
              {"v_add_f32_dpp", k_dpp_add}, {"v_exp_f32", k_exp_f32}, {"v_add_f64", k_add_f64},
              {"v_fma_f64", k_fma_f64}, {"v_mul_f64", k_mul_f64}, {"v_mul_f32", k_mul_f32},
              {"v_bitop3_b32", k_bitop3}, {"v_add_u32", k_add_u32}, {"v_min_f32", k_min_f32},
              {"v_cvt_f32_f64+f64_f32", k_cvt_f64}, {"v_mov_b32_dpp", k_movdpp},
              {"v_min3_f32", k_min3}, {"v_med3_f32", k_med3}, {"v_pk_add_f32", k_pkadd},
              {"v_alignbit_b32", k_alignbit}, {"v_lshlrev_b32", k_lshl}, {"v_lshrrev_b32", k_lshr},
              {"v_bfe_u32", k_bfe}, {"v_and_b32", k_and}, {"v_mov_b32", k_mov}, {"v_cvt_f32_ubyte0", k_cvtub},
              {"v_bcnt_u32_b32", k_bcnt}, {"v_xor_b32_dpp", k_xordpp}, {"v_and_b32_dpp", k_anddpp},
              {"v_min_u32_dpp", k_minudpp}, {"v_add_u32_dpp", k_addudpp}, {"v_cndmask_b32_vcc", k_cndmask},
              {"v_cndmask_b32", k_cndmask64},
              {"v_cmp_eq_f32", k_cmpeq}};
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
