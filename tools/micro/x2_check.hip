// Checks of the X2 (two rows per codeword) building blocks of scl_tree_kernel.hip on the GPU:
// v_permlane16_swap(v, v) as xch_rows uses it (first result = the even row's value in both rows,
// second = the odd row's), and the split-row rank against a brute-force stable (metric, index)
// rank on rows holding the same 16 candidates (random metrics with forced ties).
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/x2_check tools/micro/x2_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define PL_RANK_ROT_X2(r, m)                                                                \
    "s_mov_b32 vcc_lo, " #m "\n\t"                                                          \
    "s_mov_b32 vcc_hi, " #m "\n\t"                                                          \
    "v_subb_co_u32_dpp %1, vcc, %4, %2, vcc row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t" \
    "v_subb_co_u32_dpp %1, vcc, %5, %3, vcc row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t" \
    "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n\t"
__device__ __forceinline__ int rank16_x2(double cv) {
    const long long b = __double_as_longlong(cv);
    const int lo = (int)(b & 0xffffffffLL), hi = (int)(b >> 32);
    const int slo = __builtin_amdgcn_update_dpp(lo, lo, 0x128, 0xA, 0xF, false);
    const int shi = __builtin_amdgcn_update_dpp(hi, hi, 0x128, 0xA, 0xF, false);
    int rk, tmp;
    asm volatile(
        "s_nop 1\n\t"
        "v_mov_b32 %0, 0\n\t"
        PL_RANK_ROT_X2(1, 0xfe00fffe) PL_RANK_ROT_X2(2, 0xfc00fffc) PL_RANK_ROT_X2(3, 0xf800fff8)
        PL_RANK_ROT_X2(4, 0xf000fff0) PL_RANK_ROT_X2(5, 0xe000ffe0) PL_RANK_ROT_X2(6, 0xc000ffc0)
        PL_RANK_ROT_X2(7, 0x8000ff80) PL_RANK_ROT_X2(8, 0x0000ff00)
        : "=&v"(rk), "=&v"(tmp)
        : "v"(lo), "v"(hi), "v"(slo), "v"(shi)
        : "vcc");
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)rk, (unsigned)rk, false, false);
    return (int)(r[0] + r[1]);
}

__global__ void k(const double* metric, int* rank_out, unsigned* sw0, unsigned* sw1, int* part) {
    const int lane = threadIdx.x;
    const int c = lane >> 5, gl = lane & 15;
    const double cv = metric[c * 16 + gl];  // both rows of a codeword hold the same 16 candidates
    rank_out[lane] = rank16_x2(cv);
    const unsigned v = 1000u + lane;
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    sw0[lane] = r[0];
    sw1[lane] = r[1];
}

int main() {
    const int trials = 2000;
    double h[32];
    int rk[64];
    unsigned s0[64], s1[64];
    double* dm;
    int* dr;
    unsigned *d0, *d1;
    (void)hipMalloc(&dm, sizeof(h));
    (void)hipMalloc(&dr, sizeof(rk));
    (void)hipMalloc(&d0, sizeof(s0));
    (void)hipMalloc(&d1, sizeof(s1));
    srand(7);
    int bad = 0, badsw = 0;
    for (int t = 0; t < trials; ++t) {
        for (int i = 0; i < 32; ++i) h[i] = (double)(rand() % (t % 3 == 0 ? 4 : 1000)) * 0.5 + (t % 5 == 0 ? 30.0 : 0.0);
        (void)hipMemcpy(dm, h, sizeof(h), hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dm, dr, d0, d1, nullptr);
        if (hipDeviceSynchronize() != hipSuccess) { printf("HIP error\n"); return 1; }
        (void)hipMemcpy(rk, dr, sizeof(rk), hipMemcpyDeviceToHost);
        (void)hipMemcpy(s0, d0, sizeof(s0), hipMemcpyDeviceToHost);
        (void)hipMemcpy(s1, d1, sizeof(s1), hipMemcpyDeviceToHost);
        for (int lane = 0; lane < 64; ++lane) {
            const int c = lane >> 5, gl = lane & 15;
            int want = 0;
            for (int o = 0; o < 16; ++o) {
                const double v = h[c * 16 + o], me = h[c * 16 + gl];
                want += (v < me || (v == me && o < gl)) ? 1 : 0;
            }
            if (rk[lane] != want) ++bad;
            const unsigned even = 1000u + (lane & ~16), odd = 1000u + (lane | 16);
            if (s0[lane] != even || s1[lane] != odd) ++badsw;
        }
    }
    printf("rank16_x2: %d of %d lane ranks differ from the brute-force stable rank\n", bad, trials * 64);
    printf("permlane16_swap(v, v): %d of %d lanes not (even row's, odd row's) value\n", badsw, trials * 64);
    if (badsw) {
        for (int lane = 0; lane < 64; lane += 8) printf("lane %2d: r0 %u r1 %u\n", lane, s0[lane], s1[lane]);
    }
    return bad || badsw;
}
