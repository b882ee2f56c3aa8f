// rcp_check.hip -- accuracy of v_rcp_f64 on gfx950 over the denominators the SCL kernels divide by
// (softplus.h: the penalty's log, den = 2 + f in [1.41, 2.83]; f_exact_pm_n: den in [2, 4]), and
// whether one Newton step before the quotient's residual correction gives the same quotient as
// the two steps the kernels take.  One wave per block, deterministic xorshift arguments; writes
// per block: max relative error of the raw reciprocal (as a double) and the count of quotients
// s = f / den that differ between the one-step and the two-step forms.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/rcp_check.hip -o /tmp/rcp_check && /tmp/rcp_check
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ __launch_bounds__(64) void rcp_kernel(double lo, double span, int iters, double* maxerr, unsigned* ndiff) {
    uint64_t x = 0x9E3779B97F4A7C15ull * (blockIdx.x * 64u + threadIdx.x + 1u);
    double worst = 0.0;
    unsigned diff = 0;
    for (int it = 0; it < iters; ++it) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        const double u = (double)(x >> 11) * (1.0 / 9007199254740992.0);
        const double den = lo + span * u;
        const double f = den - 2.0;  // the kernels' numerator pairing (penalty: f = m - 1, den = 2 + f)
        const double rc0 = __builtin_amdgcn_rcp(den);
        const double e0 = __builtin_fma(-den, rc0, 1.0);  // = 1 - den rc0, exact to ~2^-106
        worst = fmax(worst, fabs(e0));
        double r1 = __builtin_fma(rc0, e0, rc0);
        const double q1 = f * r1;
        const double s1 = __builtin_fma(r1, __builtin_fma(-den, q1, f), q1);
        const double e1 = __builtin_fma(-den, r1, 1.0);
        const double r2 = __builtin_fma(r1, e1, r1);
        const double q2 = f * r2;
        const double s2 = __builtin_fma(r2, __builtin_fma(-den, q2, f), q2);
        diff += (s1 != s2) ? 1u : 0u;
    }
    // block reduction through LDS (one wave), vector stores only
    __shared__ double wm[64];
    __shared__ unsigned dc[64];
    wm[threadIdx.x] = worst;
    dc[threadIdx.x] = diff;
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = 0.0;
        unsigned d = 0;
        for (int i = 0; i < 64; ++i) {
            m = fmax(m, wm[i]);
            d += dc[i];
        }
        maxerr[blockIdx.x] = m;
        ndiff[blockIdx.x] = d;
    }
}

int main() {
    const int blocks = 4096, iters = 4096;
    double* dm;
    unsigned* dd;
    if (hipMalloc(&dm, blocks * sizeof(double)) != hipSuccess || hipMalloc(&dd, blocks * sizeof(unsigned)) != hipSuccess) {
        printf("hipMalloc failed\n");
        return 1;
    }
    const double ranges[2][2] = {{1.41, 1.42}, {2.0, 2.0}};  // [lo, span]: the penalty's den, f_exact_pm's den
    const char* names[2] = {"penalty den in [1.41, 2.83]", "f_exact den in [2, 4]"};
    for (int r = 0; r < 2; ++r) {
        hipLaunchKernelGGL(rcp_kernel, dim3(blocks), dim3(64), 0, 0, ranges[r][0], ranges[r][1], iters, dm, dd);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("kernel failed\n");
            return 1;
        }
        static double hm[4096];
        static unsigned hd[4096];
        hipMemcpy(hm, dm, sizeof(hm), hipMemcpyDeviceToHost);
        hipMemcpy(hd, dd, sizeof(hd), hipMemcpyDeviceToHost);
        double m = 0.0;
        unsigned long long d = 0;
        for (int i = 0; i < blocks; ++i) {
            m = hm[i] > m ? hm[i] : m;
            d += hd[i];
        }
        printf("%s: %llu denominators, max |1 - den rcp(den)| = %.3e (2^%.1f), one-step vs two-step quotients differing: %llu\n",
               names[r], (unsigned long long)blocks * 64ull * iters, m, log2(m), d);
    }
    return 0;
}
