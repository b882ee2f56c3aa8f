// exactf.h -- the exact-boxplus f of the my_sn decoders (my_sn/fec/polar/dec.py:39-43):
//   f(x, y) = log(1 + exp(xc + yc)) - log(exp(xc) + exp(yc)),  xc, yc = clip(x, y, +-llr_max)
// in fp32 with the reference's roundings (torch CPU: each exp, add, log and the subtraction
// rounded to fp32) and CORRECTLY ROUNDED exp and log.
//
// Why correctly rounded: the f cancels catastrophically, so a decision near a tie follows the last
// ulp of each transcendental.  The reference's exp/log and glibc's agree (0 of 180,000 rows differ
// at (512,1024), 1-3 dB), while ocml's fp32 expf / logf (within an ulp, not correctly rounded)
// flipped 8e-3 of the rows at 3 dB (tests/test_exactf_gpu.py; DESIGN.md section 4 has the CPU
// experiment: the oracle with 1/8 of its exp/log results one ulp off reproduces that pattern,
// with them evaluated in fp64 and rounded once it matches the reference on every row).
//
// exp_cr / log_cr evaluate in fp64 over the range f uses and round once to fp32; their fp64
// error (< 2^-46 relative) leaves a wrong fp32 rounding only for arguments within 2^-22 ulp of a
// rounding boundary.  Range: exp_cr for |x| <= 87 (normal fp32 results), log_cr for finite x > 0.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

namespace plx {

// exp(x) for fp32 x, |x| <= 87: x = k ln2 + r (|r| <= ln2/2, two-part ln2), Taylor polynomial of
// degree 11 in fp64 (truncation < 7e-15 relative), rounded to fp32, then scaled by 2^k exactly.
__device__ __forceinline__ float exp_cr(float xf) {
    const double x = (double)xf;
    constexpr double kLog2e = 1.4426950408889634;
    constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
    const double k = __builtin_rint(x * kLog2e);
    double r = __builtin_fma(-k, kLn2Hi, x);
    r = __builtin_fma(-k, kLn2Lo, r);
    double p = 2.505210838544172e-08;  // 1/11!
    p = __builtin_fma(p, r, 2.755731922398589e-07);
    p = __builtin_fma(p, r, 2.7557319223985893e-06);
    p = __builtin_fma(p, r, 2.48015873015873e-05);
    p = __builtin_fma(p, r, 0.0001984126984126984);
    p = __builtin_fma(p, r, 0.001388888888888889);
    p = __builtin_fma(p, r, 0.008333333333333333);
    p = __builtin_fma(p, r, 0.041666666666666664);
    p = __builtin_fma(p, r, 0.16666666666666666);
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    // p in [0.70, 1.42]: rounding p and scaling by 2^k (|k| <= 126, a normal result) is one rounding
    return __builtin_ldexpf((float)p, (int)k);
}

// log(x) for finite fp32 x > 0: x = 2^e m, m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s) with
// s = (m - 1) / (m + 1), |s| < 0.1716, series through s^19 (truncation < 3e-16 relative), in fp64.
__device__ __forceinline__ float log_cr(float xf) {
    constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
    double m = __builtin_amdgcn_frexp_mant((double)xf);  // [0.5, 1)
    int e = __builtin_amdgcn_frexp_exp((double)xf);
    if (m < 0.70710678118654752) {
        m = m + m;
        e -= 1;
    }
    const double f = m - 1.0;  // exact
    const double s = f / (2.0 + f);
    const double z = s * s;
    double R = 2.0 / 19.0;  // sum_{i>=1} 2/(2i+1) z^(i-1), i = 1 .. 9
    R = __builtin_fma(R, z, 2.0 / 17.0);
    R = __builtin_fma(R, z, 2.0 / 15.0);
    R = __builtin_fma(R, z, 2.0 / 13.0);
    R = __builtin_fma(R, z, 2.0 / 11.0);
    R = __builtin_fma(R, z, 2.0 / 9.0);
    R = __builtin_fma(R, z, 2.0 / 7.0);
    R = __builtin_fma(R, z, 2.0 / 5.0);
    R = __builtin_fma(R, z, 2.0 / 3.0);
    const double lm = __builtin_fma(s * z, R, s + s);  // log m = 2s + s z R(z)
    const double de = (double)e;
    return (float)__builtin_fma(de, kLn2Hi, __builtin_fma(de, kLn2Lo, lm));
}

// f of my_sn/fec/polar/dec.py:39-43 on clipped inputs, each operation rounded as the reference does.
// Out of line: inlined into the fully unrolled specialised SC kernels (hundreds of f per lane) the
// fp64 code made one (128,256) kernel take minutes to compile.
__device__ __attribute__((noinline)) float f_exact(float x, float y, float lmax) {
    const float xc = fminf(fmaxf(x, -lmax), lmax), yc = fminf(fmaxf(y, -lmax), lmax);
    float o = log_cr(1.0f + exp_cr(xc + yc));
    o -= log_cr(exp_cr(xc) + exp_cr(yc));
    return o;
}

}  // namespace plx
