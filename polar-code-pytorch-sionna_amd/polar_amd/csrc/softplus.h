// softplus.h -- the SCL path-metric penalty log(1 + exp(z)) in fp64 (x_run_sn_polar/polar/
// polar_scl.py:83 computes np.log(1 + np.exp(-(1-2u) * clip(llr))) in float64).
//
// Shared by scl_kernel.hip and scl_tree_kernel.hip so the two kernels produce identical metrics.
// Same three roundings as the reference -- e = exp(z), y = 1 + e, log(y) -- with exp and log
// evaluated for the range the decoder uses instead of through ocml's general routines:
//   exp: z = k ln2 + r (Cody-Waite, two-part ln2 with FMA), |r| <= ln2/2, Taylor polynomial of
//        degree 13 (truncation < 5e-18 relative), scaled by 2^k;
//   log: y = 2^e m, m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s), s = (m-1)/(m+1), |s| < 0.1716,
//        series through s^25 (truncation < 1e-18 relative).
// Both are within ~2 ulp of the correctly rounded result, like ocml's and numpy's.  Valid for
// |z| <= 700: pl_plan_create rejects list plans with llr_max > 700.
#pragma once
#include <hip/hip_runtime.h>

namespace pl {

// a * b + c as one VOP3 v_fma_f64.  Left to itself the compiler keeps the loop-invariant Horner
// coefficient c in a VGPR, copies it into the destination and uses the two-address v_fmac_f64:
// one extra v_mov_b64 per polynomial step (23 per penalty).  Same operation, same rounding.
// Same-process A/B, SCL (512,1024) L=8 bs=8192 (profiles/r02zg_scl_fma_ab.txt): plain fma()
// 1.160 ms, VGPR coefficients 1.104 ms, SGPR coefficients (s_mov pairs; 35 fewer VGPRs, more
// SGPR spills) 1.130 ms.  The compiler pads each inline-asm block with hazard s_nops (15 per
// penalty), so the default (3) issues each polynomial as one block: 1.081 vs 1.085 ms, my_sn
// exact-f fast-SCL 7.66 vs 7.73 ms (profiles/r02zj_scl_horner_ab*.txt).
#ifndef PL_SP_FMA
#define PL_SP_FMA 3  // 0: plain fma(), 1: VOP3 with a VGPR coefficient, 2: VOP3 with an SGPR coefficient,
                    // 3: each polynomial as one asm block
#endif
__device__ __forceinline__ double fma3(double a, double b, double c) {
#if PL_SP_FMA == 0
    return fma(a, b, c);
#else
    double d;
#if PL_SP_FMA == 1
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
#else
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
#endif
    return d;
#endif
}

__device__ __forceinline__ double pm_exp(double z) {
    constexpr double kLog2e = 1.4426950408889634;
    constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
    const double k = __builtin_rint(z * kLog2e);
    double r = fma(-k, kLn2Hi, z);
    r = fma(-k, kLn2Lo, r);
    // 1/i!, i = 13 .. 0
#if PL_SP_FMA == 3
    double p;  // the whole Horner chain in one block: no hazard padding between the steps
    asm("v_fma_f64 %0, %2, %1, %3\n\t"
        "v_fma_f64 %0, %0, %1, %4\n\t"
        "v_fma_f64 %0, %0, %1, %5\n\t"
        "v_fma_f64 %0, %0, %1, %6\n\t"
        "v_fma_f64 %0, %0, %1, %7\n\t"
        "v_fma_f64 %0, %0, %1, %8\n\t"
        "v_fma_f64 %0, %0, %1, %9\n\t"
        "v_fma_f64 %0, %0, %1, %10\n\t"
        "v_fma_f64 %0, %0, %1, %11\n\t"
        "v_fma_f64 %0, %0, %1, %12\n\t"
        "v_fma_f64 %0, %0, %1, 0.5\n\t"
        "v_fma_f64 %0, %0, %1, 1.0\n\t"
        "v_fma_f64 %0, %0, %1, 1.0"
        : "=&v"(p)
        : "v"(r), "v"(1.6059043836821613e-10), "v"(2.08767569878681e-09), "v"(2.505210838544172e-08),
          "v"(2.755731922398589e-07), "v"(2.7557319223985893e-06), "v"(2.48015873015873e-05),
          "v"(0.0001984126984126984), "v"(0.001388888888888889), "v"(0.008333333333333333),
          "v"(0.041666666666666664), "v"(0.16666666666666666));
#else
    double p = 1.6059043836821613e-10;
    p = fma3(p, r, 2.08767569878681e-09);
    p = fma3(p, r, 2.505210838544172e-08);
    p = fma3(p, r, 2.755731922398589e-07);
    p = fma3(p, r, 2.7557319223985893e-06);
    p = fma3(p, r, 2.48015873015873e-05);
    p = fma3(p, r, 0.0001984126984126984);
    p = fma3(p, r, 0.001388888888888889);
    p = fma3(p, r, 0.008333333333333333);
    p = fma3(p, r, 0.041666666666666664);
    p = fma3(p, r, 0.16666666666666666);
    p = fma3(p, r, 0.5);
    p = fma3(p, r, 1.0);
    p = fma3(p, r, 1.0);
#endif
    return ldexp(p, (int)k);
}

__device__ __forceinline__ double pm_log(double y) {  // y >= 1, finite
    constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
    double m = __builtin_amdgcn_frexp_mant(y);  // [0.5, 1)
    int e = __builtin_amdgcn_frexp_exp(y);
    if (m < 0.70710678118654752) {
        m = m + m;
        e -= 1;
    }
    const double f = m - 1.0;  // exact (Sterbenz)
    const double s = f / (2.0 + f);
    const double z = s * s;
    // R(z) = sum_{i>=1} 2/(2i+1) z^(i-1), i = 1 .. 12
#if PL_SP_FMA == 3
    double R;
    asm("v_fma_f64 %0, %2, %1, %3\n\t"
        "v_fma_f64 %0, %0, %1, %4\n\t"
        "v_fma_f64 %0, %0, %1, %5\n\t"
        "v_fma_f64 %0, %0, %1, %6\n\t"
        "v_fma_f64 %0, %0, %1, %7\n\t"
        "v_fma_f64 %0, %0, %1, %8\n\t"
        "v_fma_f64 %0, %0, %1, %9\n\t"
        "v_fma_f64 %0, %0, %1, %10\n\t"
        "v_fma_f64 %0, %0, %1, %11\n\t"
        "v_fma_f64 %0, %0, %1, %12\n\t"
        "v_fma_f64 %0, %0, %1, %13"
        : "=&v"(R)
        : "v"(z), "v"(2.0 / 25.0), "v"(2.0 / 23.0), "v"(2.0 / 21.0), "v"(2.0 / 19.0), "v"(2.0 / 17.0),
          "v"(2.0 / 15.0), "v"(2.0 / 13.0), "v"(2.0 / 11.0), "v"(2.0 / 9.0), "v"(2.0 / 7.0), "v"(2.0 / 5.0),
          "v"(2.0 / 3.0));
#else
    double R = 2.0 / 25.0;
    R = fma3(R, z, 2.0 / 23.0);
    R = fma3(R, z, 2.0 / 21.0);
    R = fma3(R, z, 2.0 / 19.0);
    R = fma3(R, z, 2.0 / 17.0);
    R = fma3(R, z, 2.0 / 15.0);
    R = fma3(R, z, 2.0 / 13.0);
    R = fma3(R, z, 2.0 / 11.0);
    R = fma3(R, z, 2.0 / 9.0);
    R = fma3(R, z, 2.0 / 7.0);
    R = fma3(R, z, 2.0 / 5.0);
    R = fma3(R, z, 2.0 / 3.0);
#endif
    const double lm = fma(s * z, R, s + s);  // log m = 2s + s z R(z)
    const double de = (double)e;
    return fma(de, kLn2Hi, fma(de, kLn2Lo, lm));
}

__device__ __forceinline__ double softplus_pm(double z) { return pm_log(1.0 + pm_exp(z)); }

// exp(z) as pm_exp with plain fma() Horner steps (the coefficients in SGPRs / literals): the
// exact f evaluates two per call in register-heavy code, where pm_exp's asm block (coefficients
// pinned in VGPRs) pushed the subtree kernel into spills.
__device__ __forceinline__ double exp_plain(double z) {
    constexpr double kLog2e = 1.4426950408889634;
    constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
    const double k = __builtin_rint(z * kLog2e);
    double r = fma(-k, kLn2Hi, z);
    r = fma(-k, kLn2Lo, r);
    double p = 1.6059043836821613e-10;  // 1/i!, i = 13 .. 0
    p = fma(p, r, 2.08767569878681e-09);
    p = fma(p, r, 2.505210838544172e-08);
    p = fma(p, r, 2.755731922398589e-07);
    p = fma(p, r, 2.7557319223985893e-06);
    p = fma(p, r, 2.48015873015873e-05);
    p = fma(p, r, 0.0001984126984126984);
    p = fma(p, r, 0.001388888888888889);
    p = fma(p, r, 0.008333333333333333);
    p = fma(p, r, 0.041666666666666664);
    p = fma(p, r, 0.16666666666666666);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    return ldexp(p, (int)k);
}

// log(1 + z) for z in [0, 1]: 2 atanh(s), s = z / (2 + z) in [0, 1/3], series through s^35
// (truncation < 5e-18 relative).
__device__ __forceinline__ double log1p_01(double z) {
    const double s = z / (2.0 + z);
    const double w = s * s;
    double R = 2.0 / 35.0;  // sum_{i>=1} 2/(2i+1) w^(i-1), i = 1 .. 17
    R = fma(R, w, 2.0 / 33.0);
    R = fma(R, w, 2.0 / 31.0);
    R = fma(R, w, 2.0 / 29.0);
    R = fma(R, w, 2.0 / 27.0);
    R = fma(R, w, 2.0 / 25.0);
    R = fma(R, w, 2.0 / 23.0);
    R = fma(R, w, 2.0 / 21.0);
    R = fma(R, w, 2.0 / 19.0);
    R = fma(R, w, 2.0 / 17.0);
    R = fma(R, w, 2.0 / 15.0);
    R = fma(R, w, 2.0 / 13.0);
    R = fma(R, w, 2.0 / 11.0);
    R = fma(R, w, 2.0 / 9.0);
    R = fma(R, w, 2.0 / 7.0);
    R = fma(R, w, 2.0 / 5.0);
    R = fma(R, w, 2.0 / 3.0);
    return fma(s * w, R, s + s);
}

// The exact boxplus of the my_sn list decoder (my_sn/fec/polar/dec.py:330-339, float64):
//   log(1 + e^(x+y)) - log(e^x + e^y) = sign(x) sign(y) min(|x|, |y|) + log1p(e^-|x+y|) - log1p(e^-|x-y|)
// on the clipped inputs -- algebraically the reference's expression, evaluated without its
// cancellation: two exp and two log1p on [0, 1] instead of three exp and two general logs, and a
// result closer to the exact value than the reference's own (whose rounding error is ~1e-14
// absolute at |x + y| ~ 60).  Measured against the reference's decoded rows (my_sn SCL_Dec, 5,000
// rows, tests/test_exactf_gpu.py): the C oracle with this form disagrees on 1, with the
// reference's form on 0.  Shared by scl_kernel.hip and
// scl_tree_kernel.hip, so the two kernels stay bit-identical.
__device__ __forceinline__ double f_exact_pm(double x, double y, double lmax) {
    const double xc = fmax(fmin(x, lmax), -lmax), yc = fmax(fmin(y, lmax), -lmax);
    const double m = fmin(fabs(xc), fabs(yc));
    const double sm = ((__double_as_longlong(xc) ^ __double_as_longlong(yc)) < 0) ? -m : m;
    return (sm + log1p_01(exp_plain(-fabs(xc + yc)))) - log1p_01(exp_plain(-fabs(xc - yc)));
}

}  // namespace pl
