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
// error (< 2^-50 relative) leaves a wrong fp32 rounding only for arguments within 2^-26 ulp of a
// rounding boundary.  Range: exp_cr for |x| <= 87 (normal fp32 results), log_cr for finite x > 0;
// plans with llr_max > 43 take the full-range forms (exp_cr_wide / log_cr_wide) instead.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

namespace plx {

// Polynomials: Chebyshev economisations (tools/cheb_coeffs.py) of the Taylor series -- e^r on
// |r| <= ln2/2 at degree 10 (tail < 2.2e-16, was Taylor degree 11: 7e-15) and the atanh series
// sum 2/(2i+1) z^(i-1) on z <= 0.0295 at degree 5 (tail < 5e-14, times s z <= 0.005: below 3e-16
// relative to log m, as the Taylor degree 8 it replaces).  Checked on the host against expl/logl
// rounded to fp32: 0 of 5e7 exp and 1 of 5e7 log arguments misrounded, the same as the Taylor forms.
__device__ constexpr double kExpC[11] = {
    1.0, 1.0000000000000067, 0.5000000000000019, 0.16666666666554325, 0.041666666666487974,
    0.008333333385695266, 0.001388888895234707, 0.00019841170236135905, 2.480148544815057e-05,
    2.7640194893802356e-06, 2.763265216957956e-07};
__device__ constexpr double kLogC[6] = {
    0.6666666666666206, 0.40000000011263015, 0.2857142412272895, 0.22222863785496652,
    0.18140134518808063, 0.16622633991749486};

// exp(x) for fp32 x, |x| <= 87: x = k ln2 + r (|r| <= ln2/2, two-part ln2), degree-10 polynomial
// in fp64, rounded to fp32, then scaled by 2^k exactly.
__device__ __forceinline__ float exp_cr(float xf) {
    const double x = (double)xf;
    constexpr double kLog2e = 1.4426950408889634;
    constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
    const double k = __builtin_rint(x * kLog2e);
    double r = __builtin_fma(-k, kLn2Hi, x);
    r = __builtin_fma(-k, kLn2Lo, r);
    double p = kExpC[10];
#pragma unroll
    for (int i = 9; i >= 0; --i) p = __builtin_fma(p, r, kExpC[i]);
    // p in [0.70, 1.42]: rounding p and scaling by 2^k (|k| <= 126, a normal result) is one rounding
    return __builtin_ldexpf((float)p, (int)k);
}

// log(x) for finite fp32 x > 0: x = 2^e m, m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s) with
// s = (m - 1) / (m + 1), |s| < 0.1716, in fp64; the quotient from a reciprocal with two Newton
// steps and a residual correction (denominator in [1.41, 2.83]).
__device__ __forceinline__ float log_cr(float xf) {
    constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
    double m = __builtin_amdgcn_frexp_mant((double)xf);  // [0.5, 1)
    int e = __builtin_amdgcn_frexp_exp((double)xf);
    if (m < 0.70710678118654752) {
        m = m + m;
        e -= 1;
    }
    const double f = m - 1.0;  // exact
    const double den = 2.0 + f;
    double rc = __builtin_amdgcn_rcp(den);
    double t = __builtin_fma(-den, rc, 1.0);
    rc = __builtin_fma(rc, t, rc);
    t = __builtin_fma(-den, rc, 1.0);
    rc = __builtin_fma(rc, t, rc);
    const double q = f * rc;
    const double s = __builtin_fma(rc, __builtin_fma(-den, q, f), q);
    const double z = s * s;
    double R = kLogC[5];
#pragma unroll
    for (int i = 4; i >= 0; --i) R = __builtin_fma(R, z, kLogC[i]);
    const double lm = __builtin_fma(s * z, R, s + s);  // log m = 2s + s z R(z)
    const double de = (double)e;
    return (float)__builtin_fma(de, kLn2Hi, __builtin_fma(de, kLn2Lo, lm));
}

// Full-range forms, for plans whose llr_max exceeds 43 (then xc + yc can leave exp_cr's range):
// exp rounds p 2^k once in the fp64 -> fp32 conversion (overflow to +inf and subnormal results
// correctly rounded, as torch's expf), log maps +inf to +inf and 0 to -inf (torch's logf), so
// f follows the reference through overflow (inf, or inf - inf = NaN, as the reference's own).
__device__ __forceinline__ float exp_cr_wide(float xf) {
    const double x = (double)__builtin_amdgcn_fmed3f(xf, -200.0f, 200.0f);  // e^+-200: inf / 0 in fp32
    constexpr double kLog2e = 1.4426950408889634;
    constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
    const double k = __builtin_rint(x * kLog2e);
    double r = __builtin_fma(-k, kLn2Hi, x);
    r = __builtin_fma(-k, kLn2Lo, r);
    double p = kExpC[10];
#pragma unroll
    for (int i = 9; i >= 0; --i) p = __builtin_fma(p, r, kExpC[i]);
    return (float)__builtin_ldexp(p, (int)k);  // exact scaling in fp64, one rounding to fp32
}
__device__ __forceinline__ float log_cr_wide(float xf) {
    const float r = log_cr(xf);
    return xf == __builtin_inff() ? xf : xf == 0.0f ? -__builtin_inff() : r;
}
__device__ __attribute__((noinline)) float f_exact_wide(float x, float y, float lmax) {
    const float xc = fminf(fmaxf(x, -lmax), lmax), yc = fminf(fmaxf(y, -lmax), lmax);
    float o = log_cr_wide(1.0f + exp_cr_wide(xc + yc));
    o -= log_cr_wide(exp_cr_wide(xc) + exp_cr_wide(yc));
    return o;
}
// exp_cr's range |x| <= 87 holds for every argument f forms when llr_max <= 43 (|xc + yc| <= 86)
constexpr float kExactFastLmax = 43.0f;

// f of my_sn/fec/polar/dec.py:39-43 on clipped inputs, each operation rounded as the reference does.
// Out of line: inlined into the fully unrolled specialised SC kernels (hundreds of f per lane) the
// fp64 code made one (128,256) kernel take minutes to compile.
__device__ __attribute__((noinline)) float f_exact(float x, float y, float lmax) {
    if (lmax > kExactFastLmax) return f_exact_wide(x, y, lmax);
    const float xc = fminf(fmaxf(x, -lmax), lmax), yc = fminf(fmaxf(y, -lmax), lmax);
    float o = log_cr(1.0f + exp_cr(xc + yc));
    o -= log_cr(exp_cr(xc) + exp_cr(yc));
    return o;
}

// Two f at once (one call, the two evaluations' fp64 chains interleaved by the scheduler): the
// specialised SC kernel's lane-local f loops call this for element pairs.  Each value is exactly
// f_exact's.
struct f2 {
    float a, b;
};
__device__ __attribute__((noinline)) f2 f_exact2(float x0, float y0, float x1, float y1, float lmax) {
    if (lmax > kExactFastLmax) return f2{f_exact_wide(x0, y0, lmax), f_exact_wide(x1, y1, lmax)};
    const float xc0 = fminf(fmaxf(x0, -lmax), lmax), yc0 = fminf(fmaxf(y0, -lmax), lmax);
    const float xc1 = fminf(fmaxf(x1, -lmax), lmax), yc1 = fminf(fmaxf(y1, -lmax), lmax);
    const float s0 = exp_cr(xc0 + yc0), s1 = exp_cr(xc1 + yc1);
    const float a0 = exp_cr(xc0), a1 = exp_cr(xc1);
    const float b0 = exp_cr(yc0), b1 = exp_cr(yc1);
    const float p0 = log_cr(1.0f + s0), p1 = log_cr(1.0f + s1);
    const float q0 = log_cr(a0 + b0), q1 = log_cr(a1 + b1);
    f2 r;
    r.a = p0 - q0;
    r.b = p1 - q1;
    return r;
}

}  // namespace plx
