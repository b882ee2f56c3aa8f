// softplus.h -- the SCL path-metric penalty log(1 + exp(z)) in fp64 (x_run_sn_polar/polar/
// polar_scl.py:83 computes np.log(1 + np.exp(-(1-2u) * clip(llr))) in float64).
//
// Shared by scl_kernel.hip and scl_tree_kernel.hip so the two kernels produce identical metrics.
// Same three roundings as the reference -- e = exp(z), y = 1 + e, log(y) -- with exp and log
// evaluated for the range the decoder uses instead of through ocml's general routines:
//   exp: z = k ln2 + r (Cody-Waite, two-part ln2 with FMA), |r| <= ln2/2, a polynomial, scaled
//        by 2^k;
//   log: y = 2^e m, m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s), s = (m-1)/(m+1), |s| < 0.1716.
// The default (PL_SP_FORM 2, below softplus_pm) uses Chebyshev-economised polynomials evaluated
// in Estrin form and a Newton reciprocal for s; the Taylor forms of rounds 1-2 (pm_exp / pm_log,
// degree 13 and s^25) remain as PL_SP_FORM 0.  Both are within ~1.5 ulp of the correctly rounded
// exp and log, like ocml's and numpy's.  Valid for |z| <= 700: pl_plan_create rejects list plans
// with llr_max > 700.  The exact boxplus of the my_sn list decoder (f_exact_pm_n) is at the end.
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

// Economised forms (PL_SP_FORM 1: Horner, 2: Estrin), the same three roundings -- e = exp(z),
// y = 1 + e, log(y):
//   exp(r) = 1 + r + r^2 P(r), P the degree-9 Chebyshev economisation of (e^r - 1 - r)/r^2 on
//            |r| <= ln2/2 (tail < 1.1e-16, times r^2 <= 0.12; tools/cheb_coeffs.py);
//   log m  = 2s + s z RL(z), z = s^2 <= 0.0295, RL the degree-6 economisation of
//            sum 2/(2i+1) z^(i-1) (tail < 3.1e-16, times s z <= 0.005);
//   s = f / (2 + f): a reciprocal, two Newton steps and a residual correction (denominator in
//   [1.41, 2.83]) instead of the scaled IEEE division sequence.
// 7 fewer FMAs and a shorter division than the Taylor forms above, same accuracy class (~1 ulp).
#ifndef PL_SP_FORM
#define PL_SP_FORM 2  // A/B r03l: 0.990 vs 1.000 ms (min-sum), 1.050 vs 1.113 ms (min-sum fast-SCL)
#endif
__device__ constexpr double kSpP[10] = {
    0.5000000000000001, 0.1666666666666667, 0.04166666666662413, 0.008333333333326136,
    0.001388888891721154, 0.00019841269874817515, 2.4801521299750923e-05, 2.75572554044176e-06,
    2.7620086491464514e-07, 2.5105215165649368e-08};
__device__ constexpr double kSpRL[7] = {
    0.666666666666667, 0.39999999999898955, 0.2857142862619623, 0.22222211102348335,
    0.18182891280109284, 0.15331655663402047, 0.14617206088074544};
template <bool ESTRIN>
__device__ __forceinline__ double pm_exp_e(double z) {
    constexpr double kLog2e = 1.4426950408889634;
    constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
    const double k = __builtin_rint(z * kLog2e);
    double r = fma(-k, kLn2Hi, z);
    r = fma(-k, kLn2Lo, r);
    const double r2 = r * r;
    double P;
    if constexpr (ESTRIN) {
        const double a = fma(kSpP[9], r, kSpP[8]), b = fma(kSpP[7], r, kSpP[6]), c = fma(kSpP[5], r, kSpP[4]);
        const double d = fma(kSpP[3], r, kSpP[2]), e = fma(kSpP[1], r, kSpP[0]);
        const double r4 = r2 * r2;
        const double ab = fma(a, r2, b), cd = fma(c, r2, d);
        P = fma(fma(ab, r4, cd), r2, e);
    } else {
        P = kSpP[9];
#pragma unroll
        for (int i = 8; i >= 0; --i) P = fma(P, r, kSpP[i]);
    }
    return ldexp(fma(r2, P, r) + 1.0, (int)k);
}
template <bool ESTRIN>
__device__ __forceinline__ double pm_log_e(double y) {  // y >= 1, finite
    constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
    double m = __builtin_amdgcn_frexp_mant(y);  // [0.5, 1)
    int e = __builtin_amdgcn_frexp_exp(y);
    if (m < 0.70710678118654752) {
        m = m + m;
        e -= 1;
    }
    const double f = m - 1.0;  // exact (Sterbenz)
    const double den = 2.0 + f;
    double rc = __builtin_amdgcn_rcp(den);
    double t = fma(-den, rc, 1.0);
    rc = fma(rc, t, rc);
    t = fma(-den, rc, 1.0);
    rc = fma(rc, t, rc);
    const double q = f * rc;
    const double s = fma(rc, fma(-den, q, f), q);
    const double z = s * s;
    double R;
    if constexpr (ESTRIN) {
        const double p01 = fma(kSpRL[1], z, kSpRL[0]), p23 = fma(kSpRL[3], z, kSpRL[2]);
        const double p45 = fma(kSpRL[5], z, kSpRL[4]);
        const double z2 = z * z, z4 = z2 * z2;
        R = fma(fma(kSpRL[6], z2, p45), z4, fma(p23, z2, p01));
    } else {
        R = kSpRL[6];
#pragma unroll
        for (int i = 5; i >= 0; --i) R = fma(R, z, kSpRL[i]);
    }
    const double lm = fma(s * z, R, s + s);  // log m = 2s + s z R(z)
    const double de = (double)e;
    return fma(de, kLn2Hi, fma(de, kLn2Lo, lm));
}
#if PL_SP_FORM == 0
__device__ __forceinline__ double softplus_pm(double z) { return pm_log(1.0 + pm_exp(z)); }
#else
__device__ __forceinline__ double softplus_pm(double z) {
    return pm_log_e<PL_SP_FORM == 2>(1.0 + pm_exp_e<PL_SP_FORM == 2>(z));
}
#endif

// The exact boxplus of the my_sn list decoder (my_sn/fec/polar/dec.py:330-339, float64),
//   f = log(1 + e^(x+y)) - log(e^x + e^y)
// on the clipped inputs, evaluated without the reference's cancellation.  With a = |x|, b = |y|,
// m = min(a, b), M = max(a, b), E = e^-(M-m), G = 1 - e^-2m (= -expm1(-2m)):
//   f = sign(x) sign(y) (m + log(1 + E (1 - G)) - log(1 + E)) = sign(x) sign(y) (m + log1p(-t)),
//   t = E G / (1 + E) in [0, 1/2),  log1p(-t) = 2 atanh(s),  s = -E G / (2 (1 + E) - E G),  |s| <= 1/3
// -- one exp and one expm1 (one shared degree-9 polynomial), one quotient (denominator in [2, 4]: a
// reciprocal with two Newton steps and a residual correction, no scaling needed) and one odd series
// (degree 10 in s^2), ~60 VALU instead of the reference form's three exp and two general logs.  Absolute
// error ~1e-16, against the reference's own ~1e-16 (small inputs) to ~1e-14 (|x + y| ~ 60), so
// decisions follow the exact value at least as closely as the reference's do; parity is the
// statistical row-mismatch gate of tests/test_exactf_gpu.py.
// N independent evaluations are interleaved step by step (N = 2: the x and y inputs of a node),
// so the dependent fp64 chains of one wave overlap; every lane value is the same whatever N is.
// Shared by scl_kernel.hip and scl_tree_kernel.hip, so the two kernels stay bit-identical.
__device__ __forceinline__ double vmin_nc(double a, double b) {  // v_min_f64 without canonicalisation
    double d;
    asm("v_min_f64 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
__device__ __forceinline__ double vmax_nc(double a, double b) {
    double d;
    asm("v_max_f64 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
__device__ __forceinline__ double vmin_abs_nc(double a, double b) {
    double d;
    asm("v_min_f64 %0, |%1|, |%2|" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
__device__ __forceinline__ double vmax_abs_nc(double a, double b) {
    double d;
    asm("v_max_f64 %0, |%1|, |%2|" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
template <int N>
__device__ __forceinline__ void f_exact_pm_n(const double* x, const double* y, double lmax, double* out) {
    constexpr double kLog2e = 1.4426950408889634;
    constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
    // 2 atanh(s) = 2s + s w R(w), w = s^2 <= 1/9: R of degree 10, the Chebyshev economisation of
    // sum 2/(2i+3) w^i (tail < 2.4e-18)
    constexpr double kS[11] = {
        0.6666666666666666, 0.39999999999999514, 0.28571428571603413, 0.22222222197853667,
        0.18181819920440906, 0.15384543207664578, 0.133351941539121, 0.11734082174871642,
        0.10846687166200544, 0.07485743922141379, 0.1564211337480669};
    double m[N], ze[N], zm[N], ke[N], km[N], re[N], rm[N], pe[N], pm[N];
    bool neg[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const double xc = vmax_nc(vmin_nc(x[i], lmax), -lmax), yc = vmax_nc(vmin_nc(y[i], lmax), -lmax);
        neg[i] = (__double_as_longlong(xc) ^ __double_as_longlong(yc)) < 0;
        m[i] = vmin_abs_nc(xc, yc);
        ze[i] = m[i] - vmax_abs_nc(xc, yc);  // -(M - m) <= 0
        zm[i] = -2.0 * m[i];
    }
    // exp(r) = 1 + r + r^2 P(r), expm1(r) = r + r^2 P(r), |r| <= ln2/2: P of degree 9, the Chebyshev
    // economisation of the Taylor series of (e^r - 1 - r) / r^2 (tail < 1.1e-16, times r^2 <= 0.12);
    // the coefficients and the economised series below: tools/cheb_coeffs.py
    constexpr double kP[10] = {
        0.5000000000000001, 0.1666666666666667, 0.04166666666662413, 0.008333333333326136,
        0.001388888891721154, 0.00019841269874817515, 2.4801521299750923e-05, 2.75572554044176e-06,
        2.7620086491464514e-07, 2.5105215165649368e-08};
#pragma unroll
    for (int i = 0; i < N; ++i) {  // Cody-Waite reductions of both exponents
        ke[i] = __builtin_rint(ze[i] * kLog2e);
        km[i] = __builtin_rint(zm[i] * kLog2e);
        re[i] = fma(-ke[i], kLn2Hi, ze[i]);
        rm[i] = fma(-km[i], kLn2Hi, zm[i]);
        re[i] = fma(-ke[i], kLn2Lo, re[i]);
        rm[i] = fma(-km[i], kLn2Lo, rm[i]);
        pe[i] = kP[9];
        pm[i] = kP[9];
    }
#pragma unroll
    for (int c = 8; c >= 0; --c) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            pe[i] = fma(pe[i], re[i], kP[c]);
            pm[i] = fma(pm[i], rm[i], kP[c]);
        }
    }
    double E[N], G[N], eg[N], den[N], rc[N], s[N], w[N], R[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        E[i] = ldexp(fma(re[i] * re[i], pe[i], re[i]) + 1.0, (int)ke[i]);  // exp(-(M - m))
        const double tk = ldexp(1.0, (int)km[i]);
        G[i] = -fma(tk, fma(rm[i] * rm[i], pm[i], rm[i]), tk - 1.0);  // -expm1(-2m)
        eg[i] = E[i] * G[i];
        den[i] = fma(2.0, E[i], 2.0) - eg[i];  // in [2, 4]
        rc[i] = __builtin_amdgcn_rcp(den[i]);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {  // s = -eg / den: two Newton steps on the reciprocal, one on the quotient
        double e = fma(-den[i], rc[i], 1.0);
        rc[i] = fma(rc[i], e, rc[i]);
        e = fma(-den[i], rc[i], 1.0);
        rc[i] = fma(rc[i], e, rc[i]);
        const double q = eg[i] * rc[i];
        s[i] = -fma(rc[i], fma(-den[i], q, eg[i]), q);
        w[i] = s[i] * s[i];
        R[i] = kS[10];
    }
#pragma unroll
    for (int c = 9; c >= 0; --c) {
#pragma unroll
        for (int i = 0; i < N; ++i) R[i] = fma(R[i], w[i], kS[c]);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const double v = m[i] + fma(s[i] * w[i], R[i], s[i] + s[i]);
        out[i] = neg[i] ? -v : v;
    }
}
__device__ __forceinline__ double f_exact_pm(double x, double y, double lmax) {
    double r;
    f_exact_pm_n<1>(&x, &y, lmax, &r);
    return r;
}

}  // namespace pl
