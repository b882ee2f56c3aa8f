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
//   s = f / (2 + f): a reciprocal, PL_RCP_STEPS Newton steps and a residual correction (denominator in
//   [1.41, 2.83]) instead of the scaled IEEE division sequence.
// 7 fewer FMAs and a shorter division than the Taylor forms above, same accuracy class (~1 ulp).
#ifndef PL_SP_ASM
#define PL_SP_ASM 1  // the Estrin polynomials as asm blocks of VOP3 FMAs: A/B 0.734 -> 0.714 ms min-sum SCL,
                    // bit-identical (profiles/r06zd_spasm_ab2.txt); 0: plain fma()
#endif
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
    if constexpr (ESTRIN && PL_SP_ASM) {
        // the same operations as below, each first-level pair as a VOP3 FMA with its multiplier in
        // an SGPR and its addend in a VGPR: left to itself the compiler uses the two-address
        // v_fmac_f64 and copies the (loop-invariant) addend into the destination first -- one
        // v_mov_b64 per pair; one block, so no hazard padding between the steps
        double a, b, c, d, e, r4, ab, cd, t;
        asm("v_fma_f64 %0, %9, %11, %12\n\t"
            "v_fma_f64 %1, %9, %13, %14\n\t"
            "v_fma_f64 %2, %9, %15, %16\n\t"
            "v_fma_f64 %3, %9, %17, %18\n\t"
            "v_fma_f64 %4, %9, %19, %20\n\t"
            "v_mul_f64 %5, %10, %10\n\t"
            "v_fma_f64 %6, %0, %10, %1\n\t"
            "v_fma_f64 %7, %2, %10, %3\n\t"
            "v_fma_f64 %8, %6, %5, %7\n\t"
            "v_fma_f64 %8, %8, %10, %4"
            : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d), "=&v"(e), "=&v"(r4), "=&v"(ab), "=&v"(cd), "=&v"(t)
            : "v"(r), "v"(r2), "s"(kSpP[9]), "v"(kSpP[8]), "s"(kSpP[7]), "v"(kSpP[6]), "s"(kSpP[5]),
              "v"(kSpP[4]), "s"(kSpP[3]), "v"(kSpP[2]), "s"(kSpP[1]), "v"(kSpP[0]));
        P = t;
    } else if constexpr (ESTRIN) {
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
// Newton steps on v_rcp_f64 before the quotient's residual correction (pm_log_e, f_exact_pm_n).
// With rc = (1 + e)/den the corrected quotient q + rc (f - den q) is (f/den)(1 - e^2): the
// correction squares whatever error the reciprocal has left.  v_rcp_f64 is within 2^-24.4 on
// both kernels' denominator ranges (tools/micro/rcp_check.hip, profiles/r06j_rcp_check.txt, 2.1e9
// denominators), so after one Newton step e^2 < 2^-97 and the quotient is the two-step one on
// every one of them (and on 2e7 host-emulated worst cases down to a 2^-20 reciprocal).  Same
// values, two fp64 FMAs fewer per penalty and per exact f: A/B 0.759 -> 0.735 ms min-sum SCL,
// 2.080 -> 2.021 ms my_sn SCL (profiles/r06j_scl_rcp1_ab*.txt, identical bits and metrics).
#ifndef PL_RCP_STEPS
#define PL_RCP_STEPS 1
#endif
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
    if (PL_RCP_STEPS > 1) {
        t = fma(-den, rc, 1.0);
        rc = fma(rc, t, rc);
    }
    const double q = f * rc;
    const double s = fma(rc, fma(-den, q, f), q);
    const double z = s * s;
    double R;
    if constexpr (ESTRIN && PL_SP_ASM) {  // as in pm_exp_e: VOP3 FMAs, no addend copies
        double p01, p23, p45, z2, z4, u, v;
        asm("v_fma_f64 %0, %7, %8, %9\n\t"
            "v_fma_f64 %1, %7, %10, %11\n\t"
            "v_fma_f64 %2, %7, %12, %13\n\t"
            "v_mul_f64 %3, %7, %7\n\t"
            "v_mul_f64 %4, %3, %3\n\t"
            "v_fma_f64 %5, %3, %14, %2\n\t"
            "v_fma_f64 %6, %1, %3, %0\n\t"
            "v_fma_f64 %5, %5, %4, %6"
            : "=&v"(p01), "=&v"(p23), "=&v"(p45), "=&v"(z2), "=&v"(z4), "=&v"(u), "=&v"(v)
            : "v"(z), "s"(kSpRL[1]), "v"(kSpRL[0]), "s"(kSpRL[3]), "v"(kSpRL[2]), "s"(kSpRL[5]),
              "v"(kSpRL[4]), "s"(kSpRL[6]));
        R = u;
    } else if constexpr (ESTRIN) {
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
// PL_SP_FORM 3: the log table-driven (no division).  y = 1 + e^z >= 1, so y = 2^e m with
// m in [1, 2): cell j = the top 7 bits of m's fraction, r = m c_j - 1 (one fma; |r| <= 2^-8, 2^-7 in
// cell 0 where c_0 = 1), ln y = e ln2 + (-ln c_j) + log1p(r) with log1p by degree 8 (remainder
// < 2^-59 relative) -- 21 VALU and one 16-byte LDS read instead of ~30 VALU with a reciprocal and
// two Newton steps.  The table (2 KB) lives in LDS: kernels that evaluate the penalty call
// sp_load_tables() at entry (all threads of the work-group, then a barrier).  Not the default:
// A/B r04zd, SCL (512,1024) L = 8, bs = 8192: min-sum 0.857 vs 0.850 ms (the LDS read sits on the
// leaf's dependent chain), my_sn exact + fast-SCL 1.915 vs 1.961 ms but with 7 VGPRs spilled.
struct SpCell {
    float c;    // c_j
    float lo;   // -ln c_j - hi
    double hi;  // -ln c_j rounded to fp64
};
// ---- BEGIN GENERATED SP TABLE (tools/gen_sp_tables.py) ----
// {c_j (fp32), lo(-ln c_j) (fp32), hi(-ln c_j) (fp64)} per cell j of m in [1, 2)
__device__ const SpCell kSpLogTab[128] = {
    {0x1.0000000000000p+0f, 0.0f, 0x0.0p+0},
    {0x1.fa11ca0000000p-1f, 0x1.8494a20000000p-61f, 0x1.7dc49e7810addp-7},
    {0x1.f6310a0000000p-1f, -0x1.765a220000000p-61f, 0x1.3cea5df46a5c8p-6},
    {0x1.f25f640000000p-1f, 0x1.ea33420000000p-65f, 0x1.b9fc0afaf91a1p-6},
    {0x1.ee9c800000000p-1f, -0x1.e9ae9e0000000p-60f, 0x1.1b0d90923d990p-5},
    {0x1.eae8080000000p-1f, 0x1.c6a8e80000000p-61f, 0x1.58a5b57c8e4dcp-5},
    {0x1.e741aa0000000p-1f, 0x1.e683b00000000p-61f, 0x1.95c836cc8e3f4p-5},
    {0x1.e3a9180000000p-1f, -0x1.7870f00000000p-59f, 0x1.d276b22db0b5dp-5},
    {0x1.e01e020000000p-1f, -0x1.fb25ac0000000p-59f, 0x1.075982498e472p-4},
    {0x1.dca01e0000000p-1f, -0x1.8a125a0000000p-58f, 0x1.253f6120a1419p-4},
    {0x1.d92f220000000p-1f, -0x1.5f15820000000p-58f, 0x1.42edcd9a646f2p-4},
    {0x1.d5cac80000000p-1f, -0x1.1884580000000p-58f, 0x1.60658ad3750c4p-4},
    {0x1.d272ca0000000p-1f, -0x1.73b7f00000000p-60f, 0x1.7da76907b12cfp-4},
    {0x1.cf26e60000000p-1f, -0x1.c99e340000000p-63f, 0x1.9ab42252033afp-4},
    {0x1.cbe6da0000000p-1f, -0x1.fcf0f40000000p-58f, 0x1.b78c7d2b0edb1p-4},
    {0x1.c8b2660000000p-1f, 0x1.4b0dd80000000p-58f, 0x1.d4313a96cb361p-4},
    {0x1.c5894e0000000p-1f, -0x1.80d0c40000000p-62f, 0x1.f0a30391162cap-4},
    {0x1.c26b540000000p-1f, -0x1.4e737a0000000p-59f, 0x1.06714f3ca5972p-3},
    {0x1.bf583e0000000p-1f, -0x1.4477d40000000p-57f, 0x1.14785c6e742bep-3},
    {0x1.bc4fd60000000p-1f, 0x1.e47c080000000p-61f, 0x1.2266f328a5acep-3},
    {0x1.b951e20000000p-1f, 0x1.6b519a0000000p-57f, 0x1.303d74c647fddp-3},
    {0x1.b65e2e0000000p-1f, -0x1.93a8da0000000p-62f, 0x1.3dfc2c26cc62bp-3},
    {0x1.b374840000000p-1f, -0x1.f367da0000000p-57f, 0x1.4ba37269a55f0p-3},
    {0x1.b094b40000000p-1f, 0x1.7116d20000000p-57f, 0x1.5933896982097p-3},
    {0x1.adbe880000000p-1f, -0x1.d201ca0000000p-59f, 0x1.66acd4072ad51p-3},
    {0x1.aaf1d20000000p-1f, 0x1.dfce1e0000000p-57f, 0x1.740f93fc037bap-3},
    {0x1.a82e660000000p-1f, -0x1.89e4bc0000000p-58f, 0x1.815c059c357ffp-3},
    {0x1.a574100000000p-1f, -0x1.169d820000000p-57f, 0x1.8e92902886d46p-3},
    {0x1.a2c2a80000000p-1f, -0x1.8a1c9a0000000p-61f, 0x1.9bb36547dfb89p-3},
    {0x1.a01a020000000p-1f, 0x1.493c820000000p-58f, 0x1.a8becdf082f1cp-3},
    {0x1.9d79f20000000p-1f, 0x1.f327f80000000p-57f, 0x1.b5b51740fb5abp-3},
    {0x1.9ae24e0000000p-1f, -0x1.6f6c360000000p-64f, 0x1.c2968890c18cbp-3},
    {0x1.9852f00000000p-1f, 0x1.639a220000000p-57f, 0x1.cf6359209c5eep-3},
    {0x1.95cbb00000000p-1f, 0x1.c34c640000000p-57f, 0x1.dc1bcdcabec8bp-3},
    {0x1.934c680000000p-1f, -0x1.2e03a40000000p-59f, 0x1.e8c0250aa5a60p-3},
    {0x1.90d4f20000000p-1f, -0x1.5057e20000000p-64f, 0x1.f550a0ecb7b4bp-3},
    {0x1.8e65280000000p-1f, 0x1.88d52c0000000p-58f, 0x1.00e6c38ad501ep-2},
    {0x1.8bfce80000000p-1f, 0x1.f170800000000p-58f, 0x1.071b860cd590dp-2},
    {0x1.899c100000000p-1f, 0x1.a1f63c0000000p-56f, 0x1.0d46b3d9ab750p-2},
    {0x1.87427c0000000p-1f, -0x1.0a675a0000000p-58f, 0x1.13686fa13a8b1p-2},
    {0x1.84f00c0000000p-1f, -0x1.10c2e40000000p-56f, 0x1.1980d34542370p-2},
    {0x1.82a4a00000000p-1f, -0x1.49fdfa0000000p-56f, 0x1.1f8ffa248a2f3p-2},
    {0x1.8060180000000p-1f, -0x1.deed8a0000000p-59f, 0x1.2596011df763ap-2},
    {0x1.7e22560000000p-1f, -0x1.64eb740000000p-56f, 0x1.2b93013789d31p-2},
    {0x1.7beb3a0000000p-1f, -0x1.7135ba0000000p-57f, 0x1.31871a4144190p-2},
    {0x1.79baa60000000p-1f, -0x1.6c58920000000p-57f, 0x1.37726827fd863p-2},
    {0x1.7790820000000p-1f, -0x1.bea6700000000p-56f, 0x1.3d54f7e81f71cp-2},
    {0x1.756cac0000000p-1f, -0x1.bc98b80000000p-59f, 0x1.432ef2f84e814p-2},
    {0x1.734f0c0000000p-1f, 0x1.c201e60000000p-56f, 0x1.490068ec009d2p-2},
    {0x1.7137860000000p-1f, -0x1.7450d80000000p-57f, 0x1.4ec9758200275p-2},
    {0x1.6f26020000000p-1f, -0x1.a89d020000000p-57f, 0x1.548a2aa6dd268p-2},
    {0x1.6d1a620000000p-1f, 0x1.b386940000000p-57f, 0x1.5a42ac334cfe4p-2},
    {0x1.6b14900000000p-1f, -0x1.7c60de0000000p-57f, 0x1.5ff308ea793dbp-2},
    {0x1.6914740000000p-1f, 0x1.896c2a0000000p-56f, 0x1.659b56383e1f4p-2},
    {0x1.6719f40000000p-1f, -0x1.e215d20000000p-58f, 0x1.6b3bb05b59444p-2},
    {0x1.6524f80000000p-1f, -0x1.a166400000000p-56f, 0x1.70d42f1789238p-2},
    {0x1.63356c0000000p-1f, 0x1.7695120000000p-56f, 0x1.7664dfcb9dbd2p-2},
    {0x1.614b360000000p-1f, 0x1.8fc38c0000000p-60f, 0x1.7bede21f7afc4p-2},
    {0x1.5f66440000000p-1f, 0x1.1b85140000000p-61f, 0x1.816f3fb20d49fp-2},
    {0x1.5d867c0000000p-1f, 0x1.27cd8e0000000p-58f, 0x1.86e91a5b30ba1p-2},
    {0x1.5babcc0000000p-1f, 0x1.a2a9640000000p-57f, 0x1.8c5b7dad8b48dp-2},
    {0x1.59d6200000000p-1f, -0x1.60e0ca0000000p-56f, 0x1.91c67bf45a84dp-2},
    {0x1.5805600000000p-1f, -0x1.da3f620000000p-56f, 0x1.972a345135159p-2},
    {0x1.56397c0000000p-1f, -0x1.0f7eec0000000p-56f, 0x1.9c86af25c0865p-2},
    {0x1.54725e0000000p-1f, -0x1.9f6d760000000p-56f, 0x1.a1dc07915b999p-2},
    {0x1.52aff60000000p-1f, 0x1.4b1da60000000p-56f, 0x1.a72a47a2bd9f0p-2},
    {0x1.50f22e0000000p-1f, 0x1.0958f60000000p-57f, 0x1.ac718c598b0e4p-2},
    {0x1.4f38f60000000p-1f, 0x1.18f2c80000000p-61f, 0x1.b1b1e177dfc5cp-2},
    {0x1.4d843c0000000p-1f, -0x1.28dbcc0000000p-56f, 0x1.b6eb599bcf35ep-2},
    {0x1.4bd3ee0000000p-1f, -0x1.5197900000000p-56f, 0x1.bc1e083cdad0bp-2},
    {0x1.4a27fa0000000p-1f, 0x1.2bc35e0000000p-56f, 0x1.c14a01ad5f034p-2},
    {0x1.4880520000000p-1f, 0x1.afb5c60000000p-57f, 0x1.c66f4ea3f6ff8p-2},
    {0x1.46dce40000000p-1f, 0x1.97bbb40000000p-56f, 0x1.cb8e04fcd7ad4p-2},
    {0x1.453d9e0000000p-1f, -0x1.0619900000000p-56f, 0x1.d0a63b7321e65p-2},
    {0x1.43a2740000000p-1f, 0x1.5c41360000000p-57f, 0x1.d5b7f6a62c696p-2},
    {0x1.420b520000000p-1f, 0x1.5cb9a80000000p-56f, 0x1.dac35526c5957p-2},
    {0x1.40782e0000000p-1f, 0x1.0984580000000p-58f, 0x1.dfc856946d5c7p-2},
    {0x1.3ee8f40000000p-1f, -0x1.0ac36e0000000p-56f, 0x1.e4c71b0e87705p-2},
    {0x1.3d5d9a0000000p-1f, 0x1.a8eb720000000p-58f, 0x1.e9bfa37586206p-2},
    {0x1.3bd60e0000000p-1f, 0x1.3a6e2c0000000p-58f, 0x1.eeb20b000ddf8p-2},
    {0x1.3a52440000000p-1f, 0x1.f601c00000000p-56f, 0x1.f39e5a4011e60p-2},
    {0x1.38d22e0000000p-1f, 0x1.de0ace0000000p-56f, 0x1.f884a0dbe9ecfp-2},
    {0x1.3755be0000000p-1f, -0x1.14b0ee0000000p-57f, 0x1.fd64ef2361583p-2},
    {0x1.35dce60000000p-1f, 0x1.9a0dd40000000p-57f, 0x1.011fab085ff8ap-1},
    {0x1.34679a0000000p-1f, 0x1.7eeaf00000000p-55f, 0x1.0389f052e6342p-1},
    {0x1.32f5ce0000000p-1f, -0x1.16a9000000000p-56f, 0x1.05f14d38645a4p-1},
    {0x1.3187760000000p-1f, -0x1.bf67dc0000000p-55f, 0x1.0855c7c6b4511p-1},
    {0x1.301c820000000p-1f, -0x1.d9d9080000000p-57f, 0x1.0ab76d0ee14d7p-1},
    {0x1.2eb4ea0000000p-1f, 0x1.c28cae0000000p-58f, 0x1.0d163d019d6b8p-1},
    {0x1.2d50a00000000p-1f, 0x1.7a84440000000p-55f, 0x1.0f7241e9b497dp-1},
    {0x1.2bef980000000p-1f, -0x1.79c7720000000p-55f, 0x1.11cb83007cd02p-1},
    {0x1.2a91ca0000000p-1f, -0x1.d6c3a60000000p-56f, 0x1.142200ec43d4dp-1},
    {0x1.2937260000000p-1f, -0x1.1699c20000000p-56f, 0x1.1675ca44ba60fp-1},
    {0x1.27dfa40000000p-1f, -0x1.a835da0000000p-55f, 0x1.18c6e0335cf09p-1},
    {0x1.268b380000000p-1f, 0x1.a3b8520000000p-55f, 0x1.1b154affda29fp-1},
    {0x1.2539d80000000p-1f, 0x1.0a75640000000p-56f, 0x1.1d610fbe77003p-1},
    {0x1.23eb7a0000000p-1f, -0x1.1b21260000000p-56f, 0x1.1faa33be70950p-1},
    {0x1.22a0120000000p-1f, 0x1.bb587a0000000p-56f, 0x1.21f0c0105beecp-1},
    {0x1.2157980000000p-1f, -0x1.cebb8c0000000p-57f, 0x1.2434b6fc83934p-1},
    {0x1.2012020000000p-1f, 0x1.e0eb400000000p-55f, 0x1.26761e85430e9p-1},
    {0x1.1ecf440000000p-1f, 0x1.2d09fa0000000p-55f, 0x1.28b5007b60783p-1},
    {0x1.1d8f560000000p-1f, -0x1.30fe6c0000000p-55f, 0x1.2af15fd0640b0p-1},
    {0x1.1c52300000000p-1f, 0x1.bee9d20000000p-55f, 0x1.2d2b3fa2edc9ep-1},
    {0x1.1b17c60000000p-1f, 0x1.a074380000000p-55f, 0x1.2f62aa7b09549p-1},
    {0x1.19e0120000000p-1f, 0x1.8e69120000000p-58f, 0x1.3197a0487fe6cp-1},
    {0x1.18ab080000000p-1f, 0x1.c46ba60000000p-55f, 0x1.33ca2c0b28995p-1},
    {0x1.1778a20000000p-1f, 0x1.ff7ea00000000p-55f, 0x1.35fa4e1336ea2p-1},
    {0x1.1648d60000000p-1f, -0x1.4f1bee0000000p-55f, 0x1.38280e2b8798bp-1},
    {0x1.151b9a0000000p-1f, 0x1.98b08a0000000p-55f, 0x1.3a53745debdfap-1},
    {0x1.13f0e80000000p-1f, 0x1.497f4a0000000p-56f, 0x1.3c7c81877320fp-1},
    {0x1.12c8b80000000p-1f, -0x1.19321c0000000p-56f, 0x1.3ea33a5eb2f61p-1},
    {0x1.11a3020000000p-1f, 0x1.5ab9140000000p-55f, 0x1.40c7a3ca0dcebp-1},
    {0x1.107fbc0000000p-1f, 0x1.93bee40000000p-55f, 0x1.42e9c6a1f80bfp-1},
    {0x1.0f5ee00000000p-1f, -0x1.fc07640000000p-57f, 0x1.4509a4733bb0cp-1},
    {0x1.0e40660000000p-1f, 0x1.76f66e0000000p-55f, 0x1.472742b53aab3p-1},
    {0x1.0d24460000000p-1f, -0x1.92ced00000000p-57f, 0x1.4942a7102fc0dp-1},
    {0x1.0c0a780000000p-1f, -0x1.1e810c0000000p-61f, 0x1.4b5bd75d6e276p-1},
    {0x1.0af2f80000000p-1f, 0x1.00d4bc0000000p-55f, 0x1.4d72d1fb9fd0bp-1},
    {0x1.09ddba0000000p-1f, 0x1.cdd5de0000000p-57f, 0x1.4f87a4c3026ebp-1},
    {0x1.08cabc0000000p-1f, -0x1.a3ce000000000p-55f, 0x1.519a4a87a3450p-1},
    {0x1.07b9f20000000p-1f, 0x1.dceeb00000000p-56f, 0x1.53aad18999b82p-1},
    {0x1.06ab5a0000000p-1f, -0x1.9b34360000000p-59f, 0x1.55b934dd40bcep-1},
    {0x1.059eea0000000p-1f, -0x1.dd13a40000000p-55f, 0x1.57c57f416f191p-1},
    {0x1.04949c0000000p-1f, -0x1.c3ca1e0000000p-56f, 0x1.59cfb3dbae887p-1},
    {0x1.038c6c0000000p-1f, 0x1.f8e3640000000p-55f, 0x1.5bd7d20271c77p-1},
    {0x1.0286500000000p-1f, 0x1.d9f46e0000000p-56f, 0x1.5ddde50149924p-1},
    {0x1.0182440000000p-1f, 0x1.5e74960000000p-55f, 0x1.5fe1ec791891ep-1},
    {0x1.0080400000000p-1f, -0x1.436e500000000p-56f, 0x1.61e3f01a46467p-1},
};
// ---- END GENERATED SP TABLE ----
#if PL_SP_FORM == 3
__shared__ SpCell sp_tab[128];
#endif
__device__ __forceinline__ void sp_load_tables(int tid, int nthreads) {
#if PL_SP_FORM == 3
    for (int i = tid; i < 128; i += nthreads) sp_tab[i] = kSpLogTab[i];
    __syncthreads();
#else
    (void)tid;
    (void)nthreads;
#endif
}
#if PL_SP_FORM == 3
__device__ __forceinline__ double pm_log_t(double y) {  // y >= 1, finite
    constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
    const unsigned long long b = (unsigned long long)__double_as_longlong(y);
    const uint32_t hi_w = (uint32_t)(b >> 32);
    const int e = __builtin_amdgcn_frexp_exp(y) - 1;  // y = 2^e m, m in [1, 2)
    const uint32_t j = (hi_w >> 13) & 127u;
    const double m = __longlong_as_double(
        (long long)(((unsigned long long)((hi_w & 0x000FFFFFu) | 0x3FF00000u) << 32) | (b & 0xffffffffull)));
    const SpCell cell = sp_tab[j];
    const double r = __builtin_fma(m, (double)cell.c, -1.0);
    const double r2 = r * r;
    double q = __builtin_fma(-1.0 / 8.0, r, 1.0 / 7.0);
    q = __builtin_fma(q, r, -1.0 / 6.0);
    q = __builtin_fma(q, r, 1.0 / 5.0);
    q = __builtin_fma(q, r, -1.0 / 4.0);
    q = __builtin_fma(q, r, 1.0 / 3.0);
    q = __builtin_fma(q, r, -0.5);
    const double l1 = __builtin_fma(r2, q, r);  // log1p(r)
    const double de = (double)e;
    const double h = __builtin_fma(de, kLn2Hi, cell.hi);
    const double lo = __builtin_fma(de, kLn2Lo, (double)cell.lo) + l1;
    return h + lo;
}
#endif

#if PL_SP_FORM == 0
__device__ __forceinline__ double softplus_pm(double z) { return pm_log(1.0 + pm_exp(z)); }
#elif PL_SP_FORM == 3
__device__ __forceinline__ double softplus_pm(double z) { return pm_log_t(1.0 + pm_exp_e<true>(z)); }
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
// -- two table-driven exponentials (fex_exp below), one quotient (denominator in [2, 4]: a
// reciprocal with PL_RCP_STEPS Newton steps and a residual correction, no scaling needed) and one odd series
// (degree 10 in s^2), ~65 VALU instead of the reference form's three exp and two general logs.  Absolute
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
// The exact f's two exponentials come from a 64-entry table of 2^(j/64) in LDS (fex_tab, loaded by
// fex_load_table() at kernel entry in the exact-f kernels): z = N ln2/64 + r by the 1.5 2^52 shifter
// (N in its low word, no rint / conversion), |r| <= ln2/128, e^r - 1 by degree 5 (round 6; until
// then Cody-Waite to |r| <= ln2/2 and degree 9: 75 -> 65 VALU per f, fewer constants, and with them
// fewer SGPR / VGPR spills in the list kernels -- my_sn SCL default 1.79 -> 1.65 ms,
// profiles/r06w_tab_ab_mysn.txt).  Host accuracy check of both forms against binary128:
// tools/micro/fex_tab_check.cpp (the same largest absolute error; the table form's errors ~10 %
// larger on average, far below the reference's own cancellation error).
__device__ const double kFexTab[64] = {
    0x1.0000000000000p+0, 0x1.02c9a3e778061p+0, 0x1.059b0d3158574p+0, 0x1.0874518759bc8p+0,
    0x1.0b5586cf9890fp+0, 0x1.0e3ec32d3d1a2p+0, 0x1.11301d0125b51p+0, 0x1.1429aaea92de0p+0,
    0x1.172b83c7d517bp+0, 0x1.1a35beb6fcb75p+0, 0x1.1d4873168b9aap+0, 0x1.2063b88628cd6p+0,
    0x1.2387a6e756238p+0, 0x1.26b4565e27cddp+0, 0x1.29e9df51fdee1p+0, 0x1.2d285a6e4030bp+0,
    0x1.306fe0a31b715p+0, 0x1.33c08b26416ffp+0, 0x1.371a7373aa9cbp+0, 0x1.3a7db34e59ff7p+0,
    0x1.3dea64c123422p+0, 0x1.4160a21f72e2ap+0, 0x1.44e086061892dp+0, 0x1.486a2b5c13cd0p+0,
    0x1.4bfdad5362a27p+0, 0x1.4f9b2769d2ca7p+0, 0x1.5342b569d4f82p+0, 0x1.56f4736b527dap+0,
    0x1.5ab07dd485429p+0, 0x1.5e76f15ad2148p+0, 0x1.6247eb03a5585p+0, 0x1.6623882552225p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6dfb23c651a2fp+0, 0x1.71f75e8ec5f74p+0, 0x1.75feb564267c9p+0,
    0x1.7a11473eb0187p+0, 0x1.7e2f336cf4e62p+0, 0x1.82589994cce13p+0, 0x1.868d99b4492edp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8f1ae99157736p+0, 0x1.93737b0cdc5e5p+0, 0x1.97d829fde4e50p+0,
    0x1.9c49182a3f090p+0, 0x1.a0c667b5de565p+0, 0x1.a5503b23e255dp+0, 0x1.a9e6b5579fdbfp+0,
    0x1.ae89f995ad3adp+0, 0x1.b33a2b84f15fbp+0, 0x1.b7f76f2fb5e47p+0, 0x1.bcc1e904bc1d2p+0,
    0x1.c199bdd85529cp+0, 0x1.c67f12e57d14bp+0, 0x1.cb720dcef9069p+0, 0x1.d072d4a07897cp+0,
    0x1.d5818dcfba487p+0, 0x1.da9e603db3285p+0, 0x1.dfc97337b9b5fp+0, 0x1.e502ee78b3ff6p+0,
    0x1.ea4afa2a490dap+0, 0x1.efa1bee615a27p+0, 0x1.f50765b6e4540p+0, 0x1.fa7c1819e90d8p+0,
};
__shared__ double fex_tab[64];
template <bool ON>
__device__ __forceinline__ void fex_load_table(int tid) {  // one wave: lane i loads 2^(i/64)
    if constexpr (ON) {
        fex_tab[tid & 63] = kFexTab[tid & 63];
        __syncthreads();
    }
}
// e^z for z <= 0 (z >= -2000) as 2^k T (1 + q): A = 2^k T (exact), q = e^r - 1
__device__ __forceinline__ void fex_exp(double z, double& A, double& q) {
    constexpr double kInv = 0x1.71547652b82fep+6, kCHi = 0x1.62e42fefa39efp-7, kCLo = 0x1.abc9e3b39803fp-62;
    const double t = __builtin_fma(z, kInv, 0x1.8p52);
    const int n = (int)(uint32_t)(unsigned long long)__double_as_longlong(t);
    const double nd = t - 0x1.8p52;
    double r = __builtin_fma(-nd, kCHi, z);
    r = __builtin_fma(-nd, kCLo, r);
    const double r2 = r * r;
    double h = __builtin_fma(1.0 / 120.0, r, 1.0 / 24.0);
    h = __builtin_fma(h, r, 1.0 / 6.0);
    h = __builtin_fma(h, r, 0.5);
    q = __builtin_fma(r2, h, r);
    A = __builtin_ldexp(fex_tab[n & 63], n >> 6);
}
template <int N>
__device__ __forceinline__ void f_exact_pm_n(const double* x, const double* y, double lmax, double* out) {
    // 2 atanh(s) = 2s + s w R(w), w = s^2 <= 1/9: R of degree 10, the Chebyshev economisation of
    // sum 2/(2i+3) w^i (tail < 2.4e-18)
    constexpr double kS[11] = {
        0.6666666666666666, 0.39999999999999514, 0.28571428571603413, 0.22222222197853667,
        0.18181819920440906, 0.15384543207664578, 0.133351941539121, 0.11734082174871642,
        0.10846687166200544, 0.07485743922141379, 0.1564211337480669};
    double m[N], E[N], G[N];
    uint32_t sg[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        // |clip(v, +-lmax)| = min(|v|, lmax): m and M straight from the magnitudes
        m[i] = vmin_nc(vmin_abs_nc(x[i], y[i]), lmax);
        const double M = vmin_nc(vmax_abs_nc(x[i], y[i]), lmax);
        sg[i] = ((uint32_t)((unsigned long long)__double_as_longlong(x[i]) >> 32) ^
                 (uint32_t)((unsigned long long)__double_as_longlong(y[i]) >> 32)) & 0x80000000u;
        double Ae, qe, Am, qm;
        fex_exp(vmax_nc(m[i] - M, -2000.0), Ae, qe);  // e^-2000 = 0 like e^-745: n stays in int range
        fex_exp(vmax_nc(-2.0 * m[i], -2000.0), Am, qm);
        E[i] = __builtin_fma(Ae, qe, Ae);              // exp(-(M - m))
        G[i] = __builtin_fma(-Am, qm, 1.0 - Am);       // -expm1(-2m); 1 - Am exact (Am in [1/2, 1] or G > 1/2)
    }
    double eg[N], den[N], rc[N], s[N], w[N], R[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        eg[i] = E[i] * G[i];
        den[i] = fma(2.0, E[i], 2.0) - eg[i];  // in [2, 4]
        rc[i] = __builtin_amdgcn_rcp(den[i]);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {  // s = -eg / den: PL_RCP_STEPS Newton steps on the reciprocal, one on the quotient
        double e = fma(-den[i], rc[i], 1.0);
        rc[i] = fma(rc[i], e, rc[i]);
        if (PL_RCP_STEPS > 1) {
            e = fma(-den[i], rc[i], 1.0);
            rc[i] = fma(rc[i], e, rc[i]);
        }
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
        const unsigned long long vb = (unsigned long long)__double_as_longlong(v);
        out[i] = __longlong_as_double((long long)(vb ^ ((unsigned long long)sg[i] << 32)));
    }
}
__device__ __forceinline__ double f_exact_pm(double x, double y, double lmax) {
    double r;
    f_exact_pm_n<1>(&x, &y, lmax, &r);
    return r;
}

}  // namespace pl
