// fex_tab_check.cpp -- host accuracy check of the my_sn list decoder's exact boxplus f
// (softplus.h f_exact_pm_n): the polynomial form (PL_FEX_TAB 0: Cody-Waite to |r| <= ln2/2, degree-9
// exp / expm1) against the table form (PL_FEX_TAB 1: 2^(j/64) from a 64-entry table, |r| <= ln2/128,
// degree 5), both op for op as the device code (fma, the v_rcp_f64 seed emulated with a
// reciprocal rounded to fp32, 2^-24 relative like the device's 2^-24.4), against the exact value
// in binary128 (libquadmath).  Reports the largest absolute error of each form and how often the
// two differ.
//   g++ -O2 -o /tmp/fex_tab_check tools/micro/fex_tab_check.cpp -lquadmath && /tmp/fex_tab_check
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <quadmath.h>

static const double kTab[64] = {
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

static double rcp_seed(double d) { return (double)(1.0f / (float)d); }
static double ldexp_(double x, int k) { return std::ldexp(x, k); }
static uint64_t bits(double d) { uint64_t b; std::memcpy(&b, &d, 8); return b; }

static const double kS[11] = {
    0.6666666666666666, 0.39999999999999514, 0.28571428571603413, 0.22222222197853667,
    0.18181819920440906, 0.15384543207664578, 0.133351941539121, 0.11734082174871642,
    0.10846687166200544, 0.07485743922141379, 0.1564211337480669};
static const double kP[10] = {
    0.5000000000000001, 0.1666666666666667, 0.04166666666662413, 0.008333333333326136,
    0.001388888891721154, 0.00019841269874817515, 2.4801521299750923e-05, 2.75572554044176e-06,
    2.7620086491464514e-07, 2.5105215165649368e-08};

// the tail shared by both forms: t = E G / (1 + E), log1p(-t) = 2 atanh(s)
static double tail(double m, double E, double G, bool neg) {
    const double eg = E * G;
    const double den = std::fma(2.0, E, 2.0) - eg;
    double rc = rcp_seed(den);
    const double e = std::fma(-den, rc, 1.0);
    rc = std::fma(rc, e, rc);
    const double q = eg * rc;
    const double s = -std::fma(rc, std::fma(-den, q, eg), q);
    const double w = s * s;
    double R = kS[10];
    for (int c = 9; c >= 0; --c) R = std::fma(R, w, kS[c]);
    const double v = m + std::fma(s * w, R, s + s);
    return neg ? -v : v;
}

static double f_poly(double x, double y, double lmax) {
    const double kLog2e = 1.4426950408889634;
    const double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
    const double xc = std::fmax(std::fmin(x, lmax), -lmax), yc = std::fmax(std::fmin(y, lmax), -lmax);
    const bool neg = (int64_t)(bits(xc) ^ bits(yc)) < 0;
    const double m = std::fmin(std::fabs(xc), std::fabs(yc));
    const double ze = m - std::fmax(std::fabs(xc), std::fabs(yc));
    const double zm = -2.0 * m;
    const double ke = std::rint(ze * kLog2e), km = std::rint(zm * kLog2e);
    double re = std::fma(-ke, kLn2Hi, ze), rm = std::fma(-km, kLn2Hi, zm);
    re = std::fma(-ke, kLn2Lo, re);
    rm = std::fma(-km, kLn2Lo, rm);
    double pe = kP[9], pm = kP[9];
    for (int c = 8; c >= 0; --c) {
        pe = std::fma(pe, re, kP[c]);
        pm = std::fma(pm, rm, kP[c]);
    }
    const double E = ldexp_(std::fma(re * re, pe, re) + 1.0, (int)ke);
    const double tk = ldexp_(1.0, (int)km);
    const double G = -std::fma(tk, std::fma(rm * rm, pm, rm), tk - 1.0);
    return tail(m, E, G, neg);
}

// table form: z = N ln2/64 + r by the 1.5 2^52 shifter (N in its low word), e^z = 2^(N >> 6)
// T[N & 63] (1 + q), q = e^r - 1 by degree 5
static void exp_tab(double z, double& A, double& q) {
    const double kInv = 0x1.71547652b82fep+6, kCHi = 0x1.62e42fefa39efp-7, kCLo = 0x1.abc9e3b39803fp-62;
    const double t = std::fma(z, kInv, 0x1.8p52);
    const int n = (int)(uint32_t)bits(t);
    const double nd = t - 0x1.8p52;
    double r = std::fma(-nd, kCHi, z);
    r = std::fma(-nd, kCLo, r);
    const double r2 = r * r;
    double h = std::fma(1.0 / 120.0, r, 1.0 / 24.0);
    h = std::fma(h, r, 1.0 / 6.0);
    h = std::fma(h, r, 0.5);
    q = std::fma(r2, h, r);
    A = ldexp_(kTab[n & 63], n >> 6);
}
static double f_tab(double x, double y, double lmax) {
    const double m = std::fmin(std::fmin(std::fabs(x), std::fabs(y)), lmax);
    const double M = std::fmin(std::fmax(std::fabs(x), std::fabs(y)), lmax);
    const bool neg = (int64_t)(bits(x) ^ bits(y)) < 0;
    const double ze = std::fmax(m - M, -2000.0), zm = std::fmax(-2.0 * m, -2000.0);
    double Ae, qe, Am, qm;
    exp_tab(ze, Ae, qe);
    exp_tab(zm, Am, qm);
    const double E = std::fma(Ae, qe, Ae);
    const double G = std::fma(-Am, qm, 1.0 - Am);
    return tail(m, E, G, neg);
}

static __float128 f_true(double x, double y, double lmax) {
    const double xc = std::fmax(std::fmin(x, lmax), -lmax), yc = std::fmax(std::fmin(y, lmax), -lmax);
    const __float128 a = fabsq((__float128)xc), b = fabsq((__float128)yc);
    const __float128 m = a < b ? a : b, M = a < b ? b : a;
    const __float128 E = expq(-(M - m)), G = -expm1q(-2 * m);
    const __float128 v = m + log1pq(-E * G / (1 + E));
    return ((xc < 0) != (yc < 0)) ? -v : v;
}

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next() { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; }
static double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }

int main(int argc, char** argv) {
    const long N = argc > 1 ? atol(argv[1]) : 20000000;
    const double lmaxs[3] = {30.0, 7.5, 300.0};
    for (double lmax : lmaxs) {
        double ep = 0, et = 0, rp = 0, rt = 0;
        long diff = 0, worse = 0, better = 0;
        double up = 0, ut = 0, sp = 0, st = 0;  // max and sum of the errors in ulps of the exact value
        for (long i = 0; i < N; ++i) {
            // magnitudes from 1e-6 to ~2 lmax, both signs, and exact ties / zeros now and then
            const double sx = (next() & 1) ? -1.0 : 1.0, sy = (next() & 1) ? -1.0 : 1.0;
            double x = sx * std::exp(std::log(1e-6) + uni() * (std::log(2.0 * lmax) - std::log(1e-6)));
            double y = sy * std::exp(std::log(1e-6) + uni() * (std::log(2.0 * lmax) - std::log(1e-6)));
            if ((i & 1023) == 0) y = -x;
            if ((i & 4095) == 1) x = 0.0;
            if (i & 2) y = x + sy * uni() * 1e-3;  // near-equal magnitudes
            const __float128 tv = f_true(x, y, lmax);
            const double a = f_poly(x, y, lmax), b = f_tab(x, y, lmax);
            const double da = (double)fabsq((__float128)a - tv), db = (double)fabsq((__float128)b - tv);
            const double mag = (double)fabsq(tv);
            ep = std::fmax(ep, da);
            et = std::fmax(et, db);
            const double ulp = mag > 0 ? std::ldexp(1.0, std::ilogb(mag) - 52) : 0x1p-1074;
            up = std::fmax(up, da / ulp);
            ut = std::fmax(ut, db / ulp);
            sp += da / ulp;
            st += db / ulp;
            if (mag > 0) {
                rp = std::fmax(rp, da / mag);
                rt = std::fmax(rt, db / mag);
            }
            if (a != b) {
                ++diff;
                worse += db > da;
                better += db < da;
            }
        }
        printf("llr_max %g: %ld pairs; max abs error poly %.3g table %.3g; max rel error poly %.3g table %.3g; "
               "results differing %ld (table closer %ld, farther %ld); ulps of the exact value: max poly %.3g table %.3g, "
               "mean poly %.3g table %.3g\n",
               lmax, N, ep, et, rp, rt, diff, better, worse, up, ut, sp / N, st / N);
    }
    return 0;
}
