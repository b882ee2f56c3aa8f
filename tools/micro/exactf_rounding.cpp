// Development aid (host): correct rounding of the table-driven exp_cr / log_cr of csrc/exactf.h
// (PL_EXF_LEAN forms, and the f with e^(x+y) from the product e^x e^y e^d)
// (the same tables, tools/micro/exactf_tables.inc, and the same operation sequence in fp64 with
// fma), against expl / logl rounded to fp32 -- 5e7 arguments per range -- and the exact f built
// from them against f with every transcendental correctly rounded.
//   g++ -O2 -o /tmp/exr tools/micro/exactf_rounding.cpp && /tmp/exr [N]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "exactf_tables.inc"

static double exp_d(float xf) {  // exactf.h exp_d (PL_EXF_LEAN: 2^(j/256) one-part, degree 4)
    const double x = xf;
    const double t = fma(x, kTabInvC1, 0x1.8p52);
    uint64_t tb;
    memcpy(&tb, &t, 8);
    const int n = (int)(uint32_t)tb;
    const double nd = t - 0x1.8p52;
    double r = fma(-nd, kTabC1Hi, x);
    r = fma(-nd, kTabC1Lo, r);
    const double r2 = r * r;
    double h = fma(1.0 / 24.0, r, 1.0 / 6.0);
    h = fma(h, r, 0.5);
    const double q = fma(r2, h, r);
    const double th = kTabExp1[n & 255];
    return ldexp(fma(th, q, th), n >> 8);
}
static double log_d(float xf) {  // exactf.h log_d
    uint32_t b;
    memcpy(&b, &xf, 4);
    const int32_t d = (int32_t)(b - kTabLogBase);
    const int e = d >> 23;
    const uint32_t mb = (uint32_t)d & 0x7FFFFFu;
    const int j = (int)(mb >> 15);
    const uint32_t mbits = mb + kTabLogBase;
    float mf;
    memcpy(&mf, &mbits, 4);
    const double m = mf;
    const double r = fma(m, kTabLogC[j], -1.0);
    const double r2 = r * r;
    double p = fma(-1.0 / 6.0, r, 1.0 / 5.0);
    p = fma(p, r, -0.25);
    p = fma(p, r, 1.0 / 3.0);
    p = fma(p, r, -0.5);
    const double l1 = fma(r2, p, r);
    const double de = e;
    const double hi = fma(de, kTabLn2Hi, kTabLogL[2 * j]);
    const double lo = fma(de, kTabLn2Lo, l1);  // PL_EXF_LEAN: no low part of -ln c_j
    return hi + lo;
}
static float exp_cr(float x) { return (float)exp_d(x); }
static float log_cr(float x) { return (float)log_d(x); }
static float exp_ref(float x) { return (float)expl((long double)x); }
static float log_ref(float x) { return (float)logl((long double)x); }

// exactf.h exp_sum: fp32 e^(fl(xc + yc)) from the fp64 e^xc, e^yc and the Fast2Sum error d
static float exp_sum(double ex, double ey, float xc, float yc) {  // PL_EXF_TWOSUM: the exact error by TwoSum
    volatile float s = xc + yc;
    volatile float bb = s - xc;
    volatile float t = s - bb;
    volatile float e1 = xc - t;
    volatile float e2 = yc - bb;
    volatile float e = e1 + e2;
    const double d = -(double)e;
    return (float)(ex * ey * fma(d, fma(d, 0.5, 1.0), 1.0));
}
// exactf.h f_exact (PL_EXF_LEAN)
static float f_lean(float x, float y, float lmax) {
    const float xc = fminf(fmaxf(x, -lmax), lmax), yc = fminf(fmaxf(y, -lmax), lmax);
    const double ex = exp_d(xc), ey = exp_d(yc);
    volatile float a = 1.0f + exp_sum(ex, ey, xc, yc);
    float o = log_cr(a);
    volatile float b = (float)ex + (float)ey;
    o -= log_cr(b);
    return o;
}

// my_sn dec.py:39-43 with each operation rounded to fp32
template <float (*E)(float), float (*L)(float)>
static float f_exact(float x, float y, float lmax) {
    const float xc = fminf(fmaxf(x, -lmax), lmax), yc = fminf(fmaxf(y, -lmax), lmax);
    volatile float s = xc + yc;
    volatile float a = 1.0f + E(s);
    float o = L(a);
    volatile float b = E(xc) + E(yc);
    o -= L(b);
    return o;
}

static uint64_t st = 88172645463325252ull;
static uint32_t rnd() {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return (uint32_t)(st >> 11);
}
static double uni() { return rnd() / 4294967296.0; }

#ifndef EXACTF_NO_MAIN  // tools/micro/exactf_exhaustive.cpp includes the forms above
int main(int argc, char** argv) {
    const long N = argc > 1 ? atol(argv[1]) : 50000000;
    long be = 0, bl = 0, bl1 = 0, bf = 0, bs = 0;
    for (long i = 0; i < N; ++i) {
        // exp: |x| <= 86 (xc + yc at llr_max 43), <= 4, <= 0.01
        const float x = (float)((uni() * 2 - 1) * (i % 3 == 0 ? 86.0 : (i % 3 == 1 ? 4.0 : 0.01)));
        if (exp_cr(x) != exp_ref(x)) ++be;
        // log: any normal positive fp32
        uint32_t bb = rnd() & 0x7fffffff;
        float y;
        memcpy(&y, &bb, 4);
        if (!(y >= 1.17549435e-38f) || isinf(y) || isnan(y)) y = 1.0f + (float)uni();
        if (log_cr(y) != log_ref(y)) ++bl;
        // log of 1 + e and of e1 + e2 in the f's ranges: [1, 2) densely, and near 1
        const float z = i & 1 ? 1.0f + (float)uni() : 1.0f + (float)((uni() * 2 - 1) * 0.01);
        if (log_cr(z) != log_ref(z)) ++bl1;
        // the whole f on N(0, 8^2)-ish inputs at llr_max 30
        const float fx = (float)((uni() + uni() + uni() - 1.5) * 16.0), fy = (float)((uni() + uni() + uni() - 1.5) * 16.0);
        if (f_lean(fx, fy, 30.0f) != f_exact<exp_ref, log_ref>(fx, fy, 30.0f)) ++bf;
        // e^(x + y) by the product, over the whole exp range with one input tiny or zero now and then
        const float px = (float)((uni() * 2 - 1) * 43.0), py = i % 7 == 0 ? (float)((uni() * 2 - 1) * 1e-9) : (float)((uni() * 2 - 1) * 43.0);
        if (exp_sum(exp_d(px), exp_d(py), px, py) != exp_ref(px + py)) ++bs;
    }
    printf("misrounded of %ld each: exp %ld, log (all normal) %ld, log ([1,2) and 1 +- 0.01) %ld; e^(x+y) by the product %ld; f differing %ld\n",
           N, be, bl, bl1, bs, bf);
    return 0;
}
#endif
