// Development aid (host): EXHAUSTIVE correct-rounding check of the SC exact f's exp and log forms
// (csrc/exactf.h exp_d / log_d, PL_EXF_LEAN, mirrored op for op in exactf_rounding.cpp) over every
// fp32 argument they can receive: exp on every fp32 x with |x| <= 87 (the f forms |x| <= 86 at
// llr_max <= 43), log on every positive normal fp32.  The reference value is expl / logl (x87
// extended, ~2^-63 relative) rounded to fp32; an argument whose extended value lies within 2^-58 of
// an fp32 rounding boundary is settled by libquadmath's expq / logq instead (113-bit).
//   g++ -O2 -fopenmp -o /tmp/exx tools/micro/exactf_exhaustive.cpp -lquadmath && /tmp/exx
#define EXACTF_NO_MAIN
#include "exactf_rounding.cpp"

#include <omp.h>
#include <quadmath.h>

// fp32 rounding of v (round to nearest even), and whether v is too close to a boundary for its own
// precision to decide it
static float round_checked(long double v, bool& hard) {
    const float f = (float)v;
    const float g = nextafterf(f, v > (long double)f ? INFINITY : -INFINITY);
    const long double mid = ((long double)f + (long double)g) / 2;  // exact: two floats' mean
    hard = fabsl(v - mid) <= fabsl(v) * 0x1p-58L;
    return f;
}
static float exp_true(float x, long& hard_n) {
    bool hard;
    float r = round_checked(expl((long double)x), hard);
    if (hard) {
        ++hard_n;
        r = (float)expq((__float128)x);  // 113-bit, then one rounding to fp32
    }
    return r;
}
static float log_true(float x, long& hard_n) {
    bool hard;
    float r = round_checked(logl((long double)x), hard);
    if (hard) {
        ++hard_n;
        r = (float)logq((__float128)x);
    }
    return r;
}

int main() {
    long bad_e = 0, bad_l = 0, hard_e = 0, hard_l = 0, n_e = 0, n_l = 0;
    uint32_t first_e = 0, first_l = 0;
    // exp: both signs, every bit pattern of |x| <= 87 (0x42ae0000)
#pragma omp parallel for schedule(dynamic, 1 << 16) reduction(+ : bad_e, hard_e, n_e)
    for (int64_t i = 0; i <= 2 * (int64_t)0x42ae0000; ++i) {
        const uint32_t b = i <= 0x42ae0000 ? (uint32_t)i : ((uint32_t)(i - 0x42ae0000) | 0x80000000u);
        float x;
        memcpy(&x, &b, 4);
        ++n_e;
        if (exp_cr(x) != exp_true(x, hard_e)) {
            ++bad_e;
#pragma omp critical
            if (!first_e) first_e = b;
        }
    }
    // log: every positive normal fp32 (0x00800000 .. 0x7f7fffff)
#pragma omp parallel for schedule(dynamic, 1 << 16) reduction(+ : bad_l, hard_l, n_l)
    for (int64_t b = 0x00800000; b <= 0x7f7fffff; ++b) {
        float x;
        const uint32_t bb = (uint32_t)b;
        memcpy(&x, &bb, 4);
        ++n_l;
        if (log_cr(x) != log_true(x, hard_l)) {
            ++bad_l;
#pragma omp critical
            if (!first_l) first_l = bb;
        }
    }
    printf("exp_cr: %ld fp32 arguments (|x| <= 87), %ld misrounded (first 0x%08x), %ld settled in 113 bits\n", n_e,
           bad_e, first_e, hard_e);
    printf("log_cr: %ld fp32 arguments (all positive normals), %ld misrounded (first 0x%08x), %ld settled in 113 bits\n",
           n_l, bad_l, first_l, hard_l);
    return 0;
}
