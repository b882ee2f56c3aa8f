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
// exp_cr / log_cr evaluate in fp64 and round once to fp32; their fp64 error (~2^-53 relative)
// leaves a wrong fp32 rounding only for arguments within ~2^-28 ulp of a rounding boundary (none
// of 5e7 random arguments each, tools/micro/exactf_rounding.c).  Both are table-driven (round 4):
// the tables live in LDS (load_tables() at kernel entry), exp needs a degree-5 polynomial and no
// range reduction by rint/cvt, log needs no division (the reciprocal + Newton steps of the round-3
// atanh form were ~40 % of an f).  Range: exp_cr for |x| <= 87, log_cr for normal x > 0; plans
// with llr_max > 43 take the full-range forms (exp_cr_wide / log_cr_wide) instead.
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

// The round-3 forms (no tables; the full-range path below keeps them).
// exp(x) for fp32 x, |x| <= 87: x = k ln2 + r (|r| <= ln2/2, two-part ln2), degree-10 polynomial
// in fp64, rounded to fp32, then scaled by 2^k exactly.
__device__ __forceinline__ float exp_poly(float xf) {
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
__device__ __forceinline__ float log_poly(float xf) {
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

// ---- BEGIN GENERATED TABLES (tools/gen_exactf_tables.py) ----
constexpr double kTabInvC = 0x1.71547652b82fep+7;  // 128 / ln2
constexpr double kTabCHi = 0x1.62e42fefa0000p-8, kTabCLo = 0x1.cf79abc9e3b3ap-47;  // ln2 / 128 = hi + lo
constexpr double kTabLn2Hi = 0x1.62e42fefa39efp-1, kTabLn2Lo = 0x1.abc9e3b39803fp-56;
constexpr uint32_t kTabLogBase = 0x3F3504F3u;  // fp32 bits of sqrt(1/2)
// 2^(j/128) = kTabExp[2j] + kTabExp[2j+1]
__device__ const double kTabExp[256] = {
    0x1.0000000000000p+0, 0x0.0p+0, 0x1.0163da9fb3335p+0, 0x1.b61299ab8cdb7p-54,
    0x1.02c9a3e778061p+0, -0x1.19083535b085dp-56, 0x1.04315e86e7f85p+0, -0x1.0a31c1977c96ep-54,
    0x1.059b0d3158574p+0, 0x1.d73e2a475b465p-55, 0x1.0706b29ddf6dep+0, -0x1.c91dfe2b13c27p-55,
    0x1.0874518759bc8p+0, 0x1.186be4bb284ffp-57, 0x1.09e3ecac6f383p+0, 0x1.1487818316136p-54,
    0x1.0b5586cf9890fp+0, 0x1.8a62e4adc610bp-54, 0x1.0cc922b7247f7p+0, 0x1.01edc16e24f71p-54,
    0x1.0e3ec32d3d1a2p+0, 0x1.03a1727c57b53p-59, 0x1.0fb66affed31bp+0, -0x1.b9bedc44ebd7bp-57,
    0x1.11301d0125b51p+0, -0x1.6c51039449b3ap-54, 0x1.12abdc06c31ccp+0, -0x1.1b514b36ca5c7p-58,
    0x1.1429aaea92de0p+0, -0x1.32fbf9af1369ep-54, 0x1.15a98c8a58e51p+0, 0x1.2406ab9eeab0ap-55,
    0x1.172b83c7d517bp+0, -0x1.19041b9d78a76p-55, 0x1.18af9388c8deap+0, -0x1.11023d1970f6cp-54,
    0x1.1a35beb6fcb75p+0, 0x1.e5b4c7b4968e4p-55, 0x1.1bbe084045cd4p+0, -0x1.95386352ef607p-54,
    0x1.1d4873168b9aap+0, 0x1.e016e00a2643cp-54, 0x1.1ed5022fcd91dp+0, -0x1.1df98027bb78cp-54,
    0x1.2063b88628cd6p+0, 0x1.dc775814a8495p-55, 0x1.21f49917ddc96p+0, 0x1.2a97e9494a5eep-55,
    0x1.2387a6e756238p+0, 0x1.9b07eb6c70573p-54, 0x1.251ce4fb2a63fp+0, 0x1.ac155bef4f4a4p-55,
    0x1.26b4565e27cddp+0, 0x1.2bd339940e9d9p-55, 0x1.284dfe1f56381p+0, -0x1.a4c3a8c3f0d7ep-54,
    0x1.29e9df51fdee1p+0, 0x1.612e8afad1255p-55, 0x1.2b87fd0dad990p+0, -0x1.10adcd6381aa4p-59,
    0x1.2d285a6e4030bp+0, 0x1.0024754db41d5p-54, 0x1.2ecafa93e2f56p+0, 0x1.1ca0f45d52383p-56,
    0x1.306fe0a31b715p+0, 0x1.6f46ad23182e4p-55, 0x1.32170fc4cd831p+0, 0x1.a9ce78e18047cp-55,
    0x1.33c08b26416ffp+0, 0x1.32721843659a6p-54, 0x1.356c55f929ff1p+0, -0x1.b5cee5c4e4628p-55,
    0x1.371a7373aa9cbp+0, -0x1.63aeabf42eae2p-54, 0x1.38cae6d05d866p+0, -0x1.e958d3c9904bdp-54,
    0x1.3a7db34e59ff7p+0, -0x1.5e436d661f5e3p-56, 0x1.3c32dc313a8e5p+0, -0x1.efff8375d29c3p-54,
    0x1.3dea64c123422p+0, 0x1.ada0911f09ebcp-55, 0x1.3fa4504ac801cp+0, -0x1.7d023f956f9f3p-54,
    0x1.4160a21f72e2ap+0, -0x1.ef3691c309278p-58, 0x1.431f5d950a897p+0, -0x1.1c7dde35f7999p-55,
    0x1.44e086061892dp+0, 0x1.89b7a04ef80d0p-59, 0x1.46a41ed1d0057p+0, 0x1.c944bd1648a76p-54,
    0x1.486a2b5c13cd0p+0, 0x1.3c1a3b69062f0p-56, 0x1.4a32af0d7d3dep+0, 0x1.9cb62f3d1be56p-54,
    0x1.4bfdad5362a27p+0, 0x1.d4397afec42e2p-56, 0x1.4dcb299fddd0dp+0, 0x1.8ecdbbc6a7833p-54,
    0x1.4f9b2769d2ca7p+0, -0x1.4b309d25957e3p-54, 0x1.516daa2cf6642p+0, -0x1.f768569bd93efp-55,
    0x1.5342b569d4f82p+0, -0x1.07abe1db13cadp-55, 0x1.551a4ca5d920fp+0, -0x1.d689cefede59bp-55,
    0x1.56f4736b527dap+0, 0x1.9bb2c011d93adp-54, 0x1.58d12d497c7fdp+0, 0x1.295e15b9a1de8p-55,
    0x1.5ab07dd485429p+0, 0x1.6324c054647adp-54, 0x1.5c9268a5946b7p+0, 0x1.c4b1b816986a2p-60,
    0x1.5e76f15ad2148p+0, 0x1.ba6f93080e65ep-54, 0x1.605e1b976dc09p+0, -0x1.3e2429b56de47p-54,
    0x1.6247eb03a5585p+0, -0x1.383c17e40b497p-54, 0x1.6434634ccc320p+0, -0x1.c483c759d8933p-55,
    0x1.6623882552225p+0, -0x1.bb60987591c34p-54, 0x1.68155d44ca973p+0, 0x1.038ae44f73e65p-57,
    0x1.6a09e667f3bcdp+0, -0x1.bdd3413b26456p-54, 0x1.6c012750bdabfp+0, -0x1.2895667ff0b0dp-56,
    0x1.6dfb23c651a2fp+0, -0x1.bbe3a683c88abp-57, 0x1.6ff7df9519484p+0, -0x1.83c0f25860ef6p-55,
    0x1.71f75e8ec5f74p+0, -0x1.16e4786887a99p-55, 0x1.73f9a48a58174p+0, -0x1.0a8d96c65d53cp-54,
    0x1.75feb564267c9p+0, -0x1.0245957316dd3p-54, 0x1.780694fde5d3fp+0, 0x1.866b80a02162dp-54,
    0x1.7a11473eb0187p+0, -0x1.41577ee04992fp-55, 0x1.7c1ed0130c132p+0, 0x1.f124cd1164dd6p-54,
    0x1.7e2f336cf4e62p+0, 0x1.05d02ba15797ep-56, 0x1.80427543e1a12p+0, -0x1.27c86626d972bp-54,
    0x1.82589994cce13p+0, -0x1.d4c1dd41532d8p-54, 0x1.8471a4623c7adp+0, -0x1.8d684a341cdfbp-55,
    0x1.868d99b4492edp+0, -0x1.fc6f89bd4f6bap-54, 0x1.88ac7d98a6699p+0, 0x1.994c2f37cb53ap-54,
    0x1.8ace5422aa0dbp+0, 0x1.6e9f156864b27p-54, 0x1.8cf3216b5448cp+0, -0x1.0d55e32e9e3aap-56,
    0x1.8f1ae99157736p+0, 0x1.5cc13a2e3976cp-55, 0x1.9145b0b91ffc6p+0, -0x1.dd6792e582524p-54,
    0x1.93737b0cdc5e5p+0, -0x1.75fc781b57ebcp-57, 0x1.95a44cbc8520fp+0, -0x1.64b7c96a5f039p-56,
    0x1.97d829fde4e50p+0, -0x1.d185b7c1b85d1p-54, 0x1.9a0f170ca07bap+0, -0x1.173bd91cee632p-54,
    0x1.9c49182a3f090p+0, 0x1.c7c46b071f2bep-56, 0x1.9e86319e32323p+0, 0x1.824ca78e64c6ep-56,
    0x1.a0c667b5de565p+0, -0x1.359495d1cd533p-54, 0x1.a309bec4a2d33p+0, 0x1.6305c7ddc36abp-54,
    0x1.a5503b23e255dp+0, -0x1.d2f6edb8d41e1p-54, 0x1.a799e1330b358p+0, 0x1.bcb7ecac563c7p-54,
    0x1.a9e6b5579fdbfp+0, 0x1.0fac90ef7fd31p-54, 0x1.ac36bbfd3f37ap+0, -0x1.f9234cae76cd0p-55,
    0x1.ae89f995ad3adp+0, 0x1.7a1cd345dcc81p-54, 0x1.b0e07298db666p+0, -0x1.bdef54c80e425p-54,
    0x1.b33a2b84f15fbp+0, -0x1.2805e3084d708p-57, 0x1.b59728de5593ap+0, -0x1.c71dfbbba6de3p-54,
    0x1.b7f76f2fb5e47p+0, -0x1.5584f7e54ac3bp-56, 0x1.ba5b030a1064ap+0, -0x1.efcd30e54292ep-54,
    0x1.bcc1e904bc1d2p+0, 0x1.23dd07a2d9e84p-55, 0x1.bf2c25bd71e09p+0, -0x1.efdca3f6b9c73p-54,
    0x1.c199bdd85529cp+0, 0x1.11065895048ddp-55, 0x1.c40ab5fffd07ap+0, 0x1.b4537e083c60ap-54,
    0x1.c67f12e57d14bp+0, 0x1.2884dff483cadp-54, 0x1.c8f6d9406e7b5p+0, 0x1.1acbc48805c44p-56,
    0x1.cb720dcef9069p+0, 0x1.503cbd1e949dbp-56, 0x1.cdf0b555dc3fap+0, -0x1.dd83b53829d72p-55,
    0x1.d072d4a07897cp+0, -0x1.cbc3743797a9cp-54, 0x1.d2f87080d89f2p+0, -0x1.d487b719d8578p-54,
    0x1.d5818dcfba487p+0, 0x1.2ed02d75b3707p-55, 0x1.d80e316c98398p+0, -0x1.11ec18beddfe8p-54,
    0x1.da9e603db3285p+0, 0x1.c2300696db532p-54, 0x1.dd321f301b460p+0, 0x1.2da5778f018c3p-54,
    0x1.dfc97337b9b5fp+0, -0x1.1a5cd4f184b5cp-54, 0x1.e264614f5a129p+0, -0x1.7b627817a1496p-54,
    0x1.e502ee78b3ff6p+0, 0x1.39e8980a9cc8fp-55, 0x1.e7a51fbc74c83p+0, 0x1.2d522ca0c8de2p-54,
    0x1.ea4afa2a490dap+0, -0x1.e9c23179c2893p-54, 0x1.ecf482d8e67f1p+0, -0x1.c93f3b411ad8cp-54,
    0x1.efa1bee615a27p+0, 0x1.dc7f486a4b6b0p-54, 0x1.f252b376bba97p+0, 0x1.3a1a5bf0d8e43p-54,
    0x1.f50765b6e4540p+0, 0x1.9d3e12dd8a18bp-54, 0x1.f7bfdad9cbe14p+0, -0x1.dbb12d006350ap-54,
    0x1.fa7c1819e90d8p+0, 0x1.74853f3a5931ep-55, 0x1.fd3c22b8f71f1p+0, 0x1.2eb74966579e7p-57,
};
constexpr double kTabInvC1 = 0x1.71547652b82fep+8;  // 256 / ln2
constexpr double kTabC1Hi = 0x1.62e42fefa0000p-9, kTabC1Lo = 0x1.cf79abc9e3b3ap-48;  // ln2 / 256 = hi + lo
// 2^(j/256), one fp64 value each (the lean exp)
__device__ const double kTabExp1[256] = {
    0x1.0000000000000p+0, 0x1.00b1afa5abcbfp+0, 0x1.0163da9fb3335p+0, 0x1.02168143b0281p+0,
    0x1.02c9a3e778061p+0, 0x1.037d42e11bbccp+0, 0x1.04315e86e7f85p+0, 0x1.04e5f72f654b1p+0,
    0x1.059b0d3158574p+0, 0x1.0650a0e3c1f89p+0, 0x1.0706b29ddf6dep+0, 0x1.07bd42b72a836p+0,
    0x1.0874518759bc8p+0, 0x1.092bdf66607e0p+0, 0x1.09e3ecac6f383p+0, 0x1.0a9c79b1f3919p+0,
    0x1.0b5586cf9890fp+0, 0x1.0c0f145e46c85p+0, 0x1.0cc922b7247f7p+0, 0x1.0d83b23395decp+0,
    0x1.0e3ec32d3d1a2p+0, 0x1.0efa55fdfa9c5p+0, 0x1.0fb66affed31bp+0, 0x1.1073028d7233ep+0,
    0x1.11301d0125b51p+0, 0x1.11edbab5e2ab6p+0, 0x1.12abdc06c31ccp+0, 0x1.136a814f204abp+0,
    0x1.1429aaea92de0p+0, 0x1.14e95934f312ep+0, 0x1.15a98c8a58e51p+0, 0x1.166a45471c3c2p+0,
    0x1.172b83c7d517bp+0, 0x1.17ed48695bbc0p+0, 0x1.18af9388c8deap+0, 0x1.1972658375d2fp+0,
    0x1.1a35beb6fcb75p+0, 0x1.1af99f8138a1cp+0, 0x1.1bbe084045cd4p+0, 0x1.1c82f95281c6bp+0,
    0x1.1d4873168b9aap+0, 0x1.1e0e75eb44027p+0, 0x1.1ed5022fcd91dp+0, 0x1.1f9c18438ce4dp+0,
    0x1.2063b88628cd6p+0, 0x1.212be3578a819p+0, 0x1.21f49917ddc96p+0, 0x1.22bdda27912d1p+0,
    0x1.2387a6e756238p+0, 0x1.2451ffb82140ap+0, 0x1.251ce4fb2a63fp+0, 0x1.25e85711ece75p+0,
    0x1.26b4565e27cddp+0, 0x1.2780e341ddf29p+0, 0x1.284dfe1f56381p+0, 0x1.291ba7591bb70p+0,
    0x1.29e9df51fdee1p+0, 0x1.2ab8a66d10f13p+0, 0x1.2b87fd0dad990p+0, 0x1.2c57e39771b2fp+0,
    0x1.2d285a6e4030bp+0, 0x1.2df961f641589p+0, 0x1.2ecafa93e2f56p+0, 0x1.2f9d24abd886bp+0,
    0x1.306fe0a31b715p+0, 0x1.31432edeeb2fdp+0, 0x1.32170fc4cd831p+0, 0x1.32eb83ba8ea32p+0,
    0x1.33c08b26416ffp+0, 0x1.3496266e3fa2dp+0, 0x1.356c55f929ff1p+0, 0x1.36431a2de883bp+0,
    0x1.371a7373aa9cbp+0, 0x1.37f26231e754ap+0, 0x1.38cae6d05d866p+0, 0x1.39a401b7140efp+0,
    0x1.3a7db34e59ff7p+0, 0x1.3b57fbfec6cf4p+0, 0x1.3c32dc313a8e5p+0, 0x1.3d0e544ede173p+0,
    0x1.3dea64c123422p+0, 0x1.3ec70df1c5175p+0, 0x1.3fa4504ac801cp+0, 0x1.40822c367a024p+0,
    0x1.4160a21f72e2ap+0, 0x1.423fb2709468ap+0, 0x1.431f5d950a897p+0, 0x1.43ffa3f84b9d4p+0,
    0x1.44e086061892dp+0, 0x1.45c2042a7d232p+0, 0x1.46a41ed1d0057p+0, 0x1.4786d668b3237p+0,
    0x1.486a2b5c13cd0p+0, 0x1.494e1e192aed2p+0, 0x1.4a32af0d7d3dep+0, 0x1.4b17dea6db7d7p+0,
    0x1.4bfdad5362a27p+0, 0x1.4ce41b817c114p+0, 0x1.4dcb299fddd0dp+0, 0x1.4eb2d81d8abffp+0,
    0x1.4f9b2769d2ca7p+0, 0x1.508417f4531eep+0, 0x1.516daa2cf6642p+0, 0x1.5257de83f4eefp+0,
    0x1.5342b569d4f82p+0, 0x1.542e2f4f6ad27p+0, 0x1.551a4ca5d920fp+0, 0x1.56070dde910d2p+0,
    0x1.56f4736b527dap+0, 0x1.57e27dbe2c4cfp+0, 0x1.58d12d497c7fdp+0, 0x1.59c0827ff07ccp+0,
    0x1.5ab07dd485429p+0, 0x1.5ba11fba87a03p+0, 0x1.5c9268a5946b7p+0, 0x1.5d84590998b93p+0,
    0x1.5e76f15ad2148p+0, 0x1.5f6a320dceb71p+0, 0x1.605e1b976dc09p+0, 0x1.6152ae6cdf6f4p+0,
    0x1.6247eb03a5585p+0, 0x1.633dd1d1929fdp+0, 0x1.6434634ccc320p+0, 0x1.652b9febc8fb7p+0,
    0x1.6623882552225p+0, 0x1.671c1c70833f6p+0, 0x1.68155d44ca973p+0, 0x1.690f4b19e9538p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6b052fa75173ep+0, 0x1.6c012750bdabfp+0, 0x1.6cfdcddd47645p+0,
    0x1.6dfb23c651a2fp+0, 0x1.6ef9298593ae5p+0, 0x1.6ff7df9519484p+0, 0x1.70f7466f42e87p+0,
    0x1.71f75e8ec5f74p+0, 0x1.72f8286ead08ap+0, 0x1.73f9a48a58174p+0, 0x1.74fbd35d7cbfdp+0,
    0x1.75feb564267c9p+0, 0x1.77024b1ab6e09p+0, 0x1.780694fde5d3fp+0, 0x1.790b938ac1cf6p+0,
    0x1.7a11473eb0187p+0, 0x1.7b17b0976cfdbp+0, 0x1.7c1ed0130c132p+0, 0x1.7d26a62ff86f0p+0,
    0x1.7e2f336cf4e62p+0, 0x1.7f3878491c491p+0, 0x1.80427543e1a12p+0, 0x1.814d2add106d9p+0,
    0x1.82589994cce13p+0, 0x1.8364c1eb941f7p+0, 0x1.8471a4623c7adp+0, 0x1.857f4179f5b21p+0,
    0x1.868d99b4492edp+0, 0x1.879cad931a436p+0, 0x1.88ac7d98a6699p+0, 0x1.89bd0a478580fp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8be05bad61778p+0, 0x1.8cf3216b5448cp+0, 0x1.8e06a5e0866d9p+0,
    0x1.8f1ae99157736p+0, 0x1.902fed0282c8ap+0, 0x1.9145b0b91ffc6p+0, 0x1.925c353aa2fe2p+0,
    0x1.93737b0cdc5e5p+0, 0x1.948b82b5f98e5p+0, 0x1.95a44cbc8520fp+0, 0x1.96bdd9a7670b3p+0,
    0x1.97d829fde4e50p+0, 0x1.98f33e47a22a2p+0, 0x1.9a0f170ca07bap+0, 0x1.9b2bb4d53fe0dp+0,
    0x1.9c49182a3f090p+0, 0x1.9d674194bb8d5p+0, 0x1.9e86319e32323p+0, 0x1.9fa5e8d07f29ep+0,
    0x1.a0c667b5de565p+0, 0x1.a1e7aed8eb8bbp+0, 0x1.a309bec4a2d33p+0, 0x1.a42c980460ad8p+0,
    0x1.a5503b23e255dp+0, 0x1.a674a8af46052p+0, 0x1.a799e1330b358p+0, 0x1.a8bfe53c12e59p+0,
    0x1.a9e6b5579fdbfp+0, 0x1.ab0e521356ebap+0, 0x1.ac36bbfd3f37ap+0, 0x1.ad5ff3a3c2774p+0,
    0x1.ae89f995ad3adp+0, 0x1.afb4ce622f2ffp+0, 0x1.b0e07298db666p+0, 0x1.b20ce6c9a8952p+0,
    0x1.b33a2b84f15fbp+0, 0x1.b468415b749b1p+0, 0x1.b59728de5593ap+0, 0x1.b6c6e29f1c52ap+0,
    0x1.b7f76f2fb5e47p+0, 0x1.b928cf22749e4p+0, 0x1.ba5b030a1064ap+0, 0x1.bb8e0b79a6f1fp+0,
    0x1.bcc1e904bc1d2p+0, 0x1.bdf69c3f3a207p+0, 0x1.bf2c25bd71e09p+0, 0x1.c06286141b33dp+0,
    0x1.c199bdd85529cp+0, 0x1.c2d1cd9fa652cp+0, 0x1.c40ab5fffd07ap+0, 0x1.c544778fafb22p+0,
    0x1.c67f12e57d14bp+0, 0x1.c7ba88988c933p+0, 0x1.c8f6d9406e7b5p+0, 0x1.ca3405751c4dbp+0,
    0x1.cb720dcef9069p+0, 0x1.ccb0f2e6d1675p+0, 0x1.cdf0b555dc3fap+0, 0x1.cf3155b5bab74p+0,
    0x1.d072d4a07897cp+0, 0x1.d1b532b08c968p+0, 0x1.d2f87080d89f2p+0, 0x1.d43c8eacaa1d6p+0,
    0x1.d5818dcfba487p+0, 0x1.d6c76e862e6d3p+0, 0x1.d80e316c98398p+0, 0x1.d955d71ff6075p+0,
    0x1.da9e603db3285p+0, 0x1.dbe7cd63a8315p+0, 0x1.dd321f301b460p+0, 0x1.de7d5641c0658p+0,
    0x1.dfc97337b9b5fp+0, 0x1.e11676b197d17p+0, 0x1.e264614f5a129p+0, 0x1.e3b333b16ee12p+0,
    0x1.e502ee78b3ff6p+0, 0x1.e653924676d76p+0, 0x1.e7a51fbc74c83p+0, 0x1.e8f7977cdb740p+0,
    0x1.ea4afa2a490dap+0, 0x1.eb9f4867cca6ep+0, 0x1.ecf482d8e67f1p+0, 0x1.ee4aaa2188510p+0,
    0x1.efa1bee615a27p+0, 0x1.f0f9c1cb6412ap+0, 0x1.f252b376bba97p+0, 0x1.f3ac948dd7274p+0,
    0x1.f50765b6e4540p+0, 0x1.f6632798844f8p+0, 0x1.f7bfdad9cbe14p+0, 0x1.f91d802243c89p+0,
    0x1.fa7c1819e90d8p+0, 0x1.fbdba3692d514p+0, 0x1.fd3c22b8f71f1p+0, 0x1.fe9d96b2a23d9p+0,
};
// c_j (fp32 values) of the log cells
__device__ const double kTabLogC[256] = {
    0x1.698a160000000p+0, 0x1.688b7e0000000p+0, 0x1.678e4c0000000p+0, 0x1.66927c0000000p+0,
    0x1.65980c0000000p+0, 0x1.649efa0000000p+0, 0x1.63a7400000000p+0, 0x1.62b0e00000000p+0,
    0x1.61bbd20000000p+0, 0x1.60c8180000000p+0, 0x1.5fd5aa0000000p+0, 0x1.5ee48a0000000p+0,
    0x1.5df4b40000000p+0, 0x1.5d06240000000p+0, 0x1.5c18da0000000p+0, 0x1.5b2cd00000000p+0,
    0x1.5a42060000000p+0, 0x1.5958780000000p+0, 0x1.5870260000000p+0, 0x1.57890a0000000p+0,
    0x1.56a3240000000p+0, 0x1.55be720000000p+0, 0x1.54daee0000000p+0, 0x1.53f89a0000000p+0,
    0x1.5317720000000p+0, 0x1.5237720000000p+0, 0x1.51589a0000000p+0, 0x1.507ae80000000p+0,
    0x1.4f9e560000000p+0, 0x1.4ec2e60000000p+0, 0x1.4de8940000000p+0, 0x1.4d0f600000000p+0,
    0x1.4c37440000000p+0, 0x1.4b603e0000000p+0, 0x1.4a8a500000000p+0, 0x1.49b5760000000p+0,
    0x1.48e1ac0000000p+0, 0x1.480ef20000000p+0, 0x1.473d440000000p+0, 0x1.466ca40000000p+0,
    0x1.459d0c0000000p+0, 0x1.44ce7a0000000p+0, 0x1.4400f00000000p+0, 0x1.4334680000000p+0,
    0x1.4268e20000000p+0, 0x1.419e5a0000000p+0, 0x1.40d4d20000000p+0, 0x1.400c460000000p+0,
    0x1.3f44b20000000p+0, 0x1.3e7e180000000p+0, 0x1.3db8740000000p+0, 0x1.3cf3c60000000p+0,
    0x1.3c300a0000000p+0, 0x1.3b6d3e0000000p+0, 0x1.3aab620000000p+0, 0x1.39ea760000000p+0,
    0x1.392a740000000p+0, 0x1.386b5c0000000p+0, 0x1.37ad2c0000000p+0, 0x1.36efe40000000p+0,
    0x1.3633820000000p+0, 0x1.3578040000000p+0, 0x1.34bd660000000p+0, 0x1.3403aa0000000p+0,
    0x1.334ace0000000p+0, 0x1.3292ce0000000p+0, 0x1.31dbaa0000000p+0, 0x1.3125600000000p+0,
    0x1.306ff00000000p+0, 0x1.2fbb560000000p+0, 0x1.2f07920000000p+0, 0x1.2e54a20000000p+0,
    0x1.2da2860000000p+0, 0x1.2cf13a0000000p+0, 0x1.2c40be0000000p+0, 0x1.2b91120000000p+0,
    0x1.2ae2320000000p+0, 0x1.2a341e0000000p+0, 0x1.2986d40000000p+0, 0x1.28da540000000p+0,
    0x1.282e9a0000000p+0, 0x1.2783a80000000p+0, 0x1.26d97a0000000p+0, 0x1.26300e0000000p+0,
    0x1.2587660000000p+0, 0x1.24df7e0000000p+0, 0x1.2438580000000p+0, 0x1.2391ee0000000p+0,
    0x1.22ec420000000p+0, 0x1.2247520000000p+0, 0x1.21a31c0000000p+0, 0x1.20ffa00000000p+0,
    0x1.205cda0000000p+0, 0x1.1fbace0000000p+0, 0x1.1f19760000000p+0, 0x1.1e78d40000000p+0,
    0x1.1dd8e40000000p+0, 0x1.1d39a60000000p+0, 0x1.1c9b1a0000000p+0, 0x1.1bfd3e0000000p+0,
    0x1.1b60100000000p+0, 0x1.1ac3900000000p+0, 0x1.1a27bc0000000p+0, 0x1.198c940000000p+0,
    0x1.18f2160000000p+0, 0x1.1858400000000p+0, 0x1.17bf140000000p+0, 0x1.17268e0000000p+0,
    0x1.168eae0000000p+0, 0x1.15f7740000000p+0, 0x1.1560dc0000000p+0, 0x1.14cae80000000p+0,
    0x1.1435960000000p+0, 0x1.13a0e40000000p+0, 0x1.130cd20000000p+0, 0x1.1279600000000p+0,
    0x1.11e68a0000000p+0, 0x1.1154520000000p+0, 0x1.10c2b60000000p+0, 0x1.1031b40000000p+0,
    0x1.0fa14c0000000p+0, 0x1.0f117c0000000p+0, 0x1.0e82440000000p+0, 0x1.0df3a40000000p+0,
    0x1.0d659a0000000p+0, 0x1.0cd8260000000p+0, 0x1.0c4b460000000p+0, 0x1.0bbef80000000p+0,
    0x1.0b333c0000000p+0, 0x1.0aa8140000000p+0, 0x1.0a1d7a0000000p+0, 0x1.0993720000000p+0,
    0x1.0909f80000000p+0, 0x1.08810c0000000p+0, 0x1.07f8ae0000000p+0, 0x1.0770da0000000p+0,
    0x1.06e9940000000p+0, 0x1.0662d80000000p+0, 0x1.05dca60000000p+0, 0x1.0556fc0000000p+0,
    0x1.04d1da0000000p+0, 0x1.044d400000000p+0, 0x1.03c92e0000000p+0, 0x1.0345a00000000p+0,
    0x1.02c2960000000p+0, 0x1.0240120000000p+0, 0x1.01be120000000p+0, 0x1.013c940000000p+0,
    0x1.00bb960000000p+0, 0x1.0000000000000p+0, 0x1.feecca0000000p-1, 0x1.fcf0ea0000000p-1,
    0x1.faf8fa0000000p-1, 0x1.f904ea0000000p-1, 0x1.f714b20000000p-1, 0x1.f528440000000p-1,
    0x1.f33f960000000p-1, 0x1.f15aa00000000p-1, 0x1.ef79520000000p-1, 0x1.ed9ba60000000p-1,
    0x1.ebc18e0000000p-1, 0x1.e9eb020000000p-1, 0x1.e817f60000000p-1, 0x1.e648640000000p-1,
    0x1.e47c3c0000000p-1, 0x1.e2b37a0000000p-1, 0x1.e0ee120000000p-1, 0x1.df2bfa0000000p-1,
    0x1.dd6d280000000p-1, 0x1.dbb1960000000p-1, 0x1.d9f93a0000000p-1, 0x1.d844080000000p-1,
    0x1.d691fc0000000p-1, 0x1.d4e30a0000000p-1, 0x1.d3372a0000000p-1, 0x1.d18e540000000p-1,
    0x1.cfe8800000000p-1, 0x1.ce45a60000000p-1, 0x1.cca5be0000000p-1, 0x1.cb08c00000000p-1,
    0x1.c96ea40000000p-1, 0x1.c7d7620000000p-1, 0x1.c642f20000000p-1, 0x1.c4b14e0000000p-1,
    0x1.c3226c0000000p-1, 0x1.c196480000000p-1, 0x1.c00cda0000000p-1, 0x1.be861a0000000p-1,
    0x1.bd02000000000p-1, 0x1.bb80860000000p-1, 0x1.ba01a80000000p-1, 0x1.b8855c0000000p-1,
    0x1.b70b9a0000000p-1, 0x1.b594600000000p-1, 0x1.b41fa40000000p-1, 0x1.b2ad620000000p-1,
    0x1.b13d920000000p-1, 0x1.afd02e0000000p-1, 0x1.ae65320000000p-1, 0x1.acfc940000000p-1,
    0x1.ab96520000000p-1, 0x1.aa32640000000p-1, 0x1.a8d0c40000000p-1, 0x1.a7716e0000000p-1,
    0x1.a6145a0000000p-1, 0x1.a4b9840000000p-1, 0x1.a360e80000000p-1, 0x1.a20a7c0000000p-1,
    0x1.a0b6400000000p-1, 0x1.9f642a0000000p-1, 0x1.9e14380000000p-1, 0x1.9cc6640000000p-1,
    0x1.9b7aa60000000p-1, 0x1.9a30fe0000000p-1, 0x1.98e9640000000p-1, 0x1.97a3d40000000p-1,
    0x1.9660480000000p-1, 0x1.951ebc0000000p-1, 0x1.93df2c0000000p-1, 0x1.92a1920000000p-1,
    0x1.9165ec0000000p-1, 0x1.902c300000000p-1, 0x1.8ef4600000000p-1, 0x1.8dbe720000000p-1,
    0x1.8c8a660000000p-1, 0x1.8b58340000000p-1, 0x1.8a27dc0000000p-1, 0x1.88f9540000000p-1,
    0x1.87cc9e0000000p-1, 0x1.86a1b00000000p-1, 0x1.85788a0000000p-1, 0x1.8451280000000p-1,
    0x1.832b840000000p-1, 0x1.82079a0000000p-1, 0x1.80e5680000000p-1, 0x1.7fc4e80000000p-1,
    0x1.7ea6180000000p-1, 0x1.7d88f20000000p-1, 0x1.7c6d740000000p-1, 0x1.7b539c0000000p-1,
    0x1.7a3b640000000p-1, 0x1.7924c80000000p-1, 0x1.780fc40000000p-1, 0x1.76fc580000000p-1,
    0x1.75ea7e0000000p-1, 0x1.74da320000000p-1, 0x1.73cb720000000p-1, 0x1.72be380000000p-1,
    0x1.71b2860000000p-1, 0x1.70a8540000000p-1, 0x1.6f9fa00000000p-1, 0x1.6e98680000000p-1,
    0x1.6d92a60000000p-1, 0x1.6c8e5c0000000p-1, 0x1.6b8b800000000p-1, 0x1.6a8a160000000p-1,
};
// -ln c_j = kTabLogL[2j] + kTabLogL[2j+1]
__device__ const double kTabLogL[512] = {
    -0x1.617a6cc772fc7p-2, -0x1.148e372b0b85ep-57, -0x1.5ea85646b4be9p-2, -0x1.4334c1a7cbffap-58,
    -0x1.5bd83cc0bd9dep-2, -0x1.1cabb97283ac4p-62, -0x1.590a1a6506ec7p-2, -0x1.076091a70d10ep-57,
    -0x1.563def0307e3ep-2, -0x1.a30d79b02bbdcp-58, -0x1.5373ba5ffdcbep-2, -0x1.6b557d4cd4769p-61,
    -0x1.50ab70b28cbe4p-2, -0x1.bc1af8dada69bp-57, -0x1.4de51d1f9d4b8p-2, -0x1.7832a1f3b3bb3p-56,
    -0x1.4b20adeee89d9p-2, 0x1.1d2a513bfeaddp-56, -0x1.485e2e3474d8dp-2, -0x1.63ab3790c7a06p-57,
    -0x1.459d8bfefa1fbp-2, 0x1.14b34bd23e08cp-58, -0x1.42ded2515f4fcp-2, -0x1.c35136a15e8f5p-57,
    -0x1.4021fab56e99fp-2, -0x1.553eb19626b3fp-57, -0x1.3d66fe9a3d9d9p-2, -0x1.35d42b2bf3b12p-57,
    -0x1.3aade3186e284p-2, 0x1.67f2c1cf652b6p-57, -0x1.37f69b9b5a15bp-2, -0x1.b7d42d1c65eb7p-56,
    -0x1.35412d21f2bd8p-2, 0x1.2860a0c8ad36fp-56, -0x1.328d90d3ed35ep-2, -0x1.2d37895475478p-57,
    -0x1.2fdbcba252f98p-2, -0x1.cce623c1054b0p-57, -0x1.2d2bd0a0ae807p-2, -0x1.d156ab57cd494p-58,
    -0x1.2a7da4a5eb6c5p-2, -0x1.9d4c1164f335bp-56, -0x1.27d1468fab118p-2, 0x1.eb284989ae928p-58,
    -0x1.2526a92c0fed5p-2, 0x1.303da55301d49p-57, -0x1.227dd7369e4cfp-2, 0x1.92bf137df3cfcp-57,
    -0x1.1fd6c9611aa06p-2, 0x1.3ee29b31250fep-56, -0x1.1d317841f3bf7p-2, -0x1.78a89f6c3b20ap-56,
    -0x1.1a8de87885be6p-2, 0x1.c50f6510854dap-56, -0x1.17ec1892970bcp-2, -0x1.02f6601e5640cp-58,
    -0x1.154bfade24dffp-2, 0x1.447174422fafdp-56, -0x1.12ad99f644d6cp-2, 0x1.69df0b496838dp-57,
    -0x1.1010ee2404369p-2, 0x1.3c3e98a088922p-56, -0x1.0d75fbe12247bp-2, -0x1.f62d882d06eabp-56,
    -0x1.0adcb52d3f0afp-2, -0x1.f03be5c851d79p-56, -0x1.0845183895da2p-2, 0x1.6f6f197448b81p-56,
    -0x1.05af2f8bf24ecp-2, 0x1.966af23166639p-58, -0x1.031af321df609p-2, -0x1.f54ac82a89817p-56,
    -0x1.00885ad913531p-2, 0x1.f208aba99ea8bp-56, -0x1.fbeed5e168455p-3, 0x1.626cc24855418p-57,
    -0x1.f6d0364f5d539p-3, -0x1.8767741773730p-58, -0x1.f1b4ebe6e42a4p-3, -0x1.81eeeb64dfe15p-57,
    -0x1.ec9cd969a10d2p-3, -0x1.61b222c30ae27p-58, -0x1.e787fa79c4c94p-3, 0x1.90d933653b1ddp-57,
    -0x1.e27663e9f8944p-3, 0x1.868cdcf369e9bp-58, -0x1.dd67f8036f49ap-3, -0x1.0481699682d8bp-57,
    -0x1.d85cbed3fbdf9p-3, 0x1.b52d6866b1837p-57, -0x1.d354a6f87247ap-3, -0x1.6646c7e449944p-57,
    -0x1.ce4fc5222017bp-3, -0x1.5f67a3b4955c7p-57, -0x1.c94e07c4dea71p-3, 0x1.5dd9c5b689dd4p-60,
    -0x1.c44f5d1bedec6p-3, 0x1.142cf46805526p-59, -0x1.bf53d9becf83dp-3, 0x1.f3910ed6b1d6fp-57,
    -0x1.ba5b6bbf5979ep-3, -0x1.5f359151fe7b5p-57, -0x1.b5661acf30297p-3, -0x1.f9b2d950c7e68p-59,
    -0x1.b073d4be77c1cp-3, -0x1.ed9214a5107b9p-57, -0x1.ab849420b03f2p-3, 0x1.160b8fde24c4ap-60,
    -0x1.a6986074a4064p-3, 0x1.8ac9ac9f279a8p-58, -0x1.a1af414007a07p-3, -0x1.64bb0364a4de7p-58,
    -0x1.9cc916d27b4a4p-3, -0x1.579d7727977d2p-57, -0x1.97e5e877552d7p-3, 0x1.eb712cb4954a4p-58,
    -0x1.9305b05c54321p-3, -0x1.a6996095e3adap-57, -0x1.8e2875c22e033p-3, -0x1.6b5d5bfb9904cp-57,
    -0x1.894e32bbe08f4p-3, 0x1.2066e58444ceap-57, -0x1.8476e142f1382p-3, 0x1.f4821971ade6ep-58,
    -0x1.7fa26df30df12p-3, 0x1.a6e9ddfcbc88dp-58, -0x1.7ad0ed133a49ep-3, -0x1.f84027b1223eep-57,
    -0x1.7602586834358p-3, 0x1.64d55a0ec2f29p-57, -0x1.71369c40b401ap-3, 0x1.d3431eb722106p-57,
    -0x1.6c6dbf7a4ac54p-3, 0x1.2616a6d640622p-61, -0x1.67a7bb8c66094p-3, -0x1.867eb74fcd895p-59,
    -0x1.62e49748df64ap-3, 0x1.f3c71742ff52ep-57, -0x1.5e243e8f00883p-3, -0x1.eb88a755f79f6p-60,
    -0x1.5966b80cb1741p-3, 0x1.258d0f7fe6fccp-57, -0x1.54abfce97cdd2p-3, 0x1.4978bbf47eb63p-57,
    -0x1.4ff413c720702p-3, 0x1.6536fe2267c49p-57, -0x1.4b3ee81491820p-3, 0x1.8bb9475c9d4bbp-59,
    -0x1.468c804f2bf0dp-3, -0x1.b3c794f8bd08bp-57, -0x1.41dce2fa06576p-3, 0x1.2e6606344707bp-60,
    -0x1.3d2ffb354646bp-3, 0x1.12af74eddbd76p-57, -0x1.3885cf5f4fb60p-3, 0x1.5e0906970d0a8p-57,
    -0x1.33de5817ca6dcp-3, 0x1.048836fa1ac9ep-57, -0x1.2f399bb033668p-3, -0x1.373c78070c597p-57,
    -0x1.2a9784d6e28a6p-3, 0x1.255cfabd7459fp-59, -0x1.25f8279489c93p-3, -0x1.78c2a49dbdccep-57,
    -0x1.215b6e6a4dba0p-3, 0x1.e0ffb14a9305fp-58, -0x1.1cc1518af5ce5p-3, 0x1.c05de0915377bp-57,
    -0x1.1829e4f72f3ccp-3, -0x1.b2d31b00bdd2fp-57, -0x1.139512dff52c0p-3, -0x1.96525e560cd15p-57,
    -0x1.0f02ef485fad9p-3, -0x1.b03b9b12febf9p-57, -0x1.0a7356276dcbbp-3, -0x1.6a475833ebf6dp-57,
    -0x1.05e65b6a7313dp-3, -0x1.10b9e50122ca0p-57, -0x1.015bf6eb31242p-3, -0x1.53ba0ba8c6d71p-58,
    -0x1.f9a840d0d50c1p-4, 0x1.b42d44970fc48p-58, -0x1.f09dbb644cfbfp-4, 0x1.e07645d2c0131p-62,
    -0x1.e798306970e6ap-4, -0x1.00ea0d526a6d7p-59, -0x1.de97e4251f92dp-4, -0x1.c68f95e4f9707p-59,
    -0x1.d59c8cbac8f8ap-4, 0x1.03adf8c340e1ep-58, -0x1.cca651f9e98fcp-4, -0x1.c46f7ba630960p-60,
    -0x1.c3b50601a0b14p-4, 0x1.3c549abb57450p-61, -0x1.bac8b3ebb2e01p-4, 0x1.376e3d98a73c8p-62,
    -0x1.b1e166db3854cp-4, 0x1.60bdd93534088p-59, -0x1.a8ff0d23e9e80p-4, 0x1.3484fb11477dep-59,
    -0x1.a02194e2aaf26p-4, -0x1.ac23021124c85p-59, -0x1.974908f6133f3p-4, -0x1.621892ca43524p-59,
    -0x1.8e75573d1e7a3p-4, -0x1.7545a0eaa9e87p-60, -0x1.85a68a7854e1ap-4, -0x1.f40352b454635p-59,
    -0x1.7cdc90487b1c7p-4, 0x1.c35cbe3b969b4p-63, -0x1.741756171d0ecp-4, 0x1.85e0eaab29639p-59,
    -0x1.6b5703a7b7553p-4, 0x1.a75c6e76d386fp-58, -0x1.629b68fc8c9dcp-4, 0x1.62cc070ac3fbep-59,
    -0x1.59e49071aa842p-4, -0x1.f204c3ed438f9p-58, -0x1.5132846b9a4f1p-4, -0x1.c471b1b0163a5p-58,
    -0x1.4885144611db7p-4, 0x1.c7854ba9eeb6ap-58, -0x1.3fdc67aef9155p-4, 0x1.be9ad68adf211p-58,
    -0x1.37386b4b40442p-4, 0x1.d36c6eaed15eap-58, -0x1.2e990b880ae31p-4, -0x1.16b0bc6b96d96p-58,
    -0x1.25fe52633c5b3p-4, 0x1.9f9f3cfc6f3c4p-58, -0x1.1d6849e2c8336p-4, -0x1.006cf2c60103fp-58,
    -0x1.14d6c04364175p-4, 0x1.0b7d4aeb80ef6p-61, -0x1.0c49dd338e7adp-4, -0x1.30a324517b9d7p-59,
    -0x1.03c18c9865f5ep-4, 0x1.de11c0569ccf9p-58, -0x1.f67b743daa9d8p-5, -0x1.05287aa227845p-62,
    -0x1.e57cdec842290p-5, 0x1.df8b8fa37988ep-59, -0x1.d4872fa9356f7p-5, 0x1.fbcddfe36c772p-59,
    -0x1.c39a79d999a2fp-5, -0x1.ad4598aa8ebc4p-61, -0x1.b2b6d06199f1ep-5, -0x1.4e2457095717fp-59,
    -0x1.a1dc09871aa8ap-5, 0x1.2005973c72663p-59, -0x1.910a3810134c2p-5, 0x1.afc4e94f1cbc2p-60,
    -0x1.804131bff6038p-5, -0x1.9ba3d796f9283p-59, -0x1.6f80cbe8cdbeep-5, 0x1.d706739a809bbp-62,
    -0x1.5ec918bc5bc83p-5, 0x1.9d51ac12d9a0fp-59, -0x1.4e1a67ebfa3c8p-5, -0x1.7d9b6a4657241p-59,
    -0x1.3d7413724e637p-5, 0x1.3ed55809698c4p-61, -0x1.2cd6a84e4d56ep-5, 0x1.7364948684ef4p-60,
    -0x1.1c41bd47fc88ap-5, -0x1.ac48034bc25cap-64, -0x1.0bb56417c0f8bp-5, 0x1.f0e1e6b662732p-64,
    -0x1.f6635d07920b1p-6, 0x1.de20bcfaaa783p-61, -0x1.d56c63faedcf6p-6, 0x1.461bcd8dce04bp-64,
    -0x1.b486f891608fcp-6, -0x1.7367f83e81ae8p-61, -0x1.93b244e3ba6f4p-6, 0x1.732e9ffaf79b9p-61,
    -0x1.72ee6b6a71678p-6, 0x1.c3765d52cb022p-61, -0x1.523b1155fecc4p-6, 0x1.4d3b917dba4efp-60,
    -0x1.319858939b424p-6, -0x1.eb74151b20592p-61, -0x1.1106632a90b4cp-6, 0x1.e881678893b8ep-61,
    -0x1.e10aa67809df2p-7, 0x1.4a747accafb43p-61, -0x1.a0289c7ba606ep-7, 0x1.986bbcec73a35p-62,
    -0x1.5f66ea087789dp-7, 0x1.661051d6780aep-61, -0x1.1ec6cebe7446dp-7, 0x1.ac51800a01704p-61,
    -0x1.bc8f1fcb8d659p-8, -0x1.50b740b2953c3p-63, -0x1.3bd0e1f09f6eap-8, 0x1.72810e1435734p-62,
    -0x1.76a2ce850b23fp-9, -0x1.ee09dc7f14c11p-63, 0x0.0p+0, 0x0.0p+0,
    0x1.138011cff517ap-9, -0x1.cdf62404b16a1p-63, 0x1.88b79fa14a1a5p-8, 0x1.d6f86eaf88495p-64,
    0x1.43589190866ebp-7, 0x1.2ffa05756ed3cp-61, 0x1.c1d85dd793962p-7, 0x1.91a5c9f2df359p-64,
    0x1.1feda669d2397p-6, 0x1.a1b95d8b46a90p-62, 0x1.5eb182153419dp-6, -0x1.2ea95b96c9075p-62,
    0x1.9d381715e1318p-6, 0x1.eaa42eef7f7a6p-61, 0x1.db817c50cfdc7p-6, -0x1.6fec0aa2414f7p-62,
    0x1.0cc769ecd8550p-5, -0x1.e8b2579f7370dp-59, 0x1.2baffd40f42f3p-5, -0x1.27d3edafdfbb7p-60,
    0x1.4a7aeca9fb98dp-5, -0x1.f47afae11e246p-60, 0x1.69284b3399db7p-5, 0x1.9f729a531bba9p-59,
    0x1.87b870688e2fap-5, 0x1.3f7a900903831p-59, 0x1.a62b511eea7cap-5, -0x1.3b14fd691f204p-60,
    0x1.c4818c245adbcp-5, 0x1.5958ed192e7a6p-62, 0x1.e2baf802e1bd1p-5, 0x1.654a2d0ee195ap-59,
    0x1.006bf9f7c1304p-4, 0x1.91a7cb2428bbep-59, 0x1.0f6c5fab297a2p-4, -0x1.b569c6b1e4bf7p-59,
    0x1.1e5ecdc6f80eep-4, 0x1.e515967915bbfp-58, 0x1.2d43437b981a0p-4, -0x1.4362032da4971p-58,
    0x1.3c19e3021c1adp-4, -0x1.3f8326d1b2981p-58, 0x1.4ae2e0e4abd3bp-4, -0x1.ea54b9884f4c5p-59,
    0x1.599e2d4474406p-4, -0x1.82db027cd49bep-61, 0x1.684bfe5f9cc49p-4, 0x1.358dfb48b712ap-58,
    0x1.76ec689e8f71cp-4, -0x1.be9e55253e2bfp-61, 0x1.857f81262f435p-4, 0x1.e182f5b6f4358p-61,
    0x1.94055dd8cd45ep-4, 0x1.02280e8d319acp-60, 0x1.a27e1557196ffp-4, -0x1.cb0e52fdbb5cfp-60,
    0x1.b0e9bf010f3eap-4, 0x1.c87c943bb9c75p-58, 0x1.bf4872f6de2abp-4, 0x1.0aa4a28677d19p-58,
    0x1.cd9a4a19ce0aap-4, 0x1.011060a9011eep-58, 0x1.dbdf5e0d1f7a4p-4, -0x1.9314e89c8b86ep-62,
    0x1.ea17c936e85fbp-4, 0x1.707e0bae0c260p-59, 0x1.f84394a84e56fp-4, 0x1.da5fcce375ed4p-60,
    0x1.033177241b44cp-3, -0x1.f2b3a2ba1bd8dp-57, 0x1.0a3ae72c7fbe1p-3, -0x1.a1c1a6e4851e0p-59,
    0x1.113e28fa3327bp-3, 0x1.b332c84d00a22p-62, 0x1.183b4b7d8a2d8p-3, 0x1.4c96bf4490512p-57,
    0x1.1f325e0ab2f54p-3, 0x1.252f99fcba80cp-60, 0x1.2623671dc7b49p-3, -0x1.a51d98ba6d39fp-57,
    0x1.2d0e64332eb05p-3, 0x1.cacedee6b1a9cp-59, 0x1.33f36ed1355c5p-3, -0x1.a4a5b720d22afp-59,
    0x1.3ad297af30853p-3, -0x1.481814c054338p-57, 0x1.41abd3d5395aap-3, -0x1.32f2f58fd0d84p-57,
    0x1.487f3de2b147ep-3, 0x1.988f799436bedp-57, 0x1.4f4cd4b87022cp-3, 0x1.7a376547c8f38p-57,
    0x1.5614aa46a6ce0p-3, -0x1.df4504cdbcb49p-57, 0x1.5cd6c76847201p-3, 0x1.edd4d82d5718dp-57,
    0x1.63932bbb57e05p-3, 0x1.d664b5fbc31cbp-57, 0x1.6a49f3aa8408cp-3, -0x1.b35ae79a303bcp-57,
    0x1.70fb15d741e9bp-3, -0x1.9bc19fdd35c6fp-59, 0x1.77a6a5c04d391p-3, 0x1.a3ade74806c07p-59,
    0x1.7e4cada8b9114p-3, -0x1.6bdd6f551ef16p-57, 0x1.84ed2e703d512p-3, 0x1.6f892df8e72b4p-57,
    0x1.8b883c887034bp-3, 0x1.4350813df5e8cp-58, 0x1.921dd953d4987p-3, 0x1.f55f0aec38ad2p-59,
    0x1.98ae065ec1fb1p-3, 0x1.1bdec5711dc76p-58, 0x1.9f38e2c49a7f7p-3, 0x1.65d760ec64ad7p-57,
    0x1.a5be5d0599047p-3, 0x1.00ea64b5d1e55p-57, 0x1.ac3e94da2ef33p-3, 0x1.2ba2f30902243p-58,
    0x1.b2b982f480f79p-3, -0x1.37b7de2af16f0p-57, 0x1.b92f33ea85f5cp-3, -0x1.7a3eeb34ecf82p-60,
    0x1.bf9fbe91fad5bp-3, 0x1.fc9f78c51c5a0p-58, 0x1.c60b123b18ac6p-3, -0x1.814c7811b9fadp-58,
    0x1.cc7146334eda2p-3, -0x1.4768e14ad5db5p-60, 0x1.d2d25e1ba7f6bp-3, -0x1.12542a9412dd2p-57,
    0x1.d92e67d5f62e8p-3, 0x1.e2c9dc1343f1ep-57, 0x1.df85677472da1p-3, 0x1.2a94b18e1b6f9p-59,
    0x1.e5d761364a96bp-3, 0x1.94fefcb2f66f0p-58, 0x1.ec2463b428796p-3, -0x1.a22e839fc0d99p-57,
    0x1.f26c696b83a5ep-3, 0x1.59fd8bfed772ep-59, 0x1.f8af95d8b475ap-3, 0x1.e1fe87ac146f5p-60,
    0x1.feedcf6c16335p-3, -0x1.1801de0bc899cp-58, 0x1.02939d16fab5dp-2, -0x1.481af1d6d97c0p-56,
    0x1.05ade387b0622p-2, 0x1.6733eef613487p-56, 0x1.08c5c83094141p-2, 0x1.321a05a4570f4p-59,
    0x1.0bdb43a8ccb4dp-2, -0x1.7b36d14f3d6ccp-59, 0x1.0eee688dbee4ap-2, -0x1.02f901f24115bp-57,
    0x1.11ff2a6773c8bp-2, -0x1.5d85b8a0221eap-59, 0x1.150d9c1a8db99p-2, 0x1.05acfc5ecb0a2p-60,
    0x1.1819b688ae4e8p-2, -0x1.aaf54bc7bff4dp-57, 0x1.1b237d17a4657p-2, -0x1.7b13cb5152287p-57,
    0x1.1e2af88f5d367p-2, -0x1.1cdf8462aa27ap-57, 0x1.21302c91ad6c1p-2, 0x1.aaf492327562fp-56,
    0x1.2433178669135p-2, 0x1.81fa9cd6d10e5p-56, 0x1.2733c289f1e0fp-2, -0x1.97494b16f0022p-57,
    0x1.2a322c2cb021cp-2, 0x1.7a1310a91a4acp-57, 0x1.2d2e5dc3c7e3dp-2, -0x1.fb48fded517c4p-56,
    0x1.30285608913bdp-2, 0x1.1ab5e881f3aa9p-56, 0x1.332013bcfd9b9p-2, 0x1.e825b3bb24123p-57,
    0x1.3615a07ffcebep-2, 0x1.e0411a71c1c2ap-56, 0x1.390900ab1c5b4p-2, -0x1.16ca0a5014369p-58,
    0x1.3bfa38b0c340ap-2, -0x1.f1079b1a00c80p-57, 0x1.3ee9422ff8e89p-2, -0x1.198066a1f8bd6p-57,
    0x1.41d6272f3f255p-2, -0x1.d7bc00c9bfbc1p-57, 0x1.44c0ec60085c7p-2, -0x1.5851f561bf885p-58,
    0x1.47a9910acba36p-2, -0x1.8244df1960924p-58, 0x1.4a901f8d8f424p-2, 0x1.5df10de1f59b9p-57,
    0x1.4d748c470ec4dp-2, 0x1.5f97132c71919p-56, 0x1.5056e746326ffp-2, 0x1.3e3b3acdcb717p-57,
    0x1.5337301ce5975p-2, -0x1.accb13f9ad7c4p-56, 0x1.56156666a0128p-2, -0x1.6b85993c7c109p-57,
    0x1.58f194fcc7d83p-2, 0x1.66499e0b57c66p-57, 0x1.5bcbb069d5b51p-2, 0x1.093e7595082c0p-57,
    0x1.5ea3ceeef3090p-2, 0x1.94280969feff7p-61, 0x1.6179df8c08f1cp-2, 0x1.577bae67caa2ap-57,
};
// ---- END GENERATED TABLES ----

#ifndef PL_EXF_LEAN
#define PL_EXF_LEAN 1
#endif
// LDS copies of the tables, one per work-group (6 KiB lean, 8 KiB otherwise): every kernel that evaluates the exact f
// calls load_tables() before its first f (all threads of the work-group, then a barrier).
#if PL_EXF_LEAN
struct alignas(16) Tabs {
    double e[256];   // kTabExp1
    double cl[512];  // cell j: {c_j, hi(-ln c_j)} side by side, one 16-byte read (6 KiB in all)
};
#else
struct alignas(16) Tabs {
    double e[256];  // kTabExp
    double c[256];  // kTabLogC
    double l[512];  // kTabLogL
};
#endif
__shared__ Tabs tabs;

__device__ __forceinline__ void load_tables(int tid, int nthreads) {
    for (int i = tid; i < 256; i += nthreads) {
#if PL_EXF_LEAN
        tabs.e[i] = kTabExp1[i];
        tabs.cl[2 * i] = kTabLogC[i];
        tabs.cl[2 * i + 1] = kTabLogL[2 * i];
#else
        tabs.e[i] = kTabExp[i];
        tabs.c[i] = kTabLogC[i];
        tabs.l[i] = kTabLogL[i];
        tabs.l[i + 256] = kTabLogL[i + 256];
#endif
    }
    __syncthreads();
}

// PL_EXF_LEAN (round 4): exp takes 2^(j/256) as one fp64 value (T + T q, not T_hi + (T_lo + T_hi q)
// over 2^(j/128), with a degree-4 instead of a degree-5 polynomial),
// log drops the low part of -ln c_j, and the f builds e^(xc+yc) from the two exps it evaluates
// anyway -- e^x e^y e^d, d = fl(xc + yc) - (xc + yc) exact in fp64, e^d = 1 + d + d^2/2 (|d| <=
// 2^-17) -- instead of a third exp: ~13 fewer VALU per f.  Each value's fp64 error grows from
// ~2^-53 to ~3 2^-53 relative before the one rounding to fp32; the host harness
// (tools/micro/exactf_rounding.cpp) finds 0 of 5e7 exp, log and f results changed against
// correctly rounded ones, as before.
// e^x in fp64 for fp32 x, |x| <= 200: N = rint(x 128/ln2) by the 1.5 * 2^52 shifter (its low word
// is N), r = x - N ln2/128 (|r| <= ln2/256, exact to ~2^-60), e^r - 1 = q by a degree-5 Taylor
// polynomial (remainder < 2^-60), e^x = 2^(N >> 7) T (1 + q), T = 2^((N & 127) / 128) from the
// table as hi + lo; the one rounding that matters is the final T + T q (~2^-53 relative).
__device__ __forceinline__ double exp_d(float xf) {
    const double x = (double)xf;
#if PL_EXF_LEAN
    // x = N ln2/256 + r, |r| <= ln2/512: e^r - 1 = q by degree 4 (remainder < 2^-54), T = 2^(j/256)
    // as one fp64 value, e^x = 2^(N >> 8) (T + T q)
    const double t = __builtin_fma(x, kTabInvC1, 0x1.8p52);
    const int n = (int)(uint32_t)__builtin_bit_cast(unsigned long long, t);
    const double nd = t - 0x1.8p52;
    double r = __builtin_fma(-nd, kTabC1Hi, x);
    r = __builtin_fma(-nd, kTabC1Lo, r);
    const double r2 = r * r;
    double h = __builtin_fma(1.0 / 24.0, r, 1.0 / 6.0);
    h = __builtin_fma(h, r, 0.5);
    const double q = __builtin_fma(r2, h, r);
    const double th = tabs.e[n & 255];
    return __builtin_ldexp(__builtin_fma(th, q, th), n >> 8);
#else
    const double t = __builtin_fma(x, kTabInvC, 0x1.8p52);
    const int n = (int)(uint32_t)__builtin_bit_cast(unsigned long long, t);
    const double nd = t - 0x1.8p52;
    double r = __builtin_fma(-nd, kTabCHi, x);
    r = __builtin_fma(-nd, kTabCLo, r);
    const double r2 = r * r;
    double h = __builtin_fma(1.0 / 120.0, r, 1.0 / 24.0);
    h = __builtin_fma(h, r, 1.0 / 6.0);
    h = __builtin_fma(h, r, 0.5);
    const double q = __builtin_fma(r2, h, r);
    const int j = n & 127;
    const double th = tabs.e[2 * j], tl = tabs.e[2 * j + 1];
    const double m = __builtin_fma(th, q, tl) + th;
    return __builtin_ldexp(m, n >> 7);
#endif
}
// fp32 exp(x), |x| <= 87, correctly rounded (but for ~2^-28 of the arguments): one rounding of
// the fp64 value (the 2^k scaling is exact in fp64)
__device__ __forceinline__ float exp_cr(float xf) { return (float)exp_d(xf); }
// fp32 e^(fl(xc + yc)) from the fp64 e^xc, e^yc: e^xc e^yc e^d, d = fl(xc + yc) - (xc + yc), which
// Fast2Sum gives exactly in fp32 ((s - a) - b with |a| >= |b|)
#ifndef PL_EXF_TWOSUM
#define PL_EXF_TWOSUM 1  // d by the branch-free TwoSum (5 adds) instead of the ordered Fast2Sum (compare, 2 selects, 2 subs): A/B 0.8155 -> 0.8089 ms, bit-identical (profiles/r05zz_sc_exact_twosum_ab.txt)
#endif
__device__ __forceinline__ float exp_sum(double ex, double ey, float xc, float yc) {
    const float s = xc + yc;
#if PL_EXF_TWOSUM
    // TwoSum: e = (xc + yc) - s exactly, d = -e; the same exact value as the ordered form
    const float bb = s - xc;
    const double d = -(double)((xc - (s - bb)) + (yc - bb));
#else
    const bool sw = __builtin_fabsf(yc) > __builtin_fabsf(xc);
    const float a = sw ? yc : xc, b = sw ? xc : yc;
    const double d = (double)((s - a) - b);
#endif
    return (float)(ex * ey * __builtin_fma(d, __builtin_fma(d, 0.5, 1.0), 1.0));
}

// ln x in fp64 for normal fp32 x > 0: d = bits(x) - bits(sqrt(1/2)), e = d >> 23 (arithmetic),
// m = 2^-e x in [sqrt(1/2), sqrt(2)) (its bits: the low 23 of d + bits(sqrt(1/2))), cell j = bits
// 15..22 of d; r = m c_j - 1 is exact (two 24-bit factors), |r| < 2^-9; log1p(r) by degree 6
// (remainder < 2^-56 relative); ln x = e ln2 + (-ln c_j) + log1p(r).  For e != 0, |ln x| > 0.34;
// for e = 0 the cell of 1.0 has c = 1: no cancellation anywhere.
__device__ __forceinline__ double log_d(float xf) {
    const int32_t d = (int32_t)(__float_as_uint(xf) - kTabLogBase);
    const int e = d >> 23;
    const uint32_t mb = (uint32_t)d & 0x7FFFFFu;
    const int j = (int)(mb >> 15);
    const double m = (double)__uint_as_float(mb + kTabLogBase);
#if PL_EXF_LEAN
    const double2 cl = *reinterpret_cast<const double2*>(&tabs.cl[2 * j]);
    const double r = __builtin_fma(m, cl.x, -1.0);
#else
    const double r = __builtin_fma(m, tabs.c[j], -1.0);
#endif
    const double r2 = r * r;
    double p = __builtin_fma(-1.0 / 6.0, r, 1.0 / 5.0);
    p = __builtin_fma(p, r, -0.25);
    p = __builtin_fma(p, r, 1.0 / 3.0);
    p = __builtin_fma(p, r, -0.5);
    const double l1 = __builtin_fma(r2, p, r);
    const double de = (double)e;
#if PL_EXF_LEAN
    const double hi = __builtin_fma(de, kTabLn2Hi, cl.y);
    const double lo = __builtin_fma(de, kTabLn2Lo, l1);
#else
    const double hi = __builtin_fma(de, kTabLn2Hi, tabs.l[2 * j]);
    const double lo = __builtin_fma(de, kTabLn2Lo, tabs.l[2 * j + 1]) + l1;
#endif
    return hi + lo;
}
__device__ __forceinline__ float log_cr(float xf) { return (float)log_d(xf); }

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
    const float r = log_poly(xf);  // frexp-based: subnormal arguments too
    return xf == __builtin_inff() ? xf : xf == 0.0f ? -__builtin_inff() : r;
}
// (inlined into the f functions behind a wave-uniform branch: a call there would make them
// non-leaf functions, which save their return address and a VGPR to scratch on every call)
__device__ __forceinline__ float f_exact_wide(float x, float y, float lmax) {
    const float xc = fminf(fmaxf(x, -lmax), lmax), yc = fminf(fmaxf(y, -lmax), lmax);
    float o = log_cr_wide(1.0f + exp_cr_wide(xc + yc));
    o -= log_cr_wide(exp_cr_wide(xc) + exp_cr_wide(yc));
    return o;
}
// exp_cr's range |x| <= 87 holds for every argument f forms when llr_max <= 43 (|xc + yc| <= 86)
constexpr float kExactFastLmax = 43.0f;
// PL_EXF_RANGE: 0 = each f tests llr_max (a kernel for any plan), 1 = the fast forms only, 2 = the
// full-range forms only.  The code-specialised SC kernels are built as 1 or 2 (jit.cpp: the plan's
// llr_max <= 43 or not picks the code object), so their f carry no test and the lane-level f can be
// inlined (sc_static.h PL_SC_FLANE_INLINE) without dragging the full-range path into the kernel.
#ifndef PL_EXF_RANGE
#define PL_EXF_RANGE 0
#endif
__device__ __forceinline__ bool wide_range(float lmax) {
#if PL_EXF_RANGE == 0
    return lmax > kExactFastLmax;
#else
    (void)lmax;
    return PL_EXF_RANGE == 2;
#endif
}

// clip(x, +-lmax) (dec.py:39-40) as one v_med3_f32 instead of the canonicalising v_max / v_min
// pairs fminf(fmaxf(x, -lmax), lmax) compiles to (LLRs are never NaN: DESIGN.md section 7); the
// same value for every other input, +-0 included
#ifndef PL_EXF_MED3
#define PL_EXF_MED3 1
#endif
__device__ __forceinline__ float clip_l(float x, float lmax) {
#if PL_EXF_MED3
    return __builtin_amdgcn_fmed3f(x, -lmax, lmax);
#else
    return fminf(fmaxf(x, -lmax), lmax);
#endif
}
// the plan's llr_max is the same in every lane: taken as a scalar, the wide-range test is a scalar
// branch instead of an exec-mask if/else (the out-of-line f receives it in a VGPR)
#ifndef PL_EXF_UNIFORM
#define PL_EXF_UNIFORM 1
#endif
__device__ __forceinline__ float uniform_l(float lmax) {
#if PL_EXF_UNIFORM
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, lmax)));
#else
    return lmax;
#endif
}

// f of my_sn/fec/polar/dec.py:39-43 on clipped inputs, each operation rounded as the reference does.
// Out of line: inlined into the fully unrolled specialised SC kernels (hundreds of f per lane) the
// fp64 code made one (128,256) kernel take minutes to compile.  PL_EXF_INLINE 1 inlines f_exact and
// f_exact2 (fixed-range builds only, PL_EXF_RANGE != 0).
#ifndef PL_EXF_INLINE
#define PL_EXF_INLINE 0
#endif
#if PL_EXF_INLINE && PL_EXF_RANGE == 0
#error "PL_EXF_INLINE needs PL_EXF_RANGE 1 or 2"
#endif
#if PL_EXF_INLINE
#define PL_EXF_ATTR __attribute__((always_inline))
#else
#define PL_EXF_ATTR __attribute__((noinline))
#endif
__device__ PL_EXF_ATTR float f_exact(float x, float y, float lmax) {
    lmax = uniform_l(lmax);
    if (wide_range(lmax)) return f_exact_wide(x, y, lmax);
    const float xc = clip_l(x, lmax), yc = clip_l(y, lmax);
#if PL_EXF_LEAN
    const double ex = exp_d(xc), ey = exp_d(yc);
    float o = log_cr(1.0f + exp_sum(ex, ey, xc, yc));
    o -= log_cr((float)ex + (float)ey);
#else
    float o = log_cr(1.0f + exp_cr(xc + yc));
    o -= log_cr(exp_cr(xc) + exp_cr(yc));
#endif
    return o;
}

// Two f at once (one call, the two evaluations' fp64 chains interleaved by the scheduler): the
// specialised SC kernel's lane-local f loops call this for element pairs.  Each value is exactly
// f_exact's.
struct f2 {
    float a, b;
};
__device__ PL_EXF_ATTR f2 f_exact2(float x0, float y0, float x1, float y1, float lmax) {
    lmax = uniform_l(lmax);
    if (wide_range(lmax)) return f2{f_exact_wide(x0, y0, lmax), f_exact_wide(x1, y1, lmax)};
    const float xc0 = clip_l(x0, lmax), yc0 = clip_l(y0, lmax);
    const float xc1 = clip_l(x1, lmax), yc1 = clip_l(y1, lmax);
#if PL_EXF_LEAN
    const double ea0 = exp_d(xc0), ea1 = exp_d(xc1), eb0 = exp_d(yc0), eb1 = exp_d(yc1);
    const float s0 = exp_sum(ea0, eb0, xc0, yc0), s1 = exp_sum(ea1, eb1, xc1, yc1);
    const float a0 = (float)ea0, a1 = (float)ea1, b0 = (float)eb0, b1 = (float)eb1;
#else
    const float s0 = exp_cr(xc0 + yc0), s1 = exp_cr(xc1 + yc1);
    const float a0 = exp_cr(xc0), a1 = exp_cr(xc1);
    const float b0 = exp_cr(yc0), b1 = exp_cr(yc1);
#endif
    const float p0 = log_cr(1.0f + s0), p1 = log_cr(1.0f + s1);
    const float q0 = log_cr(a0 + b0), q1 = log_cr(a1 + b1);
    f2 r;
    r.a = p0 - q0;
    r.b = p1 - q1;
    return r;
}

}  // namespace plx
