// scl_tree_kernel.hip -- SC-list polar decoder for gfx950 (MI355X), "register subtree" form.
//
// Same decoder as scl_kernel.hip (x_run_sn_polar/polar/polar_scl.py SCL_Dec, :49-234; and the
// exact-f variant of my_sn/fec/polar/dec.py:330-339 without fast-SCL pruning), restructured for
// latency and lane utilisation: the reference walks the tree leaf by leaf with a sort + full-row
// copy of all 2L paths at every information leaf (:86-120); here
//
//  * one wave decodes CPW = 64 / 2L codewords; codeword c owns the 2L-lane group
//    [2Lc, 2Lc + 2L): lanes 0..L-1 of the group are its paths, lanes L..2L-1 shadow them and
//    evaluate the u = 1 candidates, so every lane of the wave does useful work at the leaves;
//  * the bottom of the tree runs LANE-PER-PATH: a path lane decodes its path's stage-R node
//    (R = 4, 16 leaves) entirely in its VGPRs -- stage buffers 0..R-1 (fp64), the node's
//    partial sums as one bit word, the path metric.  f/g, the per-leaf metric update (:69-85)
//    and, at information leaves, the 2L-candidate selection (:86-92) run without LDS traffic:
//    candidates are ranked in the group by DPP row rotations (2L = 16), quad permutes (2L = 4),
//    ds_bpermute (2L = 8, 32) or readlane (2L = 64), in the stable (metric, candidate index)
//    order -- candidate c < L = (state c, u=0), c >= L = (state c-L, u=1), the reference's
//    logical order after _update_single_bit_np :49-68 -- and a fork (:109-120) pulls the
//    parent's LIVE stage buffers with ds_bpermute (a stage-s buffer is live iff the leaf is in
//    the left half of its stage-s node; dead ones are never copied);
//  * forks only move register state: each lane records the path it descends from at subtree
//    entry ("origin"); the LDS state of the upper tree (stage-buffer owner pointers, partial
//    sums of finished nodes) is re-pointed once per subtree, from the origins, instead of once
//    per information leaf;
//  * the upper stages run WAVE-PARALLEL over (codeword, path, element) from LDS, with lazy
//    copies (per path per stage owner pointers, as scl_kernel.hip);
//  * the channel is never copied to LDS, and the top V stages below it are never stored: a node
//    reading one recomputes its input from the channel row in global memory (L2-resident after
//    the first pass) and the path's partial sums (f/g are pure functions of those), so a
//    codeword needs ~4.5 KB of LDS at n=1024, L=8, V=4;
//  * decided bits are not tracked: the root's partial sums are x = u G_n and u = x G_n (G_n is
//    an involution over GF(2)), recovered by one butterfly per path at the end.
//
// Every f, g and metric value is computed by the same fp64 expressions, in the same order, as
// scl_kernel.hip, so the two kernels agree bit for bit (tests/test_scl_gpu.py runs both).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "../../../include/polar_mi355x.h"
#include "plan.h"
#include "softplus.h"

namespace {

// Tuning macros (A/B variants: tools/scl_variants.py)
#ifndef PL_SCL_R
#define PL_SCL_R 4  // stage of the lane-local subtree (4 or 5; A/B on MI355X: 4 is 19 % faster)
#endif
#ifndef PL_SCL_LOADGRP
#define PL_SCL_LOADGRP 0  // > 0: stage-R input read in groups of this many pairs (caps VGPRs)
#endif
#ifndef PL_SCL_UNROLL
#define PL_SCL_UNROLL 1  // 1: the 2^R leaves of a lane-local subtree fully unrolled (A/B: 2.08 vs 2.27 ms; round 6,
                        // constant leaf indices via unroll_leaves: 0.793 -> 0.744 ms, profiles/r06d_scl_unroll_ab.txt)
#endif
#ifndef PL_SCL_DIAG_NO_UPPER
#define PL_SCL_DIAG_NO_UPPER 0
#endif
#ifndef PL_SCL_DIAG_NO_UPPER_PRUNE
#define PL_SCL_DIAG_NO_UPPER_PRUNE 0  // timing diagnostic: fast-SCL only inside the lane subtrees (wrong)
#endif
#ifndef PL_SCL_DIAG_SKIP_V
#define PL_SCL_DIAG_SKIP_V 0
#endif
#ifndef PL_SCL_DIAG_SKIP_ST
#define PL_SCL_DIAG_SKIP_ST 0
#endif
#ifndef PL_SCL_FROZEN_PAIR
#define PL_SCL_FROZEN_PAIR 1  // 1: a frozen sibling leaf pair takes one exp/log per lane (shadow lanes the right leaf)
#endif
#ifndef PL_SCL_RANK_MASK
#define PL_SCL_RANK_MASK 1  // 1: 16-lane rank with a static tie mask and carry-in adds (no index DPP)
#endif
#ifndef PL_SCL_RANK_SUBB
#define PL_SCL_RANK_SUBB 1  // 1: 16-lane rank as 64-bit borrow chains with DPP sources (rank16_subb)
#endif
#ifndef PL_SCL_FG_BITS
#define PL_SCL_FG_BITS 1  // 1: min-sum f and g sign handling on the high words (f_ms, g_op)
#endif
#ifndef PL_SCL_ST_UNROLL
#define PL_SCL_ST_UNROLL 1  // 1: min-sum stored-stage node passes of 2^R / 2^(R+1) outputs unrolled, loads first
                           // (A/B r02zk: 1.081 -> 1.050 ms)
#endif
#ifndef PL_SCL_ST_CH
#define PL_SCL_ST_CH 8  // elements per lane loaded ahead in those passes
#endif
#ifndef PL_SCL_DIAG_NO_REPOINT
#define PL_SCL_DIAG_NO_REPOINT 0  // timing diagnostic (wrong results)
#endif
#ifndef PL_SCL_DIAG_NO_PULL
#define PL_SCL_DIAG_NO_PULL 0  // timing diagnostic (wrong results)
#endif
#ifndef PL_SCL_DIAG_NO_COMBINE
#define PL_SCL_DIAG_NO_COMBINE 0  // timing diagnostic (wrong results)
#endif
#ifndef PL_SCL_DIAG_VC_NOSTORE
#define PL_SCL_DIAG_VC_NOSTORE 0  // timing diagnostic (wrong results): no virtual-node cache stores (min-sum)
#endif
// Diagnostic macros (timing ablations with WRONG results) exist only in development builds.
#if !PL_DEV && (PL_SCL_DIAG_NO_UPPER || PL_SCL_DIAG_NO_UPPER_PRUNE || PL_SCL_DIAG_SKIP_V || PL_SCL_DIAG_SKIP_ST || \
                PL_SCL_DIAG_NO_REPOINT || PL_SCL_DIAG_NO_COMBINE || PL_SCL_DIAG_NO_RANK || PL_SCL_DIAG_CHEAP_PEN || \
                PL_SCL_DIAG_NO_PULL || PL_SCL_DIAG_FMS_ALL || PL_SCL_DIAG_VC_NOSTORE)
#error "PL_SCL_DIAG_* macros give wrong results: development builds (-DPL_DEV=1) only"
#endif
#ifndef PL_SCL_REPOINT_VEC
#define PL_SCL_REPOINT_VEC 1  // 1: re-pointing in 16-byte rows, two lanes per (codeword, path) pair (n >= 128)
#endif
#ifndef PL_SCL_FEX_HOIST
#define PL_SCL_FEX_HOIST 1  // 1: exact-f virtual passes evaluate the path-independent f levels once (vvisit_ex)
#endif
#ifndef PL_SCL_WPE
#define PL_SCL_WPE 2  // > 0: amdgpu_waves_per_eu minimum (2: <= 256 VGPRs, A/B on MI355X: 2.30 vs 3.62 ms at V=4)
#endif

// Phase timing (development builds, tools/scl_prof.py): per wave, s_memtime cycles spent in each
// phase of the decoder loop, written after the 2L-row metrics of out_pm (the caller sizes out_pm
// for bs * 2L + waves * 12 doubles).  Phases: 0 virtual node passes (left / f), 1 stored-stage node
// passes, 2 lane subtrees, 3 re-pointing and partial-sum stores, 4 combines, 5 pruned nodes and
// right (g) virtual passes, 6 set-up (incl. exact-f caches), 7 the final butterfly / CRC / sort /
// output; 8..11 split the lane subtrees (min-sum, no fast-SCL): leaf f/g, penalties, ranks,
// selection moves (2 keeps the rest).
#ifndef PL_SCL_PROF
#define PL_SCL_PROF 0
#endif
#if PL_SCL_PROF && !PL_DEV
#error "PL_SCL_PROF: development builds (-DPL_DEV=1) only"
#endif
#if PL_SCL_PROF
constexpr int kProfSlots = 12;  // 8..11: inside the lane subtrees -- leaf f/g, penalties, ranks, selection moves
struct Prof {
    unsigned long long acc[kProfSlots];
    unsigned long long t;
};
#define PROF_DECL                                            \
    Prof prof;                                               \
    _Pragma("unroll") for (int pi_ = 0; pi_ < kProfSlots; ++pi_) prof.acc[pi_] = 0; \
    prof.t = __builtin_amdgcn_s_memtime()
#define PROF_MARK_P(P, i)                                            \
    do {                                                             \
        const unsigned long long prof_n = __builtin_amdgcn_s_memtime(); \
        (P).acc[i] += prof_n - (P).t;                                \
        (P).t = prof_n;                                              \
    } while (0)
#define PROF_MARK(i) PROF_MARK_P(prof, i)
#endif
#if PL_SCL_PROF >= 2
// PL_SCL_PROF 2: sub-phases of the exact-f virtual pass (vvisit_ex), reported in the slots the FAST
// kernels leave empty: 8 = cache / channel loads (waited for), 10 = the four-outcome f, 11 = the
// per-path levels (the waits and LDS counters perturb the timing: for shares only)
__shared__ unsigned long long vex_prof[3];
#define VEX_T0 unsigned long long vex_t = __builtin_amdgcn_s_memtime()
#define VEX_MARK(i)                                                            \
    do {                                                                       \
        const unsigned long long vex_n = __builtin_amdgcn_s_memtime();         \
        if (lane == 0) vex_prof[i] += vex_n - vex_t;                           \
        vex_t = vex_n;                                                         \
    } while (0)
#else
#define VEX_T0
#define VEX_MARK(i)
#endif
#if PL_SCL_PROF
#define PROF_PARAM , Prof& prof
#define PROF_ARG , prof
#else
#define PROF_DECL
#define PROF_MARK(i)
#define PROF_PARAM
#define PROF_ARG
#endif

constexpr int R = PL_SCL_R;  // stage of the lane-local subtree
constexpr int T = 1 << R;    // leaves per lane-local subtree (<= one partial-sum word)
constexpr int SPS = 16;      // bytes per path of the stage-owner table (S + 1 <= 16), one 16-byte row

__host__ __device__ constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x >> 1); }
__host__ __device__ inline int align16(int x) { return (x + 15) & ~15; }

// LDS layout of ONE codeword; codeword c of a wave sits at c * bytes.
struct Lay {
    int W;    // partial-sum words per path
    int SS;   // top stored stage (R..SS in LDS); SS == R == S: the channel is the subtree input,
              // kept as fp64 in A[0, T) and shared by every path (per = 0)
    int per;  // doubles per path of stored stages
    int off_A, off_beta, off_sptr, off_org, off_ps, off_pm, off_fail, off_sv, off_sp, bytes;
};

__host__ __device__ inline Lay make_layout(int n, int S, int L, int V) {
    Lay y;
    y.W = n / 32;
    y.SS = S == R ? R : S - 1 - V;
    y.per = S == R ? 0 : (1 << (y.SS + 1)) - (1 << R);
    int o = 0;
    y.off_A = o; o = align16(o + (S == R ? T : L * y.per) * 8);
    y.off_beta = o; o = align16(o + L * y.W * 4);
    y.off_sptr = o; o = align16(o + L * SPS);
    y.off_org = o; o = align16(o + L * 4);
    y.off_ps = o; o = align16(o + L * 4);
    y.off_pm = o; o = align16(o + L * 8);
    y.off_fail = o; o = align16(o + L * 4);
    y.off_sv = o; o = align16(o + 2 * L * 8);  // final: metric + penalty of sorted row r
    y.off_sp = o; o = align16(o + 2 * L * 4);  // final: state of sorted row r
    y.bytes = o;
    return y;
}

// Exact-f leftmost-chain cache (global workspace): for k = 1 .. V, the input of the leftmost
// stage-(S-k) node, 2^(S-k) doubles at offset 2^S - 2^(S-k+1) of a codeword's slot.  Those nodes
// are reached from the channel through f levels only, so their inputs do not depend on the path:
// a virtual pass whose node lies below ns leading f levels reads the values of level ns from here
// instead of evaluating ns levels of exact f (each chain value was recomputed by every pass under
// it: 16 passes at n = 1024 for the 512 values of k = 1).
__host__ __device__ inline int chain_size(int n, int V) { return n - (n >> V); }
__host__ __device__ inline int chain_off(int n, int k) { return n - (n >> (k - 1)); }
// After the chain, the four-outcome tables of vvisit_ex (one per ns = 0 .. V-2): T_ns[4 e + 2 b1 + b2]
// = f(g(src[e], src[e + 2 D], b1), g(src[e + D], src[e + 3 D], b2)), e < D = 2^(S-ns-2), src = the
// channel (ns = 0) or chain level ns.  Every pass with the same ns reads the same table (8 passes
// for ns = 0 at n = 1024), so it is evaluated once per codeword.
__host__ __device__ inline int combo_size(int n, int V) { return V >= 2 ? 2 * n - 4 * (n >> V) : 0; }
__host__ __device__ inline int combo_off(int n, int V, int ns) { return chain_size(n, V) + 2 * n - 4 * (n >> (ns + 1)); }
__host__ __device__ inline int cache_size(int n, int V) { return chain_size(n, V) + combo_size(n, V); }

#if PL_SCL_FG_BITS
// v_min_f64 without the input canonicalisation fmin() adds (a v_max_f64 per operand that is not
// known canonical); the decoder never sees NaNs (unsupported inputs)
__device__ __forceinline__ double min_abs_nc(double a, double b) {
    double d;
    asm("v_min_f64 %0, |%1|, |%2|" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
__device__ __forceinline__ double min_nc(double a, double b) {
    double d;
    asm("v_min_f64 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
#endif

__device__ __forceinline__ double f_ms(double x, double y, double lmax) {  // polar_scl.py:93-106
#if PL_SCL_FG_BITS
    // m >= +0, so sign(x) sign(y) m is m with the sign bit x31 ^ y31 (two 32-bit ops on the high
    // words instead of a 64-bit sign test, a negation and two selects)
    const double m = min_nc(min_abs_nc(x, y), lmax);
    const unsigned long long mb = (unsigned long long)__double_as_longlong(m);
    const uint32_t sx = (uint32_t)((unsigned long long)__double_as_longlong(x) >> 32);
    const uint32_t sy = (uint32_t)((unsigned long long)__double_as_longlong(y) >> 32);
    const uint32_t hi = (uint32_t)(mb >> 32) | ((sx ^ sy) & 0x80000000u);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | (mb & 0xffffffffull)));
#else
    const double m = fmin(fmin(fabs(x), fabs(y)), lmax);
    const bool neg = (__double_as_longlong(x) ^ __double_as_longlong(y)) < 0;
    return neg ? -m : m;
#endif
}
#ifndef PL_SCL_FEX_FORM
#define PL_SCL_FEX_FORM 1  // exact f: 1 = softplus.h f_exact_pm (no cancellation), 0 = the reference's expression (ocml)
#endif
__device__ __forceinline__ double f_ex(double x, double y, double lmax) {  // my_sn dec.py:330-339
#if PL_SCL_DIAG_FMS_ALL  // timing diagnostic only (wrong results): min-sum in place of the exact f
    return fmin(fmin(fabs(x), fabs(y)), lmax) * (((x < 0) != (y < 0)) ? -1.0 : 1.0);
#elif PL_SCL_FEX_FORM == 0
    const double xc = fmax(fmin(x, lmax), -lmax), yc = fmax(fmin(y, lmax), -lmax);
    double o = log(1.0 + exp(xc + yc));
    o -= log(exp(xc) + exp(yc));
    return o;
#else
    return pl::f_exact_pm(x, y, lmax);  // softplus.h: the same value without the cancellation
#endif
}
// two exact f evaluations interleaved (independent chains overlap within the wave)
__device__ __forceinline__ void f_ex2(double x0, double y0, double x1, double y1, double lmax, double& r0, double& r1) {
#if PL_SCL_DIAG_FMS_ALL || PL_SCL_FEX_FORM == 0
    r0 = f_ex(x0, y0, lmax);
    r1 = f_ex(x1, y1, lmax);
#else
    const double x[2] = {x0, x1}, y[2] = {y0, y1};
    double r[2];
    pl::f_exact_pm_n<2>(x, y, lmax, r);
    r0 = r[0];
    r1 = r[1];
#endif
}
template <int FM>
__device__ __forceinline__ double f_op(double x, double y, double lmax) {
    if constexpr (FM == 0) return f_ms(x, y, lmax);
    else return f_ex(x, y, lmax);
}
__device__ __forceinline__ double g_op(double x, double y, uint32_t bit) {  // :107-108
#if PL_SCL_FG_BITS
    // (1 - 2u) x + y: the bit goes straight into x's sign (a shift and a xor, which the compiler
    // folds with the bit extraction, instead of a compare and a select)
    const unsigned long long xb = (unsigned long long)__double_as_longlong(x);
    return __longlong_as_double((long long)(xb ^ ((unsigned long long)(bit << 31) << 32))) + y;
#else
    return (bit ? -x : x) + y;
#endif
}
__device__ __forceinline__ uint32_t getbit(const uint32_t* w, int pos) { return (w[pos >> 5] >> (pos & 31)) & 1u; }

__device__ __forceinline__ double readlane_d(double v, int q) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), q);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), q);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ int bperm_i(int v, int src) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }
__device__ __forceinline__ double bperm_d(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)(b & 0xffffffffLL));
    const int hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffLL), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Value of group lane gl ^ L (a path lane's shadow, or a shadow lane's path).
template <int L>
__device__ __forceinline__ double half_xchg(double v, int lane) {
    if constexpr (L == 8) return dpp_d<0x120 + 8>(v);  // row_ror:8 in the 16-lane row = lane ^ 8
    else if constexpr (L == 2) return dpp_d<0x4E>(v);  // quad_perm [2,3,0,1]
    else return bperm_d(v, lane ^ L);
}

// Candidate (metric) of group lane (gl + r) mod GW, r = 1..GW-1, accumulated into the rank of
// this lane's candidate in the stable (metric, index) order.
// acc + (bit `lane` of m): one v_addc with the lane mask as carry-in
__device__ __forceinline__ int add_lane_bit(int acc, uint64_t m) {
    int r;
    uint64_t co;
    asm("v_addc_co_u32_e64 %0, %1, 0, %2, %3" : "=v"(r), "=s"(co) : "v"(acc), "s"(m));
    return r;
}

#if PL_SCL_RANK_SUBB
// Rank of this lane's candidate in its 16-lane group (the DPP row), all 15 rotations in one
// block.  Metrics are non-negative doubles (pm starts at 0 or llr_max > 0 and only ever adds
// softplus values >= +0; never -0 or NaN), so their bit patterns order like the values, and the
// stable (metric, index) comparison "v < cv, or v == cv with the lower index" is the 64-bit
// unsigned v < cv + tie, tie = 1 exactly when the rotated source has the lower index (the same
// static row mask as the ballot form above: group lanes >= r under row_ror:r).  Per rotation:
// the tie mask into VCC as the borrow-in, v_subb on the low and high words with the rotated
// candidate as the DPP source -- the final borrow is the comparison -- and one carry add into
// the rank.  3 VALU (2 of them DPP) + 2 SALU, against 2 DPP moves + 2 fp64 compares + 1 add +
// 3 SALU.
#define PL_RANK_ROT(r, m)                                                                   \
    "s_mov_b32 vcc_lo, " #m "\n\t"                                                          \
    "s_mov_b32 vcc_hi, " #m "\n\t"                                                          \
    "v_subb_co_u32_dpp %1, vcc, %2, %2, vcc row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t" \
    "v_subb_co_u32_dpp %1, vcc, %3, %3, vcc row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t" \
    "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n\t"
__device__ __forceinline__ int rank16_subb(double cv) {
    const long long b = __double_as_longlong(cv);
    const int lo = (int)(b & 0xffffffffLL), hi = (int)(b >> 32);
    int rk, tmp;
    asm volatile(
        "s_nop 1\n\t"  // the DPP sources were just written by a VALU
        "v_mov_b32 %0, 0\n\t"
        PL_RANK_ROT(1, 0xfffefffe) PL_RANK_ROT(2, 0xfffcfffc) PL_RANK_ROT(3, 0xfff8fff8)
        PL_RANK_ROT(4, 0xfff0fff0) PL_RANK_ROT(5, 0xffe0ffe0) PL_RANK_ROT(6, 0xffc0ffc0)
        PL_RANK_ROT(7, 0xff80ff80) PL_RANK_ROT(8, 0xff00ff00) PL_RANK_ROT(9, 0xfe00fe00)
        PL_RANK_ROT(10, 0xfc00fc00) PL_RANK_ROT(11, 0xf800f800) PL_RANK_ROT(12, 0xf000f000)
        PL_RANK_ROT(13, 0xe000e000) PL_RANK_ROT(14, 0xc000c000) PL_RANK_ROT(15, 0x80008000)
        : "=&v"(rk), "=&v"(tmp)
        : "v"(lo), "v"(hi)
        : "vcc");
    return rk;
}
#undef PL_RANK_ROT
#ifndef PL_SCL_RANK_SPLIT
#define PL_SCL_RANK_SPLIT 1  // 1: two independent borrow chains (VCC / SGPR pairs) instead of one (A/B r03u: 0.985 vs 0.991 ms)
#endif
// The same 15-rotation rank as two independent accumulations, interleaved: rotations 1..8 on the
// VCC borrow chain of rank16_subb, rotations 9..15 as VOP3 borrow chains through SGPR pairs on
// DPP-moved copies (5 VALU + 1 SALU each instead of 3 + 2): ~40 dependent steps instead of 75.
#define PL_RANK_ROT_A(r, m)                                                                   \
    "s_mov_b32 vcc_lo, " #m "\n\t"                                                          \
    "s_mov_b32 vcc_hi, " #m "\n\t"                                                          \
    "v_subb_co_u32_dpp %2, vcc, %7, %7, vcc row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t" \
    "v_subb_co_u32_dpp %2, vcc, %8, %8, vcc row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t" \
    "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n\t"
#define PL_RANK_ROT_B(r, m)                                                 \
    "v_mov_b32_dpp %3, %7 row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t" \
    "v_mov_b32_dpp %4, %8 row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t" \
    "v_subb_co_u32_e64 %3, %5, %3, %7, " #m "\n\t"                       \
    "v_subb_co_u32_e64 %4, %6, %4, %8, %5\n\t"                           \
    "v_addc_co_u32_e64 %1, %5, 0, %1, %6\n\t"
__device__ __forceinline__ int rank16_split(double cv) {
    const long long b = __double_as_longlong(cv);
    const int lo = (int)(b & 0xffffffffLL), hi = (int)(b >> 32);
    int ra, rb, ta, tl, th;
    uint64_t s1, s2;
    // static tie masks of rotations 9..15 (group lanes >= r under row_ror:r, every row)
    constexpr uint64_t m9 = 0xfe00fe00fe00fe00ull, m10 = 0xfc00fc00fc00fc00ull, m11 = 0xf800f800f800f800ull,
                       m12 = 0xf000f000f000f000ull, m13 = 0xe000e000e000e000ull, m14 = 0xc000c000c000c000ull,
                       m15 = 0x8000800080008000ull;
    asm volatile(
        "s_nop 1\n\t"
        "v_mov_b32 %0, 0\n\t"
        "v_mov_b32 %1, 0\n\t"
        PL_RANK_ROT_A(1, 0xfffefffe) PL_RANK_ROT_B(9, %9)
        PL_RANK_ROT_A(2, 0xfffcfffc) PL_RANK_ROT_B(10, %10)
        PL_RANK_ROT_A(3, 0xfff8fff8) PL_RANK_ROT_B(11, %11)
        PL_RANK_ROT_A(4, 0xfff0fff0) PL_RANK_ROT_B(12, %12)
        PL_RANK_ROT_A(5, 0xffe0ffe0) PL_RANK_ROT_B(13, %13)
        PL_RANK_ROT_A(6, 0xffc0ffc0) PL_RANK_ROT_B(14, %14)
        PL_RANK_ROT_A(7, 0xff80ff80) PL_RANK_ROT_B(15, %15)
        PL_RANK_ROT_A(8, 0xff00ff00)
        "v_add_u32 %0, %0, %1\n\t"
        : "=&v"(ra), "=&v"(rb), "=&v"(ta), "=&v"(tl), "=&v"(th), "=&s"(s1), "=&s"(s2)
        : "v"(lo), "v"(hi), "s"(m9), "s"(m10), "s"(m11), "s"(m12), "s"(m13), "s"(m14), "s"(m15)
        : "vcc");
    return ra;
}
#undef PL_RANK_ROT_A
#undef PL_RANK_ROT_B
#endif

template <int GW, int r>
__device__ __forceinline__ void rank_rot(double cv, int gl, int lane, int& rk) {
#if PL_SCL_RANK_SUBB
    if constexpr (GW == 16 && r == 1) {
        rk = rank16_subb(cv);
        return;
    }
#endif
#if PL_SCL_RANK_MASK
    if constexpr (GW == 16 && r < GW) {
        // row_ror:r -- group lane gl receives group lane (gl - r) mod 16, whose candidate index
        // is the lower one exactly when gl >= r: that tie mask is a constant per rotation
        const double v = dpp_d<0x120 + r>(cv);
        constexpr uint64_t tie = (uint64_t)((0xFFFFu << r) & 0xFFFFu) * 0x0001000100010001ull;
        const uint64_t lt = __builtin_amdgcn_ballot_w64(v < cv);
        const uint64_t eq = __builtin_amdgcn_ballot_w64(v == cv);
        rk = add_lane_bit(rk, lt | (eq & tie));
        rank_rot<GW, r + 1>(cv, gl, lane, rk);
        return;
    }
#endif
    if constexpr (r < GW) {
        double v;
        if constexpr (GW == 16) {
            v = dpp_d<0x120 + r>(cv);  // row_ror:r -- the 16-lane DPP row is the group
        } else if constexpr (GW == 4) {
            constexpr int q = ((0 + r) & 3) | (((1 + r) & 3) << 2) | (((2 + r) & 3) << 4) | (((3 + r) & 3) << 6);
            v = dpp_d<q>(cv);  // quad_perm rotation
        } else {
            v = bperm_d(cv, (lane & ~(GW - 1)) | ((gl + r) & (GW - 1)));
        }
        // source group lane of the rotation (DPP row_ror / quad_perm / bpermute), moved like
        // the value so the direction convention cannot matter
        int ci;
        if constexpr (GW == 16) ci = __builtin_amdgcn_mov_dpp(gl, 0x120 + r, 0xF, 0xF, true);
        else ci = (gl + r) & (GW - 1);
        rk += (v < cv || (v == cv && ci < gl)) ? 1 : 0;
        rank_rot<GW, r + 1>(cv, gl, lane, rk);
    }
}

// Element j of the stage-s node at position pos of one path, D stages below the channel,
// recomputed from the channel row (logits, negated here: polar_scl.py:219) and the path's
// partial sums -- used only for the node sums of pruned fast-SCL nodes above the stored stages.
template <int D, int FM>
__device__ double vread(const float* ch, const uint32_t* beta, int s, int pos, int j, double lmax) {
    if constexpr (D == 0) {
        return (double)(-1.0f * ch[j]);
    } else {
        const int h = 1 << s, pp = pos & ~(2 * h - 1);
        const double x = vread<D - 1, FM>(ch, beta, s + 1, pp, j, lmax);
        const double y = vread<D - 1, FM>(ch, beta, s + 1, pp, j + h, lmax);
        return pos == pp ? f_op<FM>(x, y, lmax) : g_op(x, y, getbit(beta, pp + j));
    }
}

// One codeword's state: LDS regions and its channel row.
struct Cw {
    double* A;        // [L][per] stage s (R <= s <= SS) of buffer b at A[b*per + 2^s - 2^R + j]
    uint32_t* beta;   // [L][W] partial sums by absolute position
    uint8_t* sptr;    // [L][SPS] owner buffer of stage s (s <= S)
    int* org_s;       // [L] subtree exchange: origin path
    uint32_t* ps_s;   // [L] subtree exchange: partial-sum word
    double* pm_s;     // [L] final metrics
    int* fail_s;      // [L] CRC failure flags
    double* sv;       // [2L] final sorted values
    int* sp;          // [2L] final sorted states
    const float* ch;  // [n] channel logits in global memory
};

struct St {
    unsigned char* smem;
    Lay y;
    const float* llr;
    double* vcache;  // exact f: this wave's leftmost-chain cache (chain_size(n, V) doubles per codeword), or null
    int64_t b0, bs;
    int n, S, W, SS, per;
    double lmax;
    __device__ __forceinline__ Cw cw(int c) const {
        unsigned char* base = smem + c * y.bytes;
        Cw w;
        w.A = reinterpret_cast<double*>(base + y.off_A);
        w.beta = reinterpret_cast<uint32_t*>(base + y.off_beta);
        w.sptr = base + y.off_sptr;
        w.org_s = reinterpret_cast<int*>(base + y.off_org);
        w.ps_s = reinterpret_cast<uint32_t*>(base + y.off_ps);
        w.pm_s = reinterpret_cast<double*>(base + y.off_pm);
        w.fail_s = reinterpret_cast<int*>(base + y.off_fail);
        w.sv = reinterpret_cast<double*>(base + y.off_sv);
        w.sp = reinterpret_cast<int*>(base + y.off_sp);
        int64_t row = b0 + c;
        if (row >= bs) row = bs - 1;  // a tail wave's missing codewords decode a copy, never stored
        w.ch = llr + row * n;
        return w;
    }
};

// Input element j of the stage-s node at pos, V levels below the channel, bottom-up in place:
// c[m] = negated channel element j + m 2^s (m < 2^V); level t (from the channel down) combines
// v[m] and v[m + 2^t] (m < 2^t) with f, or with g reading bit base[t] + m 2^s of the path
// (base[t] = start of the stage-(s+t+1) node + j) when the stage-(s+t) node is a right child.
// The same f/g operands as the recursion over the tree, so the same values.
template <int V, int FM>
__device__ __forceinline__ double vtree(const float* c, const uint32_t* bp, const int* base, uint32_t gmask, int hs,
                                        double lmax) {
    if constexpr (V == 0) {
        return (double)c[0];
    } else {
        constexpr int H = 1 << (V - 1);
        double v[H];
        {
            constexpr int t = V - 1;
            const bool g = (gmask >> t) & 1u;
#pragma unroll
            for (int m = 0; m < H; ++m) {
                const double x = (double)c[m], y = (double)c[m + H];
                v[m] = g ? g_op(x, y, getbit(bp, base[t] + m * hs)) : f_op<FM>(x, y, lmax);
            }
        }
#pragma unroll
        for (int t = V - 2; t >= 0; --t) {
            const int h = 1 << t;
            const bool g = (gmask >> t) & 1u;
#pragma unroll
            for (int m = 0; m < h; ++m)
                v[m] = g ? g_op(v[m], v[m + h], getbit(bp, base[t] + m * hs)) : f_op<FM>(v[m], v[m + h], lmax);
        }
        return v[0];
    }
}

// Virtual node of 64 (n = 1024, V = 4, h = 32): the input pair (x, y) = elements (j, j + 32) of
// the stage-6 node at pos, rebuilt bottom-up from the channel.  Level q (stage 6 + q) combines
// v[m] and v[m + 2^q], m < 2^q: f when the stage-(6+q) node is a left child, else g with bit j
// of partial-sum word wb[q] + 2m (x) or the next word (y) -- one 16-byte load brings the words
// of leaves m and m+1 for x and y.  The leading f levels (from the channel down to the first g)
// do not depend on the path: they are computed once per element, the rest once per path.
template <int q, int FM>
__device__ __forceinline__ void vlev_f(double* vx, double* vy, double lmax) {
    constexpr int h = 1 << q;
#pragma unroll
    for (int m = 0; m < h; ++m) {
        vx[m] = f_op<FM>(vx[m], vx[m + h], lmax);
        vy[m] = f_op<FM>(vy[m], vy[m + h], lmax);
    }
}
template <int q>
__device__ __forceinline__ void vlev_g(double* vx, double* vy, const uint32_t* wq, int j) {
    constexpr int h = 1 << q;
    if constexpr (h == 1) {
        const uint2 u2 = *reinterpret_cast<const uint2*>(wq);
        vx[0] = g_op(vx[0], vx[1], (u2.x >> j) & 1u);
        vy[0] = g_op(vy[0], vy[1], (u2.y >> j) & 1u);
    } else {
#pragma unroll
        for (int m = 0; m < h; m += 2) {
            const uint4 u4 = *reinterpret_cast<const uint4*>(wq + 2 * m);
            vx[m] = g_op(vx[m], vx[m + h], (u4.x >> j) & 1u);
            vy[m] = g_op(vy[m], vy[m + h], (u4.y >> j) & 1u);
            vx[m + 1] = g_op(vx[m + 1], vx[m + 1 + h], (u4.z >> j) & 1u);
            vy[m + 1] = g_op(vy[m + 1], vy[m + 1 + h], (u4.w >> j) & 1u);
        }
    }
}
template <int Q, int FM>
__device__ __forceinline__ void vlev_path(double* vx, double* vy, const uint32_t* bp, const int* wb, int j,
                                          uint32_t gmask, double lmax) {
    if constexpr (Q >= 0) {
        if ((gmask >> Q) & 1u) vlev_g<Q>(vx, vy, bp + wb[Q], j);
        else vlev_f<Q, FM>(vx, vy, lmax);
        vlev_path<Q - 1, FM>(vx, vy, bp, wb, j, gmask, lmax);
    }
}
template <int Q, int QE, int FM>  // per-path levels Q down to QE
__device__ __forceinline__ void vlev_range(double* vx, double* vy, const uint32_t* bp, const int* wb, int j,
                                           uint32_t gmask, double lmax) {
    if constexpr (Q >= QE && Q >= 0) {
        if ((gmask >> Q) & 1u) vlev_g<Q>(vx, vy, bp + wb[Q], j);
        else vlev_f<Q, FM>(vx, vy, lmax);
        vlev_range<Q - 1, QE, FM>(vx, vy, bp, wb, j, gmask, lmax);
    }
}
template <int Q, int QE, int FM>  // shared f levels Q down to QE
__device__ __forceinline__ void vlev_shared(double* vx, double* vy, double lmax) {
    if constexpr (Q >= QE) {
        vlev_f<Q, FM>(vx, vy, lmax);
        vlev_shared<Q - 1, QE, FM>(vx, vy, lmax);
    }
}

// The stage-6 values of the virtual node of 64 (n = 1024, V = 4) that the left pass (f into the
// stage-5 left child) computes from the channel, per (item, path) of this lane: the right pass (g
// into the right child) reads them back instead of rebuilding them from the channel.  A path's
// entry is found through the owner byte sptr[p][6] (written by the left pass, re-pointed with
// the other stage owners when paths fork), and lives in this lane's private memory: the lane that
// handles item (c, j) in one pass handles it in every pass.  Half the passes then cost one load
// and one g per path instead of 31 f/g.  Min-sum also keeps the stage-7 values (after the
// level that produces them, in the left pass of a stage-7 node's left child): the left pass of
// its right child then starts from them (one g per side and the f) instead of the channel.
#ifndef PL_SCL_VCACHE
#define PL_SCL_VCACHE 1
#endif
#ifndef PL_SCL_C7
#define PL_SCL_C7 1  // 1: min-sum caches the stage-7 values too (A/B r04i, one path per step: 0.942 vs
                     // 0.929 ms; with the batched loads, r04q: 0.868 vs 0.893 ms)
#endif
// The stage-7 cache at L <= 8 only: the wider lists' kernels spill with it (L = 16: 38 VGPRs).
template <int L, int FM>
constexpr bool c7_on() { return PL_SCL_C7 && FM == 0 && L <= 8; }
constexpr int kVcEntries = 32;  // (item, path) entries per lane: IT * L <= 32 (node_fg checks it)
template <int FM>
struct VCache {
    double2 v[kVcEntries];   // [it * L + path]: (x, y) = stage-6 elements (j, j + 32); IT * L <= 32
};
template <>
struct VCache<0> {  // min-sum
    double2 v[kVcEntries];
#if PL_SCL_C7
    double4 v7[kVcEntries];  // the stage-7 elements (j, j + 64 | j + 32, j + 96) of the same path
    int p7;          // start of the stage-7 node v7 belongs to (fast-SCL may prune the left pass
                     // that writes it: the right child's pass then recomputes); same in every lane
#endif
};

template <int L, int V, int NS, int FM>
__device__ __forceinline__ void vnode64(const St& t, const Cw& w, const float* cx, const float* cy, const int* wb,
                                        int j, uint32_t gmask, bool is_g, int pos, int ls, VCache<FM>* vc = nullptr,
                                        int it = 0, bool w7 = false) {
    constexpr int H = 1 << (V - 1);       // values per side after the channel level
    constexpr int NSS = (NS == V && c7_on<L, FM>()) ? V - 1 : NS;  // shared levels (C7: before the stage-7 boundary)
    constexpr int K = NSS > 0 ? (2 * H) >> NSS : 2 * H;  // per side after those shared levels
    double sx[K], sy[K];
    if constexpr (NS > 0) {
        double vx[H], vy[H];
#pragma unroll
        for (int m = 0; m < H; ++m) {
            vx[m] = f_op<FM>((double)cx[m], (double)cx[m + H], t.lmax);
            vy[m] = f_op<FM>((double)cy[m], (double)cy[m + H], t.lmax);
        }
        vlev_shared<V - 2, V - NSS, FM>(vx, vy, t.lmax);
#pragma unroll
        for (int m = 0; m < K; ++m) {
            sx[m] = vx[m];
            sy[m] = vy[m];
        }
    }
#pragma unroll 1
    for (int p = 0; p < L; ++p) {
        const uint32_t* bp = w.beta + p * t.W;
        double vx[H], vy[H];
        if constexpr (NS == 0) {  // the channel level is a g: per path
            const uint32_t* wq = bp + wb[V - 1];
#pragma unroll
            for (int m = 0; m < H; m += 2) {
                const uint4 u4 = *reinterpret_cast<const uint4*>(wq + 2 * m);
                vx[m] = g_op((double)cx[m], (double)cx[m + H], (u4.x >> j) & 1u);
                vy[m] = g_op((double)cy[m], (double)cy[m + H], (u4.y >> j) & 1u);
                vx[m + 1] = g_op((double)cx[m + 1], (double)cx[m + 1 + H], (u4.z >> j) & 1u);
                vy[m + 1] = g_op((double)cy[m + 1], (double)cy[m + 1 + H], (u4.w >> j) & 1u);
            }
            vlev_range<V - 2, 1, FM>(vx, vy, bp, wb, j, gmask, t.lmax);
        } else {
#pragma unroll
            for (int m = 0; m < K; ++m) {
                vx[m] = sx[m];
                vy[m] = sy[m];
            }
            vlev_range<V - NSS - 1, 1, FM>(vx, vy, bp, wb, j, gmask, t.lmax);
        }
        // the stage-7 values (levels above done): cached for the right child's left pass
#if PL_SCL_C7
        if (w7 && !PL_SCL_DIAG_VC_NOSTORE) vc->v7[it * L + p] = make_double4(vx[0], vx[1], vy[0], vy[1]);
#endif
        if constexpr (NSS == V) {  // every level shared: nothing per path
        } else if constexpr (NS == V) {  // C7: level 0 is the last shared f (same value for every path)
            vlev_f<0, FM>(vx, vy, t.lmax);
        } else {
            vlev_range<0, 0, FM>(vx, vy, bp, wb, j, gmask, t.lmax);
        }
        const double x = vx[0], y = vy[0];
        if (vc != nullptr && !PL_SCL_DIAG_VC_NOSTORE) vc->v[it * L + p] = make_double2(x, y);  // the left pass (is_g false)
        const double r = is_g ? g_op(x, y, getbit(bp, pos + j)) : f_op<FM>(x, y, t.lmax);
        w.A[p * t.per + (1 << ls) - (1 << R) + j] = r;
    }
}
// The right pass from the cache: per path, the owner's (x, y) and one g.  Every owner byte, cache
// entry and partial-sum word of the pass is loaded before the first g, so the private-memory loads
// (L2 latency) overlap instead of being paid once per path (r04n phase timing: 12.7k cycles per pass
// with one path per step).
#ifndef PL_SCL_VC_BATCH
#define PL_SCL_VC_BATCH 1
#endif
template <int L, int FM>
__device__ __forceinline__ void vnode64_cached(const St& t, const Cw& w, int j, int pos, int ls, const VCache<FM>& vc,
                                               int it) {
#if PL_SCL_VC_BATCH
    constexpr int B = L < 8 ? L : 8;  // paths per batch (registers: 6 per path)
#pragma unroll
    for (int p0 = 0; p0 < L; p0 += B) {
        int o[B];
        uint32_t wd[B];
#pragma unroll
        for (int q = 0; q < B; ++q) {
            o[q] = w.sptr[(p0 + q) * SPS + ls + 1];
            wd[q] = w.beta[(p0 + q) * t.W + ((pos + j) >> 5)];
        }
        double2 xy[B];
#pragma unroll
        for (int q = 0; q < B; ++q) xy[q] = vc.v[it * L + o[q]];
#pragma unroll
        for (int q = 0; q < B; ++q)
            w.A[(p0 + q) * t.per + (1 << ls) - (1 << R) + j] = g_op(xy[q].x, xy[q].y, (wd[q] >> ((pos + j) & 31)) & 1u);
    }
#else
#pragma unroll 1
    for (int p = 0; p < L; ++p) {
        const int o = w.sptr[p * SPS + ls + 1];
        const double2 xy = vc.v[it * L + o];
        w.A[p * t.per + (1 << ls) - (1 << R) + j] = g_op(xy.x, xy.y, getbit(w.beta + p * t.W, pos + j));
    }
#endif
}

// The left pass of a stage-7 node's right child (level 0 a g) from the stage-7 cache: per path,
// the owner's four values, one g per side, the f, and the stage-6 entry for the right pass.
#if PL_SCL_C7
template <int L>
__device__ __forceinline__ void vnode64_c7(const St& t, const Cw& w, int j, int pos, int ls, VCache<0>& vc, int it) {
    const int p7 = pos & ~127;  // start of the stage-7 node: the left child's partial sums
#if PL_SCL_VC_BATCH
    constexpr int B = L < 8 ? L : 8;  // paths per batch (registers: 10 per path)
#pragma unroll
    for (int p0 = 0; p0 < L; p0 += B) {
        double4 c[B];
        uint32_t wx[B], wy[B];
#pragma unroll
        for (int q = 0; q < B; ++q) {
            const uint32_t* bp = w.beta + (p0 + q) * t.W;
            c[q] = vc.v7[it * L + w.sptr[(p0 + q) * SPS + ls + 2]];
            wx[q] = bp[(p7 + j) >> 5];
            wy[q] = bp[(p7 + 32 + j) >> 5];
        }
#pragma unroll
        for (int q = 0; q < B; ++q) {
            const double x = g_op(c[q].x, c[q].y, (wx[q] >> ((p7 + j) & 31)) & 1u);
            const double y = g_op(c[q].z, c[q].w, (wy[q] >> ((p7 + 32 + j) & 31)) & 1u);
            if (!PL_SCL_DIAG_VC_NOSTORE) vc.v[it * L + p0 + q] = make_double2(x, y);
            w.A[(p0 + q) * t.per + (1 << ls) - (1 << R) + j] = f_ms(x, y, t.lmax);
        }
    }
#else
#pragma unroll 1
    for (int p = 0; p < L; ++p) {
        const uint32_t* bp = w.beta + p * t.W;
        const double4 c = vc.v7[it * L + w.sptr[p * SPS + ls + 2]];
        const double x = g_op(c.x, c.y, getbit(bp, p7 + j)), y = g_op(c.z, c.w, getbit(bp, p7 + 32 + j));
        if (!PL_SCL_DIAG_VC_NOSTORE) vc.v[it * L + p] = make_double2(x, y);
        w.A[p * t.per + (1 << ls) - (1 << R) + j] = f_ms(x, y, t.lmax);
    }
#endif
}
#endif

// One pass of a virtual node of 64 over the wave's (codeword, element) pairs; NS leading f
// levels (a per-pass constant, so each NS is its own loop).
template <int L, int V, int NS, int FM, int CPW>
__device__ void vvisit64(const St& t, int pos, bool is_g, int lane, const int* wb, uint32_t gmask, VCache<FM>* vc) {
    constexpr int NC = 1 << V, ls = 5, h = 32, hs = 64;
    static_assert((CPW * h + 63) / 64 * L <= kVcEntries, "VCache: items per lane x paths");
    if (vc != nullptr && is_g) {
#if PL_SCL_VC_BATCH
#pragma unroll
        for (int it = 0; it < (CPW * h + 63) / 64; ++it) {  // CPW * h = 32 at L = 32: half the lanes
            const int idx = lane + 64 * it;
            if (CPW * h % 64 == 0 || idx < CPW * h) vnode64_cached<L, FM>(t, t.cw(idx >> ls), idx & (h - 1), pos, ls, *vc, it);
        }
#else
#pragma unroll 1
        for (int idx = lane, it = 0; idx < CPW * h; idx += 64, ++it)
            vnode64_cached<L, FM>(t, t.cw(idx >> ls), idx & (h - 1), pos, ls, *vc, it);
#endif
        return;
    }
#if PL_SCL_C7
    if (c7_on<L, FM>() && vc != nullptr && (pos & 127) == 64 && vc->p7 == pos - 64) {  // right child of its stage-7 node
#pragma unroll
        for (int it = 0; it < (CPW * h + 63) / 64; ++it) {
            const int idx = lane + 64 * it;
            if (CPW * h % 64 == 0 || idx < CPW * h) vnode64_c7<L>(t, t.cw(idx >> ls), idx & (h - 1), pos, ls, *vc, it);
        }
        return;
    }
    const bool w7 = c7_on<L, FM>() && vc != nullptr && (pos & 127) == 0;  // a new stage-7 node
    if (w7) vc->p7 = pos;
#else
    const bool w7 = false;
#endif
    // channel rows addressed from the wave's first row (uniform base, 32-bit lane offsets)
    const float* ch0 = t.llr + t.b0 * t.n;
#if PL_SCL_VPF
    // software-pipelined by one element: the next element's 2 x 2^V channel values (L2) are in
    // flight while this one's paths are evaluated (CPW * h is a multiple of 64: uniform trip count)
    auto co_of = [&](int idx) {
        const int c = idx >> ls, j = idx & (h - 1);
        return (int)(t.b0 + c < t.bs ? c : t.bs - 1 - t.b0) * t.n + j;
    };
    float cx[NC], cy[NC];
    {
        const int co = co_of(lane);
#pragma unroll
        for (int m = 0; m < NC; ++m) {
            cx[m] = -1.0f * ch0[co + m * hs];
            cy[m] = -1.0f * ch0[co + h + m * hs];
        }
    }
#pragma unroll 1
    for (int idx = lane; idx < CPW * h; idx += 64) {
        const int c = idx >> ls, j = idx & (h - 1);
        const Cw w = t.cw(c);
        float nx[NC], ny[NC];
        if (idx + 64 < CPW * h) {
            const int co = co_of(idx + 64);
#pragma unroll
            for (int m = 0; m < NC; ++m) {
                nx[m] = -1.0f * ch0[co + m * hs];
                ny[m] = -1.0f * ch0[co + h + m * hs];
            }
        }
        vnode64<L, V, NS, FM>(t, w, cx, cy, wb, j, gmask, is_g, pos, ls);
#pragma unroll
        for (int m = 0; m < NC; ++m) {
            cx[m] = nx[m];
            cy[m] = ny[m];
        }
    }
#else
#pragma unroll 1
    for (int idx = lane, it = 0; idx < CPW * h; idx += 64, ++it) {
        const int c = idx >> ls, j = idx & (h - 1);
        const Cw w = t.cw(c);
        const int co = (int)(t.b0 + c < t.bs ? c : t.bs - 1 - t.b0) * t.n + j;
        float cx[NC], cy[NC];
#pragma unroll
        for (int m = 0; m < NC; ++m) {
            cx[m] = -1.0f * ch0[co + m * hs];
            cy[m] = -1.0f * ch0[co + h + m * hs];
        }
        vnode64<L, V, NS, FM>(t, w, cx, cy, wb, j, gmask, is_g, pos, ls, vc, it, w7);
    }
#endif
}

// One pass of a virtual node for the exact f (FM = 1, any V >= 1), where an f costs ~65 VALU and
// dominates: the leading f levels (from the channel down to the first g) are path-independent, so
// each lane evaluates them once per (codeword, element) -- from the workspace's leftmost-chain
// cache and four-outcome tables -- and only the levels below the first g once per path: 2.1x
// fewer f evaluations than the per-path recursion at n = 1024.  The per-path levels are unrolled
// blocks with compile-time register indices (vex_levels); at V = 4 only levels 1 and 0 can be f
// levels, so the f appears three times per path block.  (Until round 6 they were loops indexing
// register vectors with the uniform loop counter, which the backend lowered to compare-and-select
// chains over every entry.)  Level q (stage s + q) combines v[m] and v[m + 2^q], m < 2^q: f when
// the stage-(s+q) node is a left child, else g with bit base[q] + m 2^s of the path.  The same
// operands and operations as vtree(), so the same values.
#ifndef PL_SCL_VPF
#define PL_SCL_VPF 0  // 1: min-sum virtual passes load the next element's channel values ahead (A/B)
#endif
#ifndef PL_SCL_FEX_COMBO
#define PL_SCL_FEX_COMBO 1  // 1: the f level after the first per-path g from its four path-independent outcomes
#endif
template <int Q, typename F>
__device__ __forceinline__ void vex_levels(F& level) {  // level(Q), level(Q - 1), ..., level(0)
    if constexpr (Q >= 0) {
        level(std::integral_constant<int, Q>{});
        vex_levels<Q - 1>(level);
    }
}
#ifndef PL_SCL_FEX_INL
#define PL_SCL_FEX_INL 1  // 1: vvisit_ex inlined (its register blocks in the kernel's registers); 0: out of line (A/B r03i:
                          // callee register saves through scratch every pass, 4.10 vs 3.71 ms)
#endif
#if PL_SCL_FEX_INL
#define PL_FEX_PASS_ATTR __forceinline__
#else
#define PL_FEX_PASS_ATTR __noinline__
#endif
template <int L, int V, int CPW>
__device__ PL_FEX_PASS_ATTR void vvisit_ex(const float* __restrict__ llr, int64_t b0, int64_t bs, int n, int W, int per,
                                       double lmax, unsigned char* smem, int cw_bytes, int off_A, int off_beta,
                                       int s, int pos, int is_g, int lane, const double* __restrict__ vcache,
                                       VCache<1>* vc = nullptr, int off_sptr = 0) {
    // Out of line with scalar arguments only: the pass's register arrays are allocated apart from
    // the lane subtree's state (inlined, the two together spilled), and nothing goes through
    // scratch but the call's own register saves, once per pass.
    constexpr int NC = 1 << V, H = NC / 2;
    const int ls = s - 1, h = 1 << ls, hs = 1 << s;
    uint32_t gmask = 0u;  // level q is a g iff the stage-(s+q) node is a right child
    int bx[V], by[V];
#pragma unroll
    for (int q = 0; q < V; ++q) {
        const int st_ = s + q, pp = pos & ~((2 << st_) - 1);
        if ((pos & ~((1 << st_) - 1)) != pp) gmask |= 1u << q;
        bx[q] = pp;
        by[q] = pp + h;
    }
    int ns = 0;  // leading f levels (uniform)
    while (ns < V && ((gmask >> (V - 1 - ns)) & 1u) == 0u) ++ns;
    const float* ch0 = llr + b0 * n;
    // The pass's register blocks (wx, wy) are vector values, so the dynamic (uniform) indices of
    // the no-workspace fallback loops below stay in registers (as compare-and-select chains, slow
    // but rare: the product path always passes the workspace); the workspace paths and the
    // per-path levels use compile-time indices only.
    const int q1 = V - 1 - ns, h1 = 1 << (q1 > 0 ? q1 : 0), h2 = h1 >> 1;
    // First per-path level q1 (a g) followed by an f: each input of that f is one of two
    // path-independent sums (g with u = 0 or 1), so its four outcomes per element are computed
    // once and a path selects one by its two partial-sum bits -- 4 h2 f per side instead of h2 per
    // path (8 paths).  Same operands and operations as the per-path evaluation.
    const bool combo = PL_SCL_FEX_COMBO && ns < V && q1 >= 1 && ((gmask >> (q1 - 1)) & 1u) == 0u;
    typedef double wv __attribute__((ext_vector_type(NC)));
#pragma unroll 1
    for (int idx = lane, it = 0; idx < CPW * h; idx += 64, ++it) {
        const int c = idx >> ls, j = idx & (h - 1);
        unsigned char* base = smem + c * cw_bytes;
        double* A = reinterpret_cast<double*>(base + off_A);
        const uint32_t* beta = reinterpret_cast<const uint32_t*>(base + off_beta);
        if (vc != nullptr && is_g) {  // the right pass from the left pass's values (VCache)
            const uint8_t* sptr = base + off_sptr;
#if PL_SCL_VC_BATCH
            constexpr int B = L <= 8 ? L : 1;  // paths per batch (wider lists: one, as before)
#pragma unroll
            for (int p0 = 0; p0 < L; p0 += B) {
                double2 xy[B];
                uint32_t wd[B];
#pragma unroll
                for (int q = 0; q < B; ++q) {
                    xy[q] = vc->v[it * L + sptr[(p0 + q) * SPS + s]];
                    wd[q] = beta[(p0 + q) * W + ((pos + j) >> 5)];
                }
#pragma unroll
                for (int q = 0; q < B; ++q)
                    A[(p0 + q) * per + (1 << ls) - (1 << R) + j] =
                        g_op(xy[q].x, xy[q].y, (wd[q] >> ((pos + j) & 31)) & 1u);
            }
#else
#pragma unroll 1
            for (int p = 0; p < L; ++p) {
                const double2 xy = vc->v[it * L + sptr[p * SPS + s]];
                A[p * per + (1 << ls) - (1 << R) + j] = g_op(xy.x, xy.y, getbit(beta + p * W, pos + j));
            }
#endif
            continue;
        }
        VEX_T0;
        const int co = (int)(b0 + c < bs ? c : bs - 1 - b0) * n + j;
        // One register block per side holds what the path loop reads: the channel elements
        // j + m 2^s (x; y: + 2^(s-1)) as doubles when the channel level is per path (ns = 0), the
        // shared level-ns values (ns > 0), or the four-outcome table w[m + (2 b1 + b2) h2] (combo).
        double wx[NC], wy[NC];  // constant indices only: SROA keeps every entry its own register
        int hh = NC;
        const bool tab = combo && vcache != nullptr;  // the four-outcome table from the workspace
        if (tab) {
            const double* tb = vcache + c * cache_size(n, V) + combo_off(n, V, ns);
            auto load = [&](auto H2c) {
                constexpr int H2 = decltype(H2c)::value;
#pragma unroll
                for (int m = 0; m < H2; ++m) {
                    const double* ox = tb + 4 * (j + m * hs);
                    const double* oy = tb + 4 * (j + h + m * hs);
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        wx[m + k * H2] = ox[k];
                        wy[m + k * H2] = oy[k];
                    }
                }
            };
            if constexpr (H >= 8) {
                if (h2 == 4) load(std::integral_constant<int, (H >= 8 ? 4 : 1)>{});
            }
            if constexpr (H >= 4) {
                if (h2 == 2) load(std::integral_constant<int, (H >= 4 ? 2 : 1)>{});
            }
            if (h2 == 1) load(std::integral_constant<int, 1>{});
        } else if (ns == 0 || vcache == nullptr) {
#pragma unroll
            for (int m = 0; m < NC; ++m) {
                wx[m] = (double)(-1.0f * ch0[co + m * hs]);  // negated (polar_scl.py:219)
                wy[m] = (double)(-1.0f * ch0[co + h + m * hs]);
            }
        }
        if (tab) {
        } else if (ns > 0 && vcache != nullptr) {  // level ns of the leftmost chain: element j + m 2^s (x), + h (y)
            hh = NC >> ns;
            const double* cb = vcache + c * cache_size(n, V) + chain_off(n, ns) + j;
#pragma unroll
            for (int m = 0; m < H; ++m) {
                if (m < hh) {
                    wx[m] = cb[m * hs];
                    wy[m] = cb[h + m * hs];
                }
            }
        }
#if PL_SCL_PROF >= 2
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        VEX_MARK(0);
#endif
        if (vcache == nullptr && (ns > 0 || combo)) {
            // no workspace: the shared levels and the four-outcome step here, on vector copies
            // whose dynamic (uniform) indices stay in registers (compare-and-select chains)
            wv fx, fy;
#pragma unroll
            for (int m = 0; m < NC; ++m) {
                fx[m] = wx[m];
                fy[m] = wy[m];
            }
            if (ns > 0) {  // shared levels V-1 .. V-ns
#pragma unroll 1
                for (int q = V - 1; q >= V - ns; --q) {
                    hh = 1 << q;
#pragma unroll 1
                    for (int m = 0; m < hh; ++m) {
                        double a, b;
                        f_ex2(fx[m], fx[m + hh], fy[m], fy[m + hh], lmax, a, b);
                        fx[m] = a;
                        fy[m] = b;
                    }
                }
            }
            if (combo) {  // in place: block m reads and writes exactly the indices m + k h2, k < 4
#pragma unroll 1
                for (int m = 0; m < h2; ++m) {
                    const double xa = fx[m], xb = fx[m + h1], xc_ = fx[m + h2], xd = fx[m + h2 + h1];
                    const double ya = fy[m], yb = fy[m + h1], yc_ = fy[m + h2], yd = fy[m + h2 + h1];
                    const double gx0 = g_op(xa, xb, 0u), gx1 = g_op(xa, xb, 1u);
                    const double hx0 = g_op(xc_, xd, 0u), hx1 = g_op(xc_, xd, 1u);
                    const double gy0 = g_op(ya, yb, 0u), gy1 = g_op(ya, yb, 1u);
                    const double hy0 = g_op(yc_, yd, 0u), hy1 = g_op(yc_, yd, 1u);
                    double r0, r1, r2, r3, t0, t1, t2, t3;
                    f_ex2(gx0, hx0, gx0, hx1, lmax, r0, r1);
                    f_ex2(gx1, hx0, gx1, hx1, lmax, r2, r3);
                    f_ex2(gy0, hy0, gy0, hy1, lmax, t0, t1);
                    f_ex2(gy1, hy0, gy1, hy1, lmax, t2, t3);
                    fx[m] = r0;
                    fx[m + h2] = r1;
                    fx[m + 2 * h2] = r2;
                    fx[m + 3 * h2] = r3;
                    fy[m] = t0;
                    fy[m + h2] = t1;
                    fy[m + 2 * h2] = t2;
                    fy[m + 3 * h2] = t3;
                }
            }
#pragma unroll
            for (int m = 0; m < NC; ++m) {
                wx[m] = fx[m];
                wy[m] = fy[m];
            }
        }
        VEX_MARK(1);
        // Per-path levels with compile-time register indices: level q (2^q pairs) is its own
        // unrolled block, entered when q <= q0 (uniform), f or g by gmask (uniform).  (Round 6:
        // the loop form's dynamic indices into the register blocks lowered to compare-and-select
        // chains over every entry per access -- ~100 VALU per f pair, and the four-outcome pick
        // to a 16-way chain per value; A/B 2.03 -> 1.88 ms, bit-identical,
        // profiles/r06t_unr_ab_mysn.txt.)
#pragma unroll 1
        for (int p = 0; p < L; ++p) {
            const uint32_t* bp = beta + p * W;
            // an opaque per-path copy of the element index: the partial-sum addresses and shifts
            // derived from it are recomputed per path, not hoisted out of the loop (~50 VGPRs)
            int jo = j;
            asm volatile("" : "+v"(jo));
            double vx[H], vy[H];
            int q0;
            if (combo) {
                const int ox = bx[q1] + jo, oy = by[q1] + jo;
                auto pick = [&](auto H2c) {
                    constexpr int H2 = decltype(H2c)::value;
#pragma unroll
                    for (int m = 0; m < H2; ++m) {
                        const uint32_t bx1 = getbit(bp, ox + m * hs), bx2 = getbit(bp, ox + (m + H2) * hs);
                        const uint32_t by1 = getbit(bp, oy + m * hs), by2 = getbit(bp, oy + (m + H2) * hs);
                        double x0 = wx[m], x1 = wx[m + H2], x2 = wx[m + 2 * H2], x3 = wx[m + 3 * H2];
                        double y0 = wy[m], y1 = wy[m + H2], y2 = wy[m + 2 * H2], y3 = wy[m + 3 * H2];
                        asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
                        asm volatile("" : "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3));
                        vx[m] = bx1 ? (bx2 ? x3 : x2) : (bx2 ? x1 : x0);
                        vy[m] = by1 ? (by2 ? y3 : y2) : (by2 ? y1 : y0);
                    }
                };
                if constexpr (H >= 8) {
                    if (h2 == 4) pick(std::integral_constant<int, (H >= 8 ? 4 : 1)>{});
                }
                if constexpr (H >= 4) {
                    if (h2 == 2) pick(std::integral_constant<int, (H >= 4 ? 2 : 1)>{});
                }
                if (h2 == 1) pick(std::integral_constant<int, 1>{});
                q0 = q1 - 2;
            } else if (ns == 0) {  // the channel level is a g
#pragma unroll
                for (int m = 0; m < H; ++m) {
                    vx[m] = g_op(wx[m], wx[m + H], getbit(bp, bx[V - 1] + jo + m * hs));
                    vy[m] = g_op(wy[m], wy[m + H], getbit(bp, by[V - 1] + jo + m * hs));
                }
                q0 = V - 2;
            } else {
#pragma unroll
                for (int m = 0; m < H; ++m) {  // entries past hh are never read
                    vx[m] = wx[m];
                    vy[m] = wy[m];
                }
                q0 = V - 1 - ns;
            }
            auto level = [&](auto Qc) {
                constexpr int Q = decltype(Qc)::value, HQ = 1 << Q;
                if (Q > q0) return;
                const int ox = bx[Q] + jo, oy = by[Q] + jo;
                // with the four-outcome step, a per-path f level lies at least two levels below
                // the first per-path g (q1 <= V - 1): level V - 2 is always a g
                if (((gmask >> Q) & 1u) || (PL_SCL_FEX_COMBO && Q > V - 3)) {
#pragma unroll
                    for (int m = 0; m < HQ; ++m) {
                        vx[m] = g_op(vx[m], vx[m + HQ], getbit(bp, ox + m * hs));
                        vy[m] = g_op(vy[m], vy[m + HQ], getbit(bp, oy + m * hs));
                    }
                } else {
#pragma unroll
                    for (int m = 0; m < HQ; ++m) {
                        f_ex2(vx[m], vx[m + HQ], vy[m], vy[m + HQ], lmax, vx[m], vy[m]);
                    }
                }
            };
            vex_levels<V - 2>(level);
            const double x = vx[0], y = vy[0];
            if (vc != nullptr) vc->v[it * L + p] = make_double2(x, y);  // the left pass
            const double r = is_g ? g_op(x, y, getbit(bp, pos + jo)) : f_ex(x, y, lmax);
            A[p * per + (1 << ls) - (1 << R) + j] = r;
        }
        VEX_MARK(2);
    }
}

// Upper-tree node at stage s (> R), position pos: f (or g) of its input into the stage-(s-1)
// buffers of every path of every codeword (s-1 <= SS), wave-parallel over (codeword, path,
// element).  When the input is virtual (s = SS + 1, V stages below the channel) each lane keeps
// one (codeword, element) and loops over the paths, so the 2 x 2^V channel values it needs are
// read once, not once per path (lanes idle when the node has fewer than 64 / CPW elements).
// Stored-stage pass of node_fg with the stage size a compile-time constant (2^LS outputs per
// path; CPW * L = 32 (codeword, path) pairs, so 2^(LS-1) elements per lane): the owner pointers,
// operands and partial-sum words of up to 8 elements per lane are loaded before any result is
// stored, so a pass waits for ~2 LDS round trips instead of 3 per element (the stores could alias
// the loads as far as the compiler knows, which kept the runtime-bounded loop serial).
template <int L, int FM, int CPW, int LS>
__device__ __forceinline__ void node_fg_st(const St& t, int pos, bool is_g, int lane) {
    constexpr int LL = ilog2(L), h = 1 << LS, total = CPW * L * h, IT = (total + 63) / 64;
    constexpr int CH = IT < PL_SCL_ST_CH ? IT : PL_SCL_ST_CH;
    const int s = LS + 1;
    asm volatile("" : "+v"(lane));  // opaque per call: keeps the per-lane addresses from being
                                    // hoisted out of the decoder loop (they spilled the subtree)
#pragma unroll
    for (int c0 = 0; c0 < IT; c0 += CH) {
        double x[CH], y[CH];
        uint32_t wb[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int idx = (c0 + u) * 64 + lane;
            if (total % 64 == 0 || idx < total) {
                const int c = idx >> (LL + LS), p = (idx >> LS) & (L - 1), j = idx & (h - 1);
                const Cw w = t.cw(c);
                const double* in = w.A + w.sptr[p * SPS + s] * t.per + (1 << s) - (1 << R);
                x[u] = in[j];
                y[u] = in[j + h];
                wb[u] = is_g ? w.beta[p * t.W + ((pos + j) >> 5)] : 0u;
            }
        }
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int idx = (c0 + u) * 64 + lane;
            if (total % 64 == 0 || idx < total) {
                const int c = idx >> (LL + LS), p = (idx >> LS) & (L - 1), j = idx & (h - 1);
                const Cw w = t.cw(c);
                const double r = is_g ? g_op(x[u], y[u], (wb[u] >> ((pos + j) & 31)) & 1u)
                                      : f_op<FM>(x[u], y[u], t.lmax);
                w.A[p * t.per + (1 << LS) - (1 << R) + j] = r;
            }
        }
    }
}

template <int L, int V, int FM, int CPW>
__device__ void node_fg(const St& t, int s, int pos, bool is_g, int lane, VCache<FM>* vc) {
    constexpr int LL = ilog2(L);
    const int ls = s - 1, h = 1 << ls;
    // the per-lane cache holds kVcEntries (item, path) entries.  Release builds run pick_v's V,
    // whose virtual nodes have h <= 32 (S = 10: V = 4; S = 9: V = 3; below: h = 16), i.e. at most
    // CPW * 32 / 64 * L = 16 entries.  Development builds can put larger nodes on the virtual path
    // (PL_SCL_VIRTUAL below pick_v's V): such a pass runs uncached -- the left and right passes of
    // a node share h, so both see the same decision.  (A runtime check in release builds changed
    // the exact-f kernels' register allocation: 84 VGPR spills.)
#if PL_DEV
    if (vc != nullptr && ((CPW * h + 63) / 64) * L > kVcEntries) vc = nullptr;
#endif
    if (PL_SCL_DIAG_SKIP_V && s > t.SS) {
    } else if (PL_SCL_DIAG_SKIP_ST && s <= t.SS) {
    } else if (PL_SCL_ST_UNROLL && FM == 0 && s <= t.SS && ls <= R + 1) {  // exact f: spills (7.7 -> 11.2 ms)
        if (ls == R) node_fg_st<L, FM, CPW, R>(t, pos, is_g, lane);
        else node_fg_st<L, FM, CPW, R + 1>(t, pos, is_g, lane);
    } else if (FM == 1 && s <= t.SS && !is_g && (CPW * L * h) % 128 == 0) {
        // exact f, stored stage: two elements per lane per step, their f chains interleaved
        const int total = CPW * L * h;
        for (int i0 = lane; i0 < total; i0 += 128) {
            double x[2], y[2], r[2];
            double* o[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int idx = i0 + 64 * u;
                const int c = idx >> (LL + ls), p = (idx >> ls) & (L - 1), j = idx & (h - 1);
                const Cw w = t.cw(c);
                const double* in = w.A + w.sptr[p * SPS + s] * t.per + (1 << s) - (1 << R);
                x[u] = in[j];
                y[u] = in[j + h];
                o[u] = w.A + p * t.per + (1 << ls) - (1 << R) + j;
            }
            f_ex2(x[0], y[0], x[1], y[1], t.lmax, r[0], r[1]);
            *o[0] = r[0];
            *o[1] = r[1];
        }
    } else if (s <= t.SS) {
        const int total = CPW * L * h;
        for (int idx = lane; idx < total; idx += 64) {
            const int c = idx >> (LL + ls), p = (idx >> ls) & (L - 1), j = idx & (h - 1);
            const Cw w = t.cw(c);
            const uint32_t* bp = w.beta + p * t.W;
            const double* in = w.A + w.sptr[p * SPS + s] * t.per + (1 << s) - (1 << R);
            const double x = in[j], y = in[j + h];
            const double r = is_g ? g_op(x, y, getbit(bp, pos + j)) : f_op<FM>(x, y, t.lmax);
            w.A[p * t.per + (1 << ls) - (1 << R) + j] = r;
        }
    } else {
        constexpr int NC = 1 << V;
        const int hs = 1 << s;
        uint32_t gmask = 0u;  // level t is a g iff the stage-(s+t) node is a right child
        int bx[V > 0 ? V : 1], by[V > 0 ? V : 1];
#pragma unroll
        for (int q = 0; q < V; ++q) {
            const int st_ = s + q, pp = pos & ~((2 << st_) - 1);
            if ((pos & ~((1 << st_) - 1)) != pp) gmask |= 1u << q;
            bx[q] = pp;
            by[q] = pp + h;
        }
        if constexpr (V == 4 && FM == 0) {  // pick_v: V = 4 only at n = 1024 (node of 64); exact f:
            // the generic loop below (inlining 5 variants of the exp/log f spills heavily)
            int wb[V];
#pragma unroll
            for (int q = 0; q < V; ++q) wb[q] = bx[q] >> 5;  // multiples of 4 words: aligned
            // leading f levels from the channel down: path-independent
            const int ns = (gmask & 8u) ? 0 : (gmask & 4u) ? 1 : (gmask & 2u) ? 2 : (gmask & 1u) ? 3 : 4;
            switch (ns) {
                case 0: vvisit64<L, V, 0, FM, CPW>(t, pos, is_g, lane, wb, gmask, vc); break;
                case 1: vvisit64<L, V, 1, FM, CPW>(t, pos, is_g, lane, wb, gmask, vc); break;
                case 2: vvisit64<L, V, 2, FM, CPW>(t, pos, is_g, lane, wb, gmask, vc); break;
                case 3: vvisit64<L, V, 3, FM, CPW>(t, pos, is_g, lane, wb, gmask, vc); break;
                default: vvisit64<L, V, 4, FM, CPW>(t, pos, is_g, lane, wb, gmask, vc); break;
            }
        } else if constexpr (FM == 1 && V >= 1 && PL_SCL_FEX_HOIST) {
            vvisit_ex<L, V, CPW>(t.llr, t.b0, t.bs, t.n, t.W, t.per, t.lmax, t.smem, t.y.bytes, t.y.off_A,
                                 t.y.off_beta, s, pos, is_g ? 1 : 0, lane, t.vcache, vc, t.y.off_sptr);
        } else {
        // channel rows addressed from the wave's first row (uniform base, 32-bit lane offsets)
        const float* ch0 = t.llr + t.b0 * t.n;
#pragma unroll 1
        for (int idx = lane; idx < CPW * h; idx += 64) {
            const int c = idx >> ls, j = idx & (h - 1);
            const Cw w = t.cw(c);
            const int co = (int)(t.b0 + c < t.bs ? c : t.bs - 1 - t.b0) * t.n + j;
            float cx[NC], cy[NC];
#pragma unroll
            for (int m = 0; m < NC; ++m) {
                cx[m] = -1.0f * ch0[co + m * hs];
                cy[m] = -1.0f * ch0[co + h + m * hs];
            }
            int basex[V > 0 ? V : 1], basey[V > 0 ? V : 1];
#pragma unroll
            for (int q = 0; q < V; ++q) {
                basex[q] = bx[q] + j;
                basey[q] = by[q] + j;
            }

#pragma unroll 1
            for (int p = 0; p < L; ++p) {
                const uint32_t* bp = w.beta + p * t.W;
                // opaque per-iteration copies: the 2 (2^V - 1) bit addresses are recomputed per
                // path instead of being hoisted out of the loop (register pressure, occupancy)
                int bxp[V > 0 ? V : 1], byp[V > 0 ? V : 1];
#pragma unroll
                for (int q = 0; q < V; ++q) {
                    bxp[q] = basex[q];
                    byp[q] = basey[q];
                    asm volatile("" : "+v"(bxp[q]), "+v"(byp[q]));
                }
                const double x = vtree<V, FM>(cx, bp, bxp, gmask, hs, t.lmax);
                const double y = vtree<V, FM>(cy, bp, byp, gmask, hs, t.lmax);
                const double r = is_g ? g_op(x, y, getbit(bp, pos + j)) : f_op<FM>(x, y, t.lmax);
                w.A[p * t.per + (1 << ls) - (1 << R) + j] = r;
            }
        }
        }
    }
    if (lane < CPW * L) {
        uint8_t* sp = t.cw(lane >> LL).sptr + (lane & (L - 1)) * SPS;
        sp[ls] = (uint8_t)(lane & (L - 1));
        // the left pass of a cached virtual node: each path now owns its own stage-6 cache entry
        if (vc != nullptr && !is_g && s > t.SS) {
            sp[s] = (uint8_t)(lane & (L - 1));
            if (c7_on<L, FM>() && V == 4 && (pos & 127) == 0) sp[s + 1] = (uint8_t)(lane & (L - 1));
        }
    }
    __syncthreads();
}

// beta[pos, pos+h) ^= beta[pos+h, pos+2h) for every path of every codeword, h = 2^(s-1): word
// XORs for h >= 32, in-word bit ops below.
template <int L, int CPW>
__device__ void combine_upper(const St& t, int s, int pos, int lane) {
    constexpr int LL = ilog2(L);
    const int h = 1 << (s - 1);
    if (h >= 32) {
        const int lhw = s - 6, hw = 1 << lhw, w0 = pos >> 5;
        for (int idx = lane; idx < CPW * L * hw; idx += 64) {
            const int c = idx >> (LL + lhw), p = (idx >> lhw) & (L - 1), w = idx & (hw - 1);
            uint32_t* b = t.cw(c).beta + p * t.W;
            b[w0 + w] ^= b[w0 + hw + w];
        }
    } else if (lane < CPW * L) {
        uint32_t* b = t.cw(lane >> LL).beta + (lane & (L - 1)) * t.W + (pos >> 5);
        *b ^= (*b >> h) & (((1u << h) - 1u) << (pos & 31));
    }
    __syncthreads();
}

// ---- lane-local subtree --------------------------------------------------------------------
// st[2^s - 1 + j] = element j of the stage-s buffer (s < R).
constexpr int IDX(int s) { return (1 << s) - 1; }

// out[j] = f(in[j], in[j + h]), j < h.  Exact f (FM = 1): the path lane and its shadow hold the
// same stage buffers, so each evaluates half of the span (the path lane j < h/2, the shadow the
// rest, two at a time where it can: interleaved chains) and takes the other half from its partner
// (lane ^ L) -- half the f evaluations of the lane subtree, whose values are unchanged.  MEM: the
// input is the stage-R region in LDS, addressed per lane; otherwise registers, selected per lane.
#ifndef PL_SCL_FEX_SPLIT
#define PL_SCL_FEX_SPLIT 1
#endif
template <int h, int FM, int L, bool MEM>
__device__ __forceinline__ void f_span(const double* in, double* out, double lmax) {
    if constexpr (FM == 1 && h >= 2 && PL_SCL_FEX_SPLIT) {
        constexpr int q = h / 2;
        const int lane = threadIdx.x;
        const bool hi = (lane & L) != 0;
        double a[q], b[q], r[q];
        if constexpr (MEM) {
            const double* src = in + (hi ? q : 0);
#pragma unroll
            for (int j = 0; j < q; ++j) {
                a[j] = src[j];
                b[j] = src[j + h];
            }
        } else {
#pragma unroll
            for (int j = 0; j < q; ++j) {
                // selected as values (opaque to the compiler: a select of array addresses would put
                // the stage buffers in scratch)
                double a0 = in[j], a1 = in[j + q], b0 = in[j + h], b1 = in[j + q + h];
                asm("" : "+v"(a0), "+v"(a1), "+v"(b0), "+v"(b1));
                a[j] = hi ? a1 : a0;
                b[j] = hi ? b1 : b0;
            }
        }
        if constexpr (q == 1) {
            r[0] = f_ex(a[0], b[0], lmax);
        } else {
#pragma unroll
            for (int j = 0; j < q; j += 2) f_ex2(a[j], b[j], a[j + 1], b[j + 1], lmax, r[j], r[j + 1]);
        }
#pragma unroll
        for (int j = 0; j < q; ++j) {
            const double o = half_xchg<L>(r[j], lane);
            out[j] = hi ? o : r[j];
            out[j + q] = hi ? r[j] : o;
        }
    } else if constexpr (FM == 1 && h >= 2) {
#pragma unroll
        for (int j = 0; j < h; j += 2) {
            double a, b;
            f_ex2(in[j], in[j + h], in[j + 1], in[j + 1 + h], lmax, a, b);
            out[j] = a;
            out[j + 1] = b;
        }
    } else {
#pragma unroll
        for (int j = 0; j < h; ++j) out[j] = f_op<FM>(in[j], in[j + h], lmax);
    }
}

template <int s, int FM, int L>
__device__ __forceinline__ void f_down(double* st, double lmax) {
    if constexpr (s >= 1) {
        constexpr int h = 1 << (s - 1);
        f_span<h, FM, L, false>(st + IDX(s), st + IDX(s - 1), lmax);
        f_down<s - 1, FM, L>(st, lmax);
    }
}

__device__ __forceinline__ void load_group_fence(int j) {
#if PL_SCL_LOADGRP > 0
    if ((j + 1) % PL_SCL_LOADGRP == 0) __builtin_amdgcn_sched_barrier(0);
#else
    (void)j;
#endif
}

// Leaf i (> 0) with tz = ctz(i) trailing zeros: g at stage tz+1 into stage tz, then f down.
template <int tz, int FM, int L>
__device__ __forceinline__ void g_step(const double* inA, double* st, uint32_t ps, int i, double lmax) {
    constexpr int h = 1 << tz;
    const int p0 = i - h;  // start of the left sibling, whose partial sums g consumes
#pragma unroll
    for (int j = 0; j < h; ++j) {
        double x, y;
        if constexpr (tz + 1 == R) {
            x = inA[j];
            y = inA[j + h];
        } else {
            x = st[IDX(tz + 1) + j];
            y = st[IDX(tz + 1) + j + h];
        }
        st[IDX(tz) + j] = g_op(x, y, (ps >> (p0 + j)) & 1u);
        if constexpr (tz + 1 == R) load_group_fence(j);
    }
    f_down<tz, FM, L>(st, lmax);
}

// g at stage tz+1 into stage tz for leaf i (tz = ctz(i)), without descending
template <int tz>
__device__ __forceinline__ void g_only(const double* inA, double* st, uint32_t ps, int i) {
    constexpr int h = 1 << tz;
    const int p0 = i - h;
#pragma unroll
    for (int j = 0; j < h; ++j) {
        double x, y;
        if constexpr (tz + 1 == R) {
            x = inA[j];
            y = inA[j + h];
        } else {
            x = st[IDX(tz + 1) + j];
            y = st[IDX(tz + 1) + j + h];
        }
        st[IDX(tz) + j] = g_op(x, y, (ps >> (p0 + j)) & 1u);
    }
}

template <int FM, int L>
__device__ __forceinline__ void leaf_llr(const double* inA, double* st, uint32_t ps, int i, double lmax) {
    if (i == 0) {
        constexpr int h = T / 2;
        if constexpr (FM == 1) {
            f_span<h, FM, L, true>(inA, st + IDX(R - 1), lmax);
        } else {
#pragma unroll
            for (int j = 0; j < h; ++j) {
                st[IDX(R - 1) + j] = f_op<FM>(inA[j], inA[j + h], lmax);
                load_group_fence(j);
            }
        }
        f_down<R - 1, FM, L>(st, lmax);
        return;
    }
    switch (__builtin_ctz(i)) {
        case 0: g_step<0, FM, L>(inA, st, ps, i, lmax); break;
        case 1: g_step<1, FM, L>(inA, st, ps, i, lmax); break;
        case 2: g_step<2, FM, L>(inA, st, ps, i, lmax); break;
        case 3: g_step<3, FM, L>(inA, st, ps, i, lmax); break;
        default: g_step<R - 1, FM, L>(inA, st, ps, i, lmax); break;
    }
}

// Pull the live stage buffers (left half of their node at leaf i) from lane src.
template <int s>
__device__ __forceinline__ void pull_live(double* st, int i, int src) {
    if constexpr (s >= 1) {
        if (((i >> (s - 1)) & 1) == 0) {
#pragma unroll
            for (int j = 0; j < (1 << s); ++j) st[IDX(s) + j] = bperm_d(st[IDX(s) + j], src);
        }
        pull_live<s - 1>(st, i, src);
    }
}

// Selection by push (2L = 16): every candidate lane holds the whole state of its path (path and
// shadow lanes mirror each other), so after ranking it sends that state -- metric, partial sums
// with its own bit, origin and the live stage buffers -- straight to the group lane of its rank
// with ds_permute, and each shadow lane L..2L-1 then copies its path lane (gl - L) in one DPP row
// rotation by L restricted to the upper banks.  One LDS round trip per information leaf instead of
// three (push the parent code, copy it to the shadows, pull the parent's state); the same values.
// A/B r04r (min-sum, L = 8): 0.858 vs 0.864 ms.
#ifndef PL_SCL_PUSH
#define PL_SCL_PUSH 1
#endif
#ifndef PL_SCL_PUSH_DPERM
#define PL_SCL_PUSH_DPERM 0  // 1: the shadow copies by a second ds_permute to slot (rank + L) mod 2L instead of DPP
#endif
template <int L>
__device__ __forceinline__ int push_i(int v, int dst) {
    static_assert(L == 8, "push selection: 2L = 16 (one DPP row per codeword)");
#if PL_SCL_PUSH_DPERM
    // dst2 = the group lane L slots away (a permutation too): slot >= L receives the candidate of
    // rank slot - L, its path lane's
    const int dst2 = dst ^ (L << 2);
    const int r = __builtin_amdgcn_ds_permute(dst, v), r2 = __builtin_amdgcn_ds_permute(dst2, v);
    return (threadIdx.x & L) ? r2 : r;
#else
    const int r = __builtin_amdgcn_ds_permute(dst, v);
    return __builtin_amdgcn_update_dpp(r, r, 0x120 + L, 0xF, 0xC, false);  // row_ror:8, lanes 8..15 of each row
#endif
}
template <int L>
__device__ __forceinline__ double push_d(double v, int dst) {
    const long long b = __double_as_longlong(v);
    const int lo = push_i<L>((int)(b & 0xffffffffLL), dst), hi = push_i<L>((int)(b >> 32), dst);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// A live stage-s buffer whose parent stage s+1 is live too is the f of the parent's (its node is
// the left child, and neither buffer has changed since the node began): it is recomputed from the
// moved parent instead of moved (PL_SCL_PUSH_REFM), which halves the values moved per information
// leaf on average (4 doubles instead of 7); the same f, so the same values (A/B r04v: 0.847 vs 0.850 ms).
#ifndef PL_SCL_PUSH_REFM
#define PL_SCL_PUSH_REFM 1
#endif
// PL_SCL_PUSH == 2: one ds_permute sends each candidate's lane index to the slot of its rank, a
// DPP row rotation gives the shadow slots their path slot's source, and every value is then pulled
// (ds_bpermute) from that source lane -- two round trips, one forward permute (A/B r04x: 0.848
// vs 0.850 ms, within noise; a second forward permute for the shadows instead of the DPP copy,
// PL_SCL_PUSH_DPERM: 0.989 ms).
template <int L>
__device__ __forceinline__ int pull_src(int gl_lane, int dst) {
    const int r = __builtin_amdgcn_ds_permute(dst, gl_lane);
    return __builtin_amdgcn_update_dpp(r, r, 0x120 + L, 0xF, 0xC, false);
}
template <int L, int FM, int s>
__device__ __forceinline__ void pull2_live(double* st, int i, int src, double lmax) {
    if constexpr (s >= 1) {
        if (((i >> (s - 1)) & 1) == 0) {
            if (PL_SCL_PUSH_REFM && s + 1 < R && ((i >> s) & 1) == 0) {
                constexpr int h = 1 << s, sp = s + 1 < R ? s + 1 : s;
#pragma unroll
                for (int j = 0; j < h; ++j) st[IDX(s) + j] = f_op<FM>(st[IDX(sp) + j], st[IDX(sp) + j + h], lmax);
            } else {
#pragma unroll
                for (int j = 0; j < (1 << s); ++j) st[IDX(s) + j] = bperm_d(st[IDX(s) + j], src);
            }
        }
        pull2_live<L, FM, s - 1>(st, i, src, lmax);
    }
}
template <int L, int FM, int s>
__device__ __forceinline__ void push_live(double* st, int i, int dst, double lmax) {
    if constexpr (s >= 1) {
        if (((i >> (s - 1)) & 1) == 0) {
            if (PL_SCL_PUSH_REFM && s + 1 < R && ((i >> s) & 1) == 0) {
                constexpr int h = 1 << s, sp = s + 1 < R ? s + 1 : s;
#pragma unroll
                for (int j = 0; j < h; ++j) st[IDX(s) + j] = f_op<FM>(st[IDX(sp) + j], st[IDX(sp) + j + h], lmax);
            } else {
#pragma unroll
                for (int j = 0; j < (1 << s); ++j) st[IDX(s) + j] = push_d<L>(st[IDX(s) + j], dst);
            }
        }
        push_live<L, FM, s - 1>(st, i, dst, lmax);
    }
}

// Selection by speculative push (PL_SCL_SPEC; 2L = 16: the L = 8 min-sum push above, and
// select_2l's permute for the exact-f and fast-SCL kernels).  The push waits for the rank; the
// round-5 rank from the metrics' high words also waited for its permutation check -- a chain of
// five DPP ORs, a compare and a wave-uniform branch between the rank and the first ds_permute,
// ~0.04 ms of the bench kernel on its own (r05w_scl_fb2_ab.txt).  Here the rank is taken on a
// 32-bit key that is UNIQUE in the row, so it is always a permutation and every candidate is pushed
// at once; the order is checked afterwards, on the pushed metrics, while the other pushes are
// still in flight (same-process A/B on the bench's AWGN input, profiles/r06a/r06b_scl_spec_ab*.txt:
// 0.836 -> 0.797 ms min-sum, 2.070 -> 2.049 ms my_sn exact f + fast-SCL):
//   * key = 6 exponent bits (from 2^-44) and the top 22 mantissa bits of the metric, then the group
//     lane in the low 4 bits.  In [2^-44, 2^20) the key is non-decreasing in the metric, so keys
//     order the candidates like (metric, index) unless two metrics differ below the key's
//     resolution (2^-22 relative; mostly metrics a few ulps apart: ~0.7 % of a codeword's
//     information leaves at 2 dB, CPU count on the oracle); equal metrics -- the common tie, LLRs
//     of exactly 0 and the dead paths' equal metrics -- have equal key bits and keep the index order;
//   * after the push slot s holds the candidate of key rank s; the order is the stable (metric,
//     index) order iff every slot's metric is >= its left neighbour's (64-bit compare, one DPP
//     row shift per word): equal keys are in index order, so equal metrics are too;
//   * if any row of the wave fails, the pushed candidates are ranked again by the full 64-bit
//     stable rank (rank16_subb, the slot as the index -- equal metrics are in candidate order in
//     the slots) and pushed once more; then the shadow slots copy their path slot as before.
// Same selection, same values as the other forms (every SCL parity test runs this kernel).
#ifndef PL_SCL_SPEC
#define PL_SCL_SPEC 1
#endif
__device__ __forceinline__ uint32_t rank_key16(double cv, int gl) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(cv);
    // bits 57..26 of the metric's bits minus 979 << 52: in range (2^-44 <= metric < 2^20) the 6
    // exponent bits above 979 and 26 mantissa bits; out of range the key wraps (not monotone: the
    // order check below catches it).  The low 4 bits are the group lane: every key is unique.
    const uint32_t he = (uint32_t)(b >> 32) - (979u << 20);
    const uint32_t k = __builtin_amdgcn_alignbit(he, (uint32_t)(b & 0xffffffffull), 26);
    uint32_t r;
    asm("v_and_or_b32 %0, %1, -16, %2" : "=v"(r) : "v"(k), "v"(gl));
    return r;
}
#define PL_RANK_ROT_K(r)                                                                     \
    "v_sub_co_u32_dpp %1, vcc, %2, %2 row_ror:" #r " row_mask:0xf bank_mask:0xf\n\t" \
    "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n\t"
// rank of a unique key in its 16-lane row: per rotation one DPP subtract (borrow = the rotated key
// is smaller) and one carry add
__device__ __forceinline__ int rank16_key(uint32_t key) {
    int rk, tmp;
    asm volatile(
        "s_nop 1\n\t"  // the DPP source was just written by a VALU
        "v_sub_co_u32_dpp %1, vcc, %2, %2 row_ror:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_e64 %0, 0, 1, vcc\n\t"
        PL_RANK_ROT_K(2) PL_RANK_ROT_K(3) PL_RANK_ROT_K(4) PL_RANK_ROT_K(5)
        PL_RANK_ROT_K(6) PL_RANK_ROT_K(7) PL_RANK_ROT_K(8) PL_RANK_ROT_K(9) PL_RANK_ROT_K(10)
        PL_RANK_ROT_K(11) PL_RANK_ROT_K(12) PL_RANK_ROT_K(13) PL_RANK_ROT_K(14) PL_RANK_ROT_K(15)
        : "=&v"(rk), "=&v"(tmp)
        : "v"(key)
        : "vcc");
    return rk;
}
#undef PL_RANK_ROT_K
__device__ __forceinline__ double push_raw_d(double v, int dst) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_permute(dst, (int)(b & 0xffffffffLL));
    const int hi = __builtin_amdgcn_ds_permute(dst, (int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int L>
__device__ __forceinline__ int reshadow_i(int r) {
    return __builtin_amdgcn_update_dpp(r, r, 0x120 + L, 0xF, 0xC, false);  // row_ror:8, lanes 8..15 of each row
}
template <int L>
__device__ __forceinline__ double reshadow_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = reshadow_i<L>((int)(b & 0xffffffffLL)), hi = reshadow_i<L>((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// slot s's metric >= slot s-1's (64-bit unsigned: metrics are non-negative doubles); slot 0 of
// each row compares with 0
__device__ __forceinline__ bool row_order_ok(double p) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(p);
    const uint32_t plo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffull), 0x111, 0xF, 0xF, true);
    const uint32_t phi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x111, 0xF, 0xF, true);
    return (((unsigned long long)phi << 32) | plo) <= b;
}
// some row of the wave is out of order (rare: taken out of line)
#if PL_DEV && defined(PL_SCL_DIAG_SPEC_FB)  // 1 = always re-rank the pushed candidates (same results), 2 = never (timing)
#define PL_SPEC_REDO(p) \
    (PL_SCL_DIAG_SPEC_FB == 1 || (PL_SCL_DIAG_SPEC_FB == 0 && __builtin_amdgcn_ballot_w64(!row_order_ok(p)) != 0))
#else
#define PL_SPEC_REDO(p) __builtin_expect(__builtin_amdgcn_ballot_w64(!row_order_ok(p)) != 0, 0)
#endif
// the moved live buffers (those push_live moves), without the shadow copy
template <int s>
__device__ __forceinline__ void push_live_raw(double* st, int i, int dst) {
    if constexpr (s >= 1) {
        if (((i >> (s - 1)) & 1) == 0 && !(PL_SCL_PUSH_REFM && s + 1 < R && ((i >> s) & 1) == 0)) {
#pragma unroll
            for (int j = 0; j < (1 << s); ++j) st[IDX(s) + j] = push_raw_d(st[IDX(s) + j], dst);
        }
        push_live_raw<s - 1>(st, i, dst);
    }
}
// the shadow copies of the moved live buffers, then the recomputed ones (push_live's order)
template <int L, int FM, int s>
__device__ __forceinline__ void reshadow_live(double* st, int i, double lmax) {
    if constexpr (s >= 1) {
        if (((i >> (s - 1)) & 1) == 0) {
            if (PL_SCL_PUSH_REFM && s + 1 < R && ((i >> s) & 1) == 0) {
                constexpr int h = 1 << s, sp = s + 1 < R ? s + 1 : s;
#pragma unroll
                for (int j = 0; j < h; ++j) st[IDX(s) + j] = f_op<FM>(st[IDX(sp) + j], st[IDX(sp) + j + h], lmax);
            } else {
#pragma unroll
                for (int j = 0; j < (1 << s); ++j) st[IDX(s) + j] = reshadow_d<L>(st[IDX(s) + j]);
            }
        }
        reshadow_live<L, FM, s - 1>(st, i, lmax);
    }
}

// Selection of the L best of the 2L candidates of a codeword group: group lane c holds candidate
// c (c < L = (state c, u=0), c >= L = (state c-L, u=1)) with metric cv.  Its rank in the stable
// (metric, index) order comes from 2L-1 in-group broadcasts; one ds_permute then sends every
// candidate to the group lane of its rank (ranks are a permutation of [0, 2L), so every lane is
// written exactly once), and slots >= L re-shadow slot - L.  Returns the lane's new metric, the
// path (group index) it descends from and the bit the candidate appended.
template <int L, int FM>
__device__ __forceinline__ int rank_2l(double cv, int gl, int lane) {
    constexpr int GW = 2 * L;
    int rk = 0;
#if PL_SCL_DIAG_NO_RANK  // timing diagnostic only (wrong selection)
    if (true) {
        rk = gl;
    } else
#endif
    if constexpr (GW == 64) {
#pragma unroll
        for (int c = 0; c < 2 * L; ++c) {
            const double v = readlane_d(cv, c);
            rk += (v < cv || (v == cv && c < lane)) ? 1 : 0;
        }
    } else if constexpr (GW == 16 && FM == 0 && PL_SCL_RANK_SUBB && PL_SCL_RANK_SPLIT) {
        rk = rank16_split(cv);  // min-sum kernels only: its 14 mask SGPRs spill the exact-f ones
    } else {
        rank_rot<GW, 1>(cv, gl, lane, rk);
    }
    return rk;
}
template <int L, int FM>
__device__ __forceinline__ void select_2l(double cv, int gl, int gbase, int lane, double& npm, int& par,
                                          uint32_t& bit) {
    const bool hi = (gl & L) != 0;
    const int code = (gl & (L - 1)) | (hi ? 256 : 0);
    int rcode, rlo, rhi;
#if PL_SCL_DIAG_NO_RANK
    if constexpr (false) {
#else
    if constexpr (PL_SCL_SPEC && 2 * L == 16) {
#endif
        // the speculative form of the push selection (rank16_key, row_order_ok): candidates go to
        // the slot of their key rank at once, and a misordered row re-ranks the pushed candidates
        const int dst = (gbase + rank16_key(rank_key16(cv, gl))) << 2;
        double p = push_raw_d(cv, dst);
        rcode = __builtin_amdgcn_ds_permute(dst, code);
        if (PL_SPEC_REDO(p)) {
            const int dst2 = (gbase + rank16_subb(p)) << 2;
            p = push_raw_d(p, dst2);
            rcode = __builtin_amdgcn_ds_permute(dst2, rcode);
        }
        const long long pb = __double_as_longlong(p);
        rlo = (int)(pb & 0xffffffffLL);
        rhi = (int)(pb >> 32);
    } else {
        const int dst = gbase + rank_2l<L, FM>(cv, gl, lane);
        const long long cb = __double_as_longlong(cv);
        rcode = __builtin_amdgcn_ds_permute(dst << 2, code);
        rlo = __builtin_amdgcn_ds_permute(dst << 2, (int)(cb & 0xffffffffLL));
        rhi = __builtin_amdgcn_ds_permute(dst << 2, (int)(cb >> 32));
    }
    const int me = gbase + (gl & (L - 1));
    rcode = bperm_i(rcode, me);
    rlo = bperm_i(rlo, me);
    rhi = bperm_i(rhi, me);
    par = rcode & 255;
    bit = (uint32_t)rcode >> 8;
    npm = __longlong_as_double(((long long)rhi << 32) | (unsigned int)rlo);
}

// numpy's pairwise np.sum of len = 2^s terms (len < 8: sequentially from 0; up to 128: 8
// interleaved partial sums combined ((0+1)+(2+3))+((4+5)+(6+7)); larger: blocks of 128 combined
// pairwise), the node sums of fast-SCL (my_sn dec.py:276-280, :297-300)
__device__ __forceinline__ double pairwise8(const double (&r)[8]) {
    return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
}

// fast-SCL node test from the frozen bits fb of a node of len positions (mask m = all ones):
// rate-0 = all frozen (dec.py:369-372), repetition = all but the last frozen (:373-376)
__device__ __forceinline__ int prune_kind(uint32_t fb, uint32_t m) {
    return fb == m ? 1 : (fb == (m >> 1) ? 2 : 0);
}

// Lane-level fast-SCL descent from stage s (its input st[IDX(s)] ready) at leaf position i of
// the subtree: a rate-0 / repetition node is not descended -- returns its stage, kind 1 rate-0 /
// 2 repetition; otherwise f down to the leaf (returns 0, st[0] = the leaf LLR).
template <int s, int FM, int L>
__device__ __forceinline__ int descend_fast(double* st, uint32_t fz, int i, double lmax, int& kind) {
    if constexpr (s == 0) {
        return 0;
    } else {
        constexpr int len = 1 << s;
        const int kd = prune_kind((fz >> i) & ((1u << len) - 1u), (1u << len) - 1u);
        if (kd != 0) {
            kind = kd;
            return s;
        }
        constexpr int h = len / 2;
        f_span<h, FM, L, false>(st + IDX(s), st + IDX(s - 1), lmax);
        return descend_fast<s - 1, FM, L>(st, fz, i, lmax, kind);
    }
}

// Metric term sum of a pruned lane-level node of 2^s inputs v[0, 2^s) (2, 4 or 8), numpy order:
// len < 8 sequentially from 0, len = 8 as 8 partial sums combined pairwise.  A repetition node's
// shadow lanes sum the u = 1 branch (negated inputs).  (Splitting a rate-0 node's terms between
// path and shadow lanes measured no faster: 1.357 vs 1.359 ms.)
template <int s>
__device__ __forceinline__ double node_sum_lane(const double* v, int kind, bool hi, double lmax) {
    constexpr int len = 1 << s;
    const double sg = (kind == 2 && hi) ? -1.0 : 1.0;
    double tt[len];
#pragma unroll
    for (int j = 0; j < len; ++j) {
        const double l = fmax(fmin(sg * v[j], lmax), -lmax);
        tt[j] = pl::softplus_pm(-l);
    }
    if constexpr (len == 8) {
        return pairwise8(tt);
    } else {
        double r = 0.0;
#pragma unroll
        for (int j = 0; j < len; ++j) r += tt[j];
        return r;
    }
}

// f(0), f(1), ..., f(sizeof...(I) - 1) with constant arguments
template <typename F, int... I>
__device__ __forceinline__ void unroll_leaves(F& f, std::integer_sequence<int, I...>) {
    (f(I), ...);
}

// Decode the stage-R node at absolute position i0 for every path of every codeword of the wave
// (group lanes < L own paths; group lanes >= L shadow lane gl - L).  pm, org: the lane's metric
// and origin (path index inside the group).  FAST: fast-SCL pruning of the rate-0 / repetition
// nodes inside the subtree (sizes 2..8; the stage-R node itself is tested by the caller).
template <int L, int FM, int CPW, bool FAST>
__device__ void subtree(const St& t, int i0, uint32_t fz, double& pm, int& org, uint32_t& ps, int lane PROF_PARAM) {
    constexpr int GW = 2 * L;
    const int gl = lane & (GW - 1), gbase = lane & ~(GW - 1);
    const bool hi = (gl & L) != 0;
    const Cw w = t.cw(lane / GW);
    double st[T - 1];
    ps = 0u;
    org = gl & (L - 1);
    const double* inA = w.A + org * t.per;  // stage R sits at offset 0 of a path's region
    int resume = 0;                          // FAST: first leaf after a pruned node
    bool pair = false;                       // !FAST: leaf i-1 started a frozen sibling pair
    // one leaf of the subtree (i: its index); !FAST kernels unroll all T leaves with constant
    // indices (unroll_leaves) -- the loop form below was unrolled only by 8 once the body grew,
    // which left every leaf-index shift, combine and g stage a run-time choice
    auto leaf = [&](const int i) __attribute__((always_inline)) {
        if (FAST && i < resume) return;
        if (!FAST && PL_SCL_FROZEN_PAIR && (i & 1) && pair) return;  // done with leaf i-1
        if (i > 0) {  // nodes that ended at leaf i-1 (stages 1..ctz(i)): [uL ^ uR, uR] (:147-153)
            const int tz = __builtin_ctz(i);
            for (int s = 1; s <= tz; ++s) {
                const int h = 1 << (s - 1), pos = i - (1 << s);
                ps ^= (ps >> h) & (((1u << h) - 1u) << pos);
            }
            if (tz + 1 == R) inA = w.A + org * t.per;  // the origin may have changed
        }
        if constexpr (!FAST) {
            leaf_llr<FM, L>(inA, st, ps, i, t.lmax);
            PROF_MARK(8);
        } else {
            // the node input at stage top = R-1 (leaf 0: f of the stage-R input) or ctz(i) (g of
            // the parent's input), then the pruning descent
            int top;
            if (i == 0) {
                constexpr int h = T / 2;
                f_span<h, FM, L, true>(inA, st + IDX(R - 1), t.lmax);
                top = R - 1;
            } else {
                top = __builtin_ctz(i);
                switch (top) {
                    case 0: g_only<0>(inA, st, ps, i); break;
                    case 1: g_only<1>(inA, st, ps, i); break;
                    case 2: g_only<2>(inA, st, ps, i); break;
                    default: g_only<R - 1>(inA, st, ps, i); break;
                }
            }
            int kind = 0, ps_ = 0;
            switch (top) {
                case 0: ps_ = 0; break;
                case 1: ps_ = descend_fast<1, FM, L>(st, fz, i, t.lmax, kind); break;
                case 2: ps_ = descend_fast<2, FM, L>(st, fz, i, t.lmax, kind); break;
                default: ps_ = descend_fast<R - 1, FM, L>(st, fz, i, t.lmax, kind); break;
            }
            if (ps_ > 0) {  // pruned node of size 2^ps_ at leaf i: its input is st[IDX(ps_)]
                // repetition: shadow lanes evaluate the u = 1 branch (negated LLRs, dec.py:294)
                double nsum;
                switch (ps_) {
                    case 1: nsum = node_sum_lane<1>(st + IDX(1), kind, hi, t.lmax); break;
                    case 2: nsum = node_sum_lane<2>(st + IDX(2), kind, hi, t.lmax); break;
                    default: nsum = node_sum_lane<3>(st + IDX(3), kind, hi, t.lmax); break;
                }
                const int last = i + (1 << ps_) - 1;
                resume = last + 1;
                if (kind == 1) {  // rate-0: the node sum replaces its leaves' updates
                    pm = pm + nsum;
                } else {  // repetition: 2L candidates on the node sums, bit on the last leaf
                    double npm;
                    int par;
                    uint32_t bit;
                    select_2l<L, FM>(pm + nsum, gl, gbase, lane, npm, par, bit);
                    pm = npm;
                    ps = (uint32_t)bperm_i((int)ps, gbase + par) | (bit << last);
                    org = bperm_i(org, gbase + par);
                    inA = w.A + org * t.per;
                    pull_live<R - 1>(st, last, gbase + par);
                }
                return;
            }
        }
        // Frozen sibling pair (leaves i, i+1 both frozen, i even): u_i = 0 is known, so the
        // shadow lanes take leaf i+1's LLR g(a, b, 0) from the stage-1 input and the pair costs
        // one exp/log per lane; the metric still adds the two terms in order.
        double lv = st[0];
        if constexpr (!FAST && PL_SCL_FROZEN_PAIR) {
            pair = (i & 1) == 0 && ((fz >> i) & 3u) == 3u;
            if (pair && hi) lv = g_op(st[IDX(1)], st[IDX(1) + 1], 0u);
        }
        const double l = fmax(fmin(lv, t.lmax), -t.lmax);
        // metric update (:83): pen = log(1 + exp(-(1-2u) l)).  At an information leaf shadow
        // lanes evaluate u = 1, path lanes u = 0: one exp/log per lane gives all 2L candidates.
        // Same expression as the reference, so same rounding.
        const bool info = ((fz >> i) & 1u) == 0u;
        const double sl = (info && hi) ? -1.0 * l : 1.0 * l;
#if PL_SCL_DIAG_CHEAP_PEN  // timing diagnostic only (wrong metrics)
        const double pen = fmax(-sl, 0.0);
#else
        const double pen = pl::softplus_pm(-sl);
#endif
        if (!info) {  // frozen leaf: metric update only (u = 0)
            if (!FAST && PL_SCL_FROZEN_PAIR && pair) {
                const double oth = half_xchg<L>(pen, lane);
                pm = (pm + (hi ? oth : pen)) + (hi ? pen : oth);
            } else {
                pm = pm + pen;  // invariant: pm >= +0 (pen = softplus >= +0), which the ranks rely on
            }
            PROF_MARK(9);
            return;
        }
#if PL_SCL_PROF
        asm volatile("" ::"v"(pen));
        PROF_MARK(9);
#endif
        if constexpr (PL_SCL_SPEC && PL_SCL_PUSH == 1 && L == 8 && FM == 0 && !PL_SCL_DIAG_NO_PULL) {
            const double cv = pm + pen;
            const int dst = (gbase + rank16_key(rank_key16(cv, gl))) << 2;
            double p = push_raw_d(cv, dst);
            int pps = __builtin_amdgcn_ds_permute(dst, (int)(ps | ((hi ? 1u : 0u) << i)));
            int pog = __builtin_amdgcn_ds_permute(dst, org);
            push_live_raw<R - 1>(st, i, dst);
            if (PL_SPEC_REDO(p)) {
                // metrics closer than the key resolves, in the wrong order: the stable 64-bit rank
                // of the pushed candidates, and the push once more
                const int dst2 = (gbase + rank16_subb(p)) << 2;
                p = push_raw_d(p, dst2);
                pps = __builtin_amdgcn_ds_permute(dst2, pps);
                pog = __builtin_amdgcn_ds_permute(dst2, pog);
                push_live_raw<R - 1>(st, i, dst2);
            }
            pm = reshadow_d<L>(p);
            ps = (uint32_t)reshadow_i<L>(pps);
            org = reshadow_i<L>(pog);
            inA = w.A + org * t.per;
            reshadow_live<L, FM, R - 1>(st, i, t.lmax);
#if PL_SCL_PROF
            asm volatile("" ::"v"(pm), "v"(ps), "v"(org));
            PROF_MARK(11);
#endif
            return;
        }
        if constexpr (PL_SCL_PUSH == 2 && L == 8 && FM == 0 && !PL_SCL_DIAG_NO_PULL) {
            const double cv = pm + pen;
            const int dst = (gbase + rank_2l<L, FM>(cv, gl, lane)) << 2;
            const int src = pull_src<L>(lane, dst);
            pm = bperm_d(cv, src);
            ps = (uint32_t)bperm_i((int)(ps | ((hi ? 1u : 0u) << i)), src);
            org = bperm_i(org, src);
            inA = w.A + org * t.per;
            pull2_live<L, FM, R - 1>(st, i, src, t.lmax);
            return;
        }
        if constexpr (PL_SCL_PUSH == 1 && L == 8 && FM == 0 && !PL_SCL_DIAG_NO_PULL) {  // exact f: spills (r04r)
            const double cv = pm + pen;
            const int dst = (gbase + rank_2l<L, FM>(cv, gl, lane)) << 2;
#if PL_SCL_PROF
            asm volatile("" ::"v"(dst));
            PROF_MARK(10);
#endif
            pm = push_d<L>(cv, dst);
            ps = (uint32_t)push_i<L>((int)(ps | ((hi ? 1u : 0u) << i)), dst);
            org = push_i<L>(org, dst);
            inA = w.A + org * t.per;
            push_live<L, FM, R - 1>(st, i, dst, t.lmax);
#if PL_SCL_PROF
            asm volatile("" ::"v"(pm), "v"(ps), "v"(org));
            PROF_MARK(11);
#endif
            return;
        }
        double npm;
        int par;
        uint32_t bit;
        select_2l<L, FM>(pm + pen, gl, gbase, lane, npm, par, bit);
        pm = npm;
        ps = (uint32_t)bperm_i((int)ps, gbase + par) | (bit << i);
        org = bperm_i(org, gbase + par);
        inA = w.A + org * t.per;
#if !PL_SCL_DIAG_NO_PULL  // timing diagnostic only
        pull_live<R - 1>(st, i, gbase + par);
#endif
    };
    if constexpr (!FAST && PL_SCL_UNROLL) {
        unroll_leaves(leaf, std::make_integer_sequence<int, T>{});
    } else {
#pragma unroll
        for (int i = 0; i < T; ++i) leaf(i);
    }
    for (int s = 1; s <= R; ++s) {  // the nodes ending at the last leaf, up to stage R
        const int h = 1 << (s - 1), pos = T - (1 << s);
        ps ^= (ps >> h) & (((1u << h) - 1u) << pos);
    }
}


// Metric term of element j of a virtual stage-s node (D = S - s stages below the channel).
template <int D, int FM>
__device__ __noinline__ double vterm(const float* ch, const uint32_t* bp, int s, int pos, int j, double sg,
                                     double lmax) {
    const double l = fmax(fmin(sg * vread<D, FM>(ch, bp, s, pos, j, lmax), lmax), -lmax);
    return pl::softplus_pm(-l);
}

// Metric term sum (numpy pairwise order) of the stage-s node at pos for path p, with sign sg:
// stored stage (s <= SS, inline), or recomputed from the channel (virtual, D = S - s <= V
// stages: the out-of-line vterm, scalar arguments only so nothing is passed through scratch).
template <int V, int FM>
__device__ __forceinline__ double upper_node_sum(const St& t, const Cw& w, int p, int s, int pos, double sg) {
    const int len = 1 << s;
    const uint32_t* bp = w.beta + p * t.W;
    const double* in = s <= t.SS ? w.A + w.sptr[p * SPS + s] * t.per + (1 << s) - (1 << R) : nullptr;
    const int D = t.S - s;
    const int blk = len < 128 ? len : 128;
    double lvl[8];
    int nl = 0;
    for (int b0 = 0; b0 < len; b0 += blk) {
        double acc[8];
        for (int i = 0; i < blk; i += 8) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int e = b0 + i + j;
                double tj;
                if (in) {
                    const double l = fmax(fmin(sg * in[e], t.lmax), -t.lmax);
                    tj = pl::softplus_pm(-l);
                } else if (D == 0) {
                    tj = vterm<0, FM>(w.ch, bp, s, pos, e, sg, t.lmax);
                } else if (D == 1 || V < 2) {
                    tj = vterm<1, FM>(w.ch, bp, s, pos, e, sg, t.lmax);
                } else if (D == 2 || V < 3) {
                    tj = vterm<(V >= 2 ? 2 : 1), FM>(w.ch, bp, s, pos, e, sg, t.lmax);
                } else if (D == 3 || V < 4) {
                    tj = vterm<(V >= 3 ? 3 : 1), FM>(w.ch, bp, s, pos, e, sg, t.lmax);
                } else {
                    tj = vterm<(V >= 4 ? 4 : 1), FM>(w.ch, bp, s, pos, e, sg, t.lmax);
                }
                acc[j] = i == 0 ? tj : acc[j] + tj;
            }
        }
        lvl[nl++] = pairwise8(acc);
    }
    while (nl > 1) {
        for (int i = 0; i < nl / 2; ++i) lvl[i] = lvl[2 * i] + lvl[2 * i + 1];
        nl /= 2;
    }
    return lvl[0];
}

// fast-SCL type of the node of 2^s positions at pos (s >= R) from the frozen words
__device__ __forceinline__ int node_kind(const uint32_t* __restrict__ fw, int s, int pos) {
    if (s < 5) {
        const uint32_t m = (1u << (1 << s)) - 1u;
        return prune_kind((fw[pos >> 5] >> (pos & 31)) & m, m);
    }
    const int w0 = pos >> 5, nw = 1 << (s - 5);
    for (int w = 0; w < nw - 1; ++w)
        if (fw[w0 + w] != ~0u) return 0;
    return prune_kind(fw[w0 + nw - 1], ~0u);
}

// Re-point the upper-tree state of every path to its origin path org_s[]: partial-sum words
// before i0 and the stage owners.
template <int L, int V, int CPW>
__device__ void repoint(const St& t, int i0, int lane) {
    constexpr int LL = ilog2(L);
#if PL_SCL_REPOINT_VEC
    if (V >= 2 || t.W >= 4) {  // V >= 2: n >= 128, so W >= 4 (the word loop below is not compiled in)
        // LPP = 64 / (CPW * L) lanes per (codeword, path) pair (2 at CPW * L = 32, 4 with two rows
        // per codeword): one origin load each, the pair's partial-sum row in 16-byte quads (words
        // past i0 are copied too: they belong to leaves not decided yet and are overwritten before
        // anything reads them) and its 16-byte stage-owner row -- 6 LDS loads and 5 stores per
        // lane instead of 22 and 22 (LPP = 2)
        constexpr int LPP = 64 / (CPW * L), QPL = 8 / LPP;  // quads per lane (W <= 32 words = 8 quads)
        static_assert(64 % (CPW * L) == 0 && LPP >= 2 && LPP <= 8, "repoint: lanes per (codeword, path) pair");
        asm volatile("" : "+v"(lane));  // per-call addresses (not hoisted out of the decoder loop)
        const int cp = lane >> ilog2(LPP), h = lane & (LPP - 1), p = cp & (L - 1);  // lane is opaque: shifts, not signed division
        const Cw cw = t.cw(cp >> LL);
        const int o = cw.org_s[p];
        const int nq = min(t.W >> 2, (((i0 + 31) >> 5) + 3) >> 2);
        const uint4* src = reinterpret_cast<const uint4*>(cw.beta + o * t.W);
        uint4 v0 = make_uint4(0u, 0u, 0u, 0u), v1 = v0, v2 = v0, v3 = v0, sp = v0;  // QPL <= 4 quads
        if (h < nq) v0 = src[h];
        if (QPL > 1 && h + LPP < nq) v1 = src[h + LPP];
        if (QPL > 2 && h + 2 * LPP < nq) v2 = src[h + 2 * LPP];
        if (QPL > 3 && h + 3 * LPP < nq) v3 = src[h + 3 * LPP];
        if (h == 0) sp = *reinterpret_cast<const uint4*>(cw.sptr + o * SPS);
        __syncthreads();
        uint4* dst = reinterpret_cast<uint4*>(cw.beta + p * t.W);
        if (h < nq) dst[h] = v0;
        if (QPL > 1 && h + LPP < nq) dst[h + LPP] = v1;
        if (QPL > 2 && h + 2 * LPP < nq) dst[h + 2 * LPP] = v2;
        if (QPL > 3 && h + 3 * LPP < nq) dst[h + 3 * LPP] = v3;
        if (h == 0) *reinterpret_cast<uint4*>(cw.sptr + p * SPS) = sp;
        __syncthreads();
        return;
    }
#endif
    if constexpr (PL_SCL_REPOINT_VEC && V >= 2) return;
    const int W = t.W, w_lim = (i0 + 31) >> 5;
    // CPW * L = 32 (codeword, path) pairs per wave, <= 32 words each (n <= 1024)
    constexpr int RB = 32 * 32 / 64;
    uint32_t vb[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        const int idx = r * 64 + lane;
        const int cp = idx >> 5, w = idx & 31;
        if (w < w_lim) {
            const Cw cw = t.cw(cp >> LL);
            vb[r] = cw.beta[cw.org_s[cp & (L - 1)] * W + w];
        }
    }
    constexpr int RS = (32 * 11 + 63) / 64;
    uint8_t vs[RS];
    const int S1 = t.S + 1;  // entries per row (rows are SPS bytes apart)
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        const int idx = r * 64 + lane;
        if (idx < 32 * S1) {
            const int cp = idx / S1, e = idx - cp * S1;
            const Cw cw = t.cw(cp >> LL);
            vs[r] = cw.sptr[cw.org_s[cp & (L - 1)] * SPS + e];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        const int idx = r * 64 + lane;
        const int cp = idx >> 5, w = idx & 31;
        if (w < w_lim) t.cw(cp >> LL).beta[(cp & (L - 1)) * W + w] = vb[r];
    }
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        const int idx = r * 64 + lane;
        if (idx < 32 * S1) {
            const int cp = idx / S1, e = idx - cp * S1;
            t.cw(cp >> LL).sptr[(cp & (L - 1)) * SPS + e] = vs[r];
        }
    }
    __syncthreads();
}

// A pruned fast-SCL node of 2^s >= 2^R positions at pos (kind 1 rate-0, 2 repetition): the
// node sums replace the descent (dec.py:269-306).  Repetition: 2L candidates on the sums, the
// paths re-pointed to their parents, and the node's partial sums x = u..u set through its last
// 16-position chunk (the chunks before stay 0; the combines of the stages above R complete x).
template <int L, int V, int FM, int CPW>
__device__ void upper_prune(const St& t, int s, int pos, int kind, double& pm, int lane) {
    constexpr int GW = 2 * L;
    const int gl = lane & (GW - 1), gbase = lane & ~(GW - 1);
    const bool hi = (gl & L) != 0;
    const Cw w = t.cw(lane / GW);
    const double sg = (kind == 2 && hi) ? -1.0 : 1.0;
    const double nsum = upper_node_sum<V, FM>(t, w, gl & (L - 1), s, pos, sg);
    if (kind == 1) {
        pm = pm + nsum;
        return;
    }
    double npm;
    int par;
    uint32_t bit;
    select_2l<L, FM>(pm + nsum, gl, gbase, lane, npm, par, bit);
    pm = npm;
    if (gl < L) w.org_s[gl] = par;
    __syncthreads();
    repoint<L, V, CPW>(t, pos, lane);
    if (gl < L && bit) {
        const int b = pos + (1 << s) - T;
        w.beta[gl * t.W + (b >> 5)] |= ((1u << T) - 1u) << (b & 31);
    }
    __syncthreads();
}

template <int L, int V, int FM, bool FAST>
__global__ __launch_bounds__(64)
#if PL_SCL_WPE > 0
__attribute__((amdgpu_waves_per_eu(PL_SCL_WPE)))
#endif
void scl_tree_kernel(const float* __restrict__ llr, int64_t bs, void* __restrict__ out,
                                                      int out_kind, double* __restrict__ out_pm,
                                                      const uint32_t* __restrict__ frozen_words,
                                                      const int32_t* __restrict__ info_pos, int n, int S, int k,
                                                      double lmax, int crc_deg, uint32_t crc_g,
                                                      double* __restrict__ vcache) {
    constexpr int GW = 2 * L, CPW = 64 / GW, LL = ilog2(L);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    St t;
    t.smem = smem;
    t.y = make_layout(n, S, L, V);
    t.llr = llr;
    t.b0 = (int64_t)blockIdx.x * CPW;
    t.bs = bs;
    t.n = n;
    t.S = S;
    t.W = t.y.W;
    t.SS = t.y.SS;
    t.per = t.y.per;
    t.lmax = lmax;
    t.vcache = (FM == 1 && V >= 1 && vcache != nullptr) ? vcache + t.b0 * cache_size(n, V) : nullptr;
    const int W = t.W, LW = ilog2(W);
    const int gl = lane & (GW - 1), my_c = lane / GW;
    const Cw mine = t.cw(my_c);
    pl::sp_load_tables(lane, 64);  // the penalty's log table (softplus.h, PL_SP_FORM 3)
    pl::fex_load_table<FM == 1>(lane);  // the exact f's 2^(j/64) table (softplus.h fex_exp)
    PROF_DECL;
#if PL_SCL_PROF >= 2
    if (lane < 3) vex_prof[lane] = 0ull;
    __syncthreads();
#endif

    for (int i = lane; i < CPW * L * W; i += 64) t.cw(i >> (LL + LW)).beta[i & (L * W - 1)] = 0u;
    for (int i = lane; i < CPW * L * SPS; i += 64) {
        const int c = i / (L * SPS), e = i - c * (L * SPS);
        t.cw(c).sptr[e] = (uint8_t)(e / SPS);
    }
    if (S == R)  // the whole tree is one lane-local subtree: its input is the channel, as fp64
        for (int i = lane; i < CPW * T; i += 64) {
            const Cw w = t.cw(i / T);
            w.A[i % T] = (double)(-1.0f * w.ch[i % T]);
        }
    __syncthreads();

    if constexpr (FM == 1 && V >= 1) {
        if (t.vcache != nullptr) {  // fill the leftmost chain, level by level (wave-parallel, pairs of f)
            const int cs = cache_size(n, V);
#pragma unroll 1
            for (int k = 1; k <= V; ++k) {
                const int sz = n >> k, lsz = S - k;
                const double* prev = t.vcache + (k > 1 ? chain_off(n, k - 1) : 0);
                double* cur = t.vcache + chain_off(n, k);
#pragma unroll 1
                for (int i0 = lane; i0 < CPW * sz; i0 += 128) {
                    double a[2], b[2], r[2];
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const int idx = min(i0 + 64 * u, CPW * sz - 1);  // a clamped duplicate is recomputed, not stored
                        const int c = idx >> lsz, i = idx & (sz - 1);
                        if (k == 1) {
                            const float* ch = t.cw(c).ch;
                            a[u] = (double)(-1.0f * ch[i]);
                            b[u] = (double)(-1.0f * ch[i + sz]);
                        } else {
                            a[u] = prev[c * cs + i];
                            b[u] = prev[c * cs + i + sz];
                        }
                    }
                    f_ex2(a[0], b[0], a[1], b[1], t.lmax, r[0], r[1]);
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const int idx = i0 + 64 * u;
                        if (idx < CPW * sz) cur[(idx >> lsz) * cs + (idx & (sz - 1))] = r[u];
                    }
                }
                __threadfence_block();
                __syncthreads();
            }
#if PL_SCL_FEX_COMBO
#pragma unroll 1
            for (int ns = 0; ns + 2 <= V; ++ns) {  // the four-outcome tables (combo_off)
                const int D = n >> (ns + 2), lsz = S - ns - 2;
                const double* src = t.vcache + chain_off(n, ns > 0 ? ns : 1);
                double* tab = t.vcache + combo_off(n, V, ns);
#pragma unroll 1
                for (int idx = lane; idx < CPW * D; idx += 64) {
                    const int c = idx >> lsz, e = idx & (D - 1);
                    double a, b, cc, d;
                    if (ns == 0) {
                        const float* ch = t.cw(c).ch;
                        a = (double)(-1.0f * ch[e]);
                        b = (double)(-1.0f * ch[e + 2 * D]);
                        cc = (double)(-1.0f * ch[e + D]);
                        d = (double)(-1.0f * ch[e + 3 * D]);
                    } else {
                        const double* sc = src + c * cs;
                        a = sc[e];
                        b = sc[e + 2 * D];
                        cc = sc[e + D];
                        d = sc[e + 3 * D];
                    }
                    const double g0 = g_op(a, b, 0u), g1 = g_op(a, b, 1u);
                    const double h0 = g_op(cc, d, 0u), h1 = g_op(cc, d, 1u);
                    double r0, r1, r2, r3;
                    f_ex2(g0, h0, g0, h1, t.lmax, r0, r1);
                    f_ex2(g1, h0, g1, h1, t.lmax, r2, r3);
                    double* o = tab + c * cs + 4 * e;
                    o[0] = r0;
                    o[1] = r1;
                    o[2] = r2;
                    o[3] = r3;
                }
            }
            __threadfence_block();
            __syncthreads();
#endif
        }
    }

    PROF_MARK(6);
    VCache<FM> vcache_lane;  // the virtual-node cache (vnode64, vvisit_ex)
#if PL_SCL_C7
    if constexpr (FM == 0) vcache_lane.p7 = -1;
#endif
    VCache<FM>* vcp = (PL_SCL_VCACHE && !PL_SCL_VPF && ((FM == 0 && V == 4) || (FM == 1 && V >= 1 && PL_SCL_FEX_HOIST)))
                      ? &vcache_lane : nullptr;
    double pm = gl == 0 || gl == L ? 0.0 : lmax;  // :192-194 ([0, 30 x (L-1)] per half)
    const int nsub = n >> R;
    int q = 0;
    while (q < nsub) {
        const int i0 = q << R;
        // input of the stage-R node at i0: g of the node that ends the finished left sibling,
        // then f down to stage R (stored stages only; virtual ones are recomputed on read),
        // testing every node entered for fast-SCL pruning (my_sn dec.py:367-376)
        int top;
        if (q == 0) {
            top = S;
        } else {
            const int tz = __builtin_ctz(i0);
            if (!PL_SCL_DIAG_NO_UPPER && tz <= t.SS) {
                node_fg<L, V, FM, CPW>(t, tz + 1, i0 & ~((2 << tz) - 1), true, lane, vcp);
                if (tz + 1 > t.SS) PROF_MARK(5); else PROF_MARK(1);  // 5: right (g) virtual passes
            }
            top = tz;
        }
        int pr = 0, kind = 0;
        for (int s = top; s >= R; --s) {
            if constexpr (FAST) {
                kind = PL_SCL_DIAG_NO_UPPER_PRUNE ? 0 : node_kind(frozen_words, s, i0);
                if (kind != 0) {
                    pr = s;
                    break;
                }
            }
            if (!PL_SCL_DIAG_NO_UPPER && s > R && s - 1 <= t.SS) {
                node_fg<L, V, FM, CPW>(t, s, i0, false, lane, vcp);
                if (s > t.SS) PROF_MARK(0); else PROF_MARK(1);
            }
        }
        if (FAST && kind != 0) {
            upper_prune<L, V, FM, CPW>(t, pr, i0, kind, pm, lane);
            PROF_MARK(5);
            q += 1 << (pr - R);
        } else {
            int org;
            uint32_t ps;
            subtree<L, FM, CPW, FAST>(t, i0, frozen_words[i0 >> 5] >> (i0 & 31), pm, org, ps, lane PROF_ARG);
            PROF_MARK(2);
            // re-point the upper-tree state of every path to its origin's, then store the
            // subtree's partial sums: partial-sum words before i0 and stage owners R..SS
            if (gl < L) mine.org_s[gl] = org;
            __syncthreads();
            if (!PL_SCL_DIAG_NO_REPOINT) repoint<L, V, CPW>(t, i0, lane);
            const int w_i = i0 >> 5, off = i0 & 31;
            if (gl < L) {
                uint32_t* bw = mine.beta + gl * W + w_i;
                *bw = off == 0 ? ps : ((*bw & ((1u << off) - 1u)) | (ps << off));
            }
            __syncthreads();
            PROF_MARK(3);
            q += 1;
        }
        // nodes above R that end here
        const int nxt = q << R;
        const int top2 = nxt < n ? __builtin_ctz(nxt) : S;
        if (!PL_SCL_DIAG_NO_COMBINE)
            for (int s = R + 1; s <= top2; ++s) combine_upper<L, CPW>(t, s, nxt - (1 << s), lane);
        PROF_MARK(4);
    }
    if (gl < L) mine.pm_s[gl] = pm;

    // u = x G_n per path (x = the root's partial sums): in-word spans, then word spans
    for (int idx = lane; idx < CPW * L * W; idx += 64) {
        uint32_t* bw = t.cw(idx >> (LL + LW)).beta + (idx & (L * W - 1));
        uint32_t w = *bw;
        w ^= (w >> 1) & 0x55555555u;
        w ^= (w >> 2) & 0x33333333u;
        w ^= (w >> 4) & 0x0f0f0f0fu;
        w ^= (w >> 8) & 0x00ff00ffu;
        w ^= (w >> 16) & 0x0000ffffu;
        *bw = w;
    }
    __syncthreads();
    for (int m = 1; m < W; m <<= 1) {
        for (int idx = lane; idx < CPW * L * W; idx += 64) {
            if ((idx & m) == 0) {
                uint32_t* bw = t.cw(idx >> (LL + LW)).beta + (idx & (L * W - 1));
                bw[0] ^= bw[m];
            }
        }
        __syncthreads();
    }

    // CRC check per path (my_sn dec.py:507-518)
    if (gl < L) {
        int f = 0;
        if (crc_deg > 0) {
            const uint32_t* U = mine.beta + gl * W;
            const uint32_t mask = (1u << crc_deg) - 1u;
            uint32_t reg = 0;
            for (int m = 0; m < k; ++m) {
                const int pos = info_pos[m];
                const uint32_t fb = ((reg >> (crc_deg - 1)) & 1u) ^ ((U[pos >> 5] >> (pos & 31)) & 1u);
                reg = (reg << 1) & mask;
                if (fb) reg ^= crc_g;
            }
            f = reg != 0u;
        }
        mine.fail_s[gl] = f;
    }
    __syncthreads();
    // Final stable sort of the 2L logical rows (row r < L = state r, row r >= L its copy) by
    // metric, penalty per failing row, first argmin in that order (:204-206, :224): group lane
    // r ranks row r and files it at its rank; the group's first lane scans the sorted rows.
    {
        const int p = gl & (L - 1);
        const double mv = mine.pm_s[p];
        int rk = 0;
        for (int c = 0; c < GW; ++c) {
            const double v = mine.pm_s[c & (L - 1)];
            rk += (v < mv || (v == mv && c < gl)) ? 1 : 0;
        }
        const double val = mv + (mine.fail_s[p] ? t.lmax * (double)k : 0.0);
        mine.sv[rk] = val;
        mine.sp[rk] = p;
        if (out_pm != nullptr && t.b0 + my_c < bs) out_pm[(t.b0 + my_c) * GW + rk] = val;
    }
    __syncthreads();
    if (gl == 0) {
        double bestv = mine.sv[0];
        int best = mine.sp[0];
        for (int r = 1; r < GW; ++r)
            if (mine.sv[r] < bestv) {
                bestv = mine.sv[r];
                best = mine.sp[r];
            }
        mine.org_s[0] = best;
    }
    __syncthreads();
    for (int c = 0; c < CPW; ++c) {
        const int64_t b = t.b0 + c;
        if (b >= bs) break;
        const Cw w = t.cw(c);
        const uint32_t* U = w.beta + w.org_s[0] * W;
        for (int m = lane; m < k; m += 64) {
            const int pos = info_pos[m];
            const uint32_t bit = (U[pos >> 5] >> (pos & 31)) & 1u;
            if (out_kind == PL_OUT_F32) static_cast<float*>(out)[b * k + m] = bit ? 1.0f : 0.0f;
            else static_cast<uint8_t*>(out)[b * k + m] = (uint8_t)bit;
        }
    }
#if PL_SCL_PROF
    PROF_MARK(7);
#if PL_SCL_PROF >= 2
    if constexpr (FM == 1 && FAST) {  // the vvisit_ex sub-phases (inside slot 0's time)
        prof.acc[8] = vex_prof[0];
        prof.acc[10] = vex_prof[1];
        prof.acc[11] = vex_prof[2];
    }
#endif
    if (out_pm != nullptr && lane < kProfSlots) {
        unsigned long long v = prof.acc[0];
#pragma unroll
        for (int i = 1; i < kProfSlots; ++i) v = lane == i ? prof.acc[i] : v;
        reinterpret_cast<unsigned long long*>(out_pm)[bs * GW + (int64_t)blockIdx.x * kProfSlots + lane] = v;
    }
#endif
}

}  // namespace

// Instantiations are split over translation units, one per list size (the build compiles this
// file once per PL_SCL_TREE_L in parallel, plus once with PL_SCL_TREE_DISPATCH for the launcher).
namespace pl {
template <int L>
const void* scl_tree_fn(int v, bool exact, bool fast);
}

#ifdef PL_SCL_TREE_L
namespace pl {
template <>
const void* scl_tree_fn<PL_SCL_TREE_L>(int v, bool exact, bool fast) {
    constexpr int L = PL_SCL_TREE_L;
#define PL_FM(V)                                                                                  \
    (exact ? (fast ? (const void*)scl_tree_kernel<L, V, 1, true> : (const void*)scl_tree_kernel<L, V, 1, false>) \
           : (fast ? (const void*)scl_tree_kernel<L, V, 0, true> : (const void*)scl_tree_kernel<L, V, 0, false>))
    switch (v) {
        case 0: return PL_FM(0);
        case 1: return PL_FM(1);
        case 2: return PL_FM(2);
        case 3: return PL_FM(3);
        default: return PL_FM(4);
    }
#undef PL_FM
}
}  // namespace pl
#endif

#ifdef PL_SCL_TREE_DISPATCH
namespace {
int pick_v(int S) {
    int vmax = 4;  // the channel is read from global memory, so virtual stages cost no LDS
#if PL_DEV
    if (const char* e = getenv("PL_SCL_VIRTUAL")) vmax = atoi(e);  // development A/B (tools/)
#endif
    if (vmax > 4) vmax = 4;  // instantiated: V = 0..4 (the kernel's layout must match the host's)
    int v = S - 1 - R;
    if (v > vmax) v = vmax;
    if (v == 4 && S != 10) v = 3;  // the V = 4 instance assumes n = 1024 (virtual node of 64)
    return v < 0 ? 0 : v;
}
}  // namespace

namespace pl {

// Eligible plans: 2 <= L <= 32, 32 <= n <= 1024, no fast-SCL pruning.
bool scl_tree_eligible(const pl_plan* p) {
    if (p->flags & PL_PLAN_GENERIC) return false;
#if PL_DEV
    if (const char* e = getenv("PL_SCL_TREE_FAST"))  // fast-SCL plans on the generic kernel (A/B, tools/)
        if (e[0] == '0' && (p->flags & PL_PLAN_FAST_SCL)) return false;
#endif
    if (const char* e = getenv("PL_SCL_TREE"))
        if (e[0] == '0') return false;
    return p->list_size >= 2 && p->list_size <= 32 && p->log_n >= 5 && p->log_n <= 10;
}

// Workspace: the exact-f kernels' leftmost-chain cache and four-outcome tables, one slot per
// codeword of every launched wave (a tail wave's clamped codewords get their own slots).  A batch
// larger than kSclWsChunk codewords is decoded as consecutive launches of kSclWsChunk (each two
// full rounds of the chip's 2048 resident waves at L = 8) that reuse one chunk's workspace:
// 22 KB per codeword at n = 1024 bounds it to 360 MB whatever the batch.
constexpr int64_t kSclWsChunk = 16384;
size_t scl_tree_workspace_size(const pl_plan* p, int64_t bs) {
    if (!scl_tree_eligible(p) || p->f_mode != PL_F_EXACT || bs <= 0) return 0;
    const int V = pick_v(p->log_n);
    if (V < 1) return 0;
    const int cpw = 32 / p->list_size;
    const int64_t b = bs < kSclWsChunk ? bs : kSclWsChunk;  // larger batches run in chunks of kSclWsChunk
    const int64_t slots = (b + cpw - 1) / cpw * cpw;
    return (size_t)slots * (size_t)cache_size(p->n, V) * sizeof(double);
}

int launch_scl_tree(const pl_plan* p, const float* llr, int64_t bs, void* out, int out_kind, double* out_pm,
                    void* ws, size_t ws_bytes, hipStream_t st) {
    if (bs == 0) return PL_OK;
    if (bs > 0x7fffffffLL) {
        set_error("SCL decode: batch too large for one launch");
        return PL_EINVAL;
    }
    const int S = p->log_n, L = p->list_size, V = pick_v(S);
    const bool exact = p->f_mode == PL_F_EXACT;
    const bool fast = (p->flags & PL_PLAN_FAST_SCL) != 0;
    const void* fn = nullptr;
#ifdef PL_SCL_VARIANT_ONLY_L8  // development variant libraries (tools/scl_variants.py)
    if (L != 8) {
        set_error("variant library: L = 8 only");
        return PL_ENOTSUP;
    }
    fn = scl_tree_fn<8>(V, exact, fast);
#else
    switch (L) {
        case 2: fn = scl_tree_fn<2>(V, exact, fast); break;
        case 4: fn = scl_tree_fn<4>(V, exact, fast); break;
        case 8: fn = scl_tree_fn<8>(V, exact, fast); break;
        case 16: fn = scl_tree_fn<16>(V, exact, fast); break;
        default: fn = scl_tree_fn<32>(V, exact, fast); break;
    }
#endif
    const Lay y = make_layout(p->n, S, L, V);
    const int cpw = 32 / L;  // codewords per wave: one 2L-lane group each
    const int lds = cpw * y.bytes;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return check_hip(e, "SCL decode: LDS attribute");
    }
    int n = p->n, k = p->k, cdeg = p->crc_deg;
    double lmax = (double)p->llr_max;
    uint32_t cg = p->crc_g;
    const uint32_t* fw = p->d_frozen_words;
    const int32_t* ip = p->d_info_pos;
    double* vc = ws_bytes >= scl_tree_workspace_size(p, bs) && scl_tree_workspace_size(p, bs) > 0
                     ? static_cast<double*>(ws) : nullptr;
    const int64_t chunk = vc != nullptr ? kSclWsChunk : bs;  // the workspace holds one chunk's slots
    const size_t out_elem = out_kind == PL_OUT_F32 ? sizeof(float) : sizeof(uint8_t);
    for (int64_t off = 0; off < bs; off += chunk) {
        int64_t cbs = bs - off < chunk ? bs - off : chunk;
        const float* cllr = llr + off * n;
        void* cout = static_cast<unsigned char*>(out) + (size_t)off * (size_t)k * out_elem;
        double* cpm = out_pm != nullptr ? out_pm + off * 2 * L : nullptr;
        void* args[] = {(void*)&cllr, (void*)&cbs, (void*)&cout, (void*)&out_kind, (void*)&cpm, (void*)&fw,
                        (void*)&ip, (void*)&n, (void*)&S, (void*)&k, (void*)&lmax, (void*)&cdeg, (void*)&cg, (void*)&vc};
        const int64_t blocks = (cbs + cpw - 1) / cpw;
        hipError_t e = hipLaunchKernel(fn, dim3((unsigned)blocks), dim3(64), args, lds, st);
        if (e != hipSuccess) return check_hip(e, "SCL decode launch (subtree kernel)");
    }
    return check_hip(hipGetLastError(), "SCL decode launch (subtree kernel)");
}

}  // namespace pl
#endif  // PL_SCL_TREE_DISPATCH
