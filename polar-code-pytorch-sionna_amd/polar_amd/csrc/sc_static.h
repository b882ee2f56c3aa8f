// sc_static.h -- code-specialised SC polar decoder kernel for gfx950 (MI355X).
//
// This header is compiled once per frozen set: at plan time through hiprtc (jit.cpp), or
// ahead of time for the codes build.py pre-compiles.  The code is described by a struct
//   struct PlCode { static constexpr int LOG_N = ..; static constexpr int FM = ..;
//                   static constexpr unsigned char NT[2 * N] = {..}; };
// where NT is the node-type table in heap order (node of size 2^s at position p has index
// (N >> s) + (p >> s)); types R0/R1/REP/SPC/GEN as classified by capi.cpp.  Every branch on a
// node type is therefore resolved at compile time: the decoder is a straight-line program for
// that code (the "unrolled decoder" of the fast-SSC literature), with data-dependent branches
// only where an exactness precondition of a shortcut can fail.
//
// Reference semantics (bit-exact): x_run_sn_polar/polar/polar_sc.py -- f = min-sum on clipped
// inputs (:33-48, min-sum forced at :46), g = (1-2u)x + y unclipped (:49-53), leaf u = 1 iff
// llr <= 0 (:90-98), partial sums [uL^uR, uR] (:83-89).  FM = 1 selects the exact boxplus f of
// my_sn/fec/polar/dec.py:39-43 (shortcuts limited to rate-0 and repetition nodes there).
//
// Layout ("mirror butterfly").  A wave64 decodes 64/G codewords, G = max(1, n/128) lanes each
// (n/64 lanes for min-sum n = 256 .. 1024, jit.cpp static_log_g).
// Element i of a stage buffer lives in slot i/G of the lane holding residue i mod G.  Residues
// are placed so that the two residues an f/g pairs at every level of the bottom of the tree
// (r and r + S/2 inside a size-S block, S <= G) sit in lanes q and q ^ (S-1): the "mirror" of a
// 2/4/8/16-lane block, which is ONE DPP op (quad_perm / row_half_mirror / row_mirror).  A node
// of size S <= G is decoded replicated: both lanes of a mirror pair compute the same value
// (f is symmetric, g adds commutatively, the sign flip is exact), so no gather and no
// broadcast is ever needed.  Nodes of size >= 2G pair slots j and j + E/2 inside one lane.
//
// Exact node shortcuts (what the reference recursion computes, not approximations):
//   rate-0     beta = 0
//   REP        u = HD(sum of the node LLRs in SC's pairwise g order), beta = u...u
//   rate-1     beta = HD(alpha) when no node LLR is exactly 0                  (min-sum only)
//   SPC        beta = HD(alpha), flip at the unique min |alpha| < llr_max when the parity is
//              odd; requires no zero LLR and, for odd parity, a unique unclipped min (min-sum only)
// When a precondition fails anywhere in the wave the node is decoded by the full recursion.
#ifndef PL_SC_STATIC_H
#define PL_SC_STATIC_H
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#else  // hiprtc: no libc headers
typedef unsigned char uint8_t;
typedef int int32_t;
typedef unsigned int uint32_t;
typedef long long int64_t;
typedef unsigned long long uint64_t;
typedef unsigned long uintptr_t;
#endif
#include "exactf.h"  // build.py inlines it into the embedded source

// Tuning macros (overridable per build; development libraries, -DPL_DEV=1, take A/B overrides from jit.cpp)
#ifndef PL_SC_F_BITOP3
#define PL_SC_F_BITOP3 0  // A/B on MI355X: 1 (explicit v_bitop3 sign merge) was slower
#endif
#ifndef PL_SC_F_BOUNDED
#define PL_SC_F_BOUNDED 1  // min-sum f of a left child (inputs are f outputs, |x|, |y| <= llr_max) as one med3
#endif
#ifndef PL_SC_LANE31
#define PL_SC_LANE31 1  // lane-level partial sums as bit-31-only flags (one-op hard decision, bitop3 combines)
#endif
#ifndef PL_SC_EMIT_PRE
#define PL_SC_EMIT_PRE 1  // preload the output table entries at kernel start (8 VGPRs)
#endif
#ifndef PL_SC_BIT31_ASM
#define PL_SC_BIT31_ASM 0  // 1: opaque shift (no v_mul_lo fusion); measured slower overall
#endif
#ifndef PL_SC_SPC_BALLOT
#define PL_SC_SPC_BALLOT 0  // 1: SALU ballot uniqueness test instead of a DPP count; measured slower
#endif
#ifndef PL_SC_HD_SUB
#define PL_SC_HD_SUB 1  // leaf decisions as one fp32 subtract of the smallest denormal
#endif
#ifndef PL_SC_VA_RECOMPUTE
#define PL_SC_VA_RECOMPUTE 0  // 1: recompute the left virtual LLRs for the g pass (-32 VGPRs); measured slower
#endif
#ifndef PL_SC_CH_LDS
#define PL_SC_CH_LDS 1  // the upper half of the channel slots lives in LDS (LDS-DMA), not VGPRs (see Ch)
#endif
#ifndef PL_SC_DMA_ASM
#define PL_SC_DMA_ASM 1  // LDS-DMA of the channel half in the saddr form (inline asm)
#endif
#ifndef PL_SC_NT
#define PL_SC_NT 2  // non-temporal hints: bit 0 channel loads, bit 1 output stores (see st_out4)
#endif
#ifndef PL_SC_WIDE
#define PL_SC_WIDE 16  // in-lane partial sums of nodes with <= this many slots per lane: one word per slot
#endif
#ifndef PL_SC_PK_G
#define PL_SC_PK_G 1  // in-lane g adds in pairs (v_pk_add_f32)
#endif
#ifndef PL_SC_ROOT_MODE
#define PL_SC_ROOT_MODE 0
#endif
#ifndef PL_SC_MINW
#define PL_SC_MINW 2
#endif
#ifndef PL_SC_STAMPS
#define PL_SC_STAMPS 0
#endif
#ifndef PL_SC_DIAG_SKIP_LANE
#define PL_SC_DIAG_SKIP_LANE 0
#endif
#ifndef PL_SC_DIAG_NO_LOAD
#define PL_SC_DIAG_NO_LOAD 0
#endif
#ifndef PL_SC_DIAG_NO_TREE
#define PL_SC_DIAG_NO_TREE 0
#endif
#ifndef PL_SC_DIAG_SKIP_SPECIAL
#define PL_SC_DIAG_SKIP_SPECIAL 0
#endif
// Diagnostic macros (timing ablations with WRONG results) exist only in development builds
// (jit.cpp marks a PL_DEV library's sources with PL_DEV).
#if !defined(PL_DEV) && (PL_SC_DIAG_SKIP_LANE || PL_SC_DIAG_NO_LOAD || PL_SC_DIAG_NO_TREE || PL_SC_DIAG_SKIP_SPECIAL)
#error "PL_SC_DIAG_* macros give wrong results: development builds (PL_DEV) only"
#endif
#ifndef PL_SC_PERSIST
#define PL_SC_PERSIST 0  // 1: persistent software-pipelined waves (grid = resident waves)
#endif
// PL_SC_PERSIST 2: persistent waves whose next batch of channel rows is staged in LDS by an
// asynchronous global->LDS copy (global_load_lds_dwordx4) while the current batch is decoded:
// no channel-load latency on the critical path, 2 waves/SIMD (the staging takes 16 KiB of LDS
// per wave at n = 1024).  Needs N >= 256 (whole 1-KiB copies per row).

namespace pls {

enum : int { R0 = 0, R1 = 1, REP = 2, SPC = 3, GEN = 4 };
enum : int { OUT_F32 = 0, OUT_U8 = 1, OUT_CNT = 2, OUT_SIM = 3 };
#ifndef PL_SC_KWAVES
// One-wave work-groups: a wave's slot and its 8 KiB of LDS are refilled as soon as it retires,
// instead of when the slowest of its work-group's four waves does (the waves of a SIMD finish
// up to 1.5x apart).  Same-process A/B (profiles/r02zu_sc_ab_waves.txt, r02zv_*): (512,1024)
// 0.0813 / 0.0807 vs 0.0817 / 0.0815 ms, (128,256) bs = 4096 0.0078 vs 0.0079 ms.
#define PL_SC_KWAVES 1
#endif
constexpr int kWaves = PL_SC_KWAVES;  // waves per workgroup (the launcher reads pl_sc_waves)

template <bool B, class T, class F>
struct Cond {
    using type = T;
};
template <class T, class F>
struct Cond<false, T, F> {
    using type = F;
};
template <int E>
using Beta = typename Cond<(E <= 32), uint32_t, uint64_t>::type;

// PL_SC_CH_LDS applies to n = 1024 at 16 lanes per codeword (64 channel slots per lane): 8 KiB of
// LDS per wave, 32 KiB per block, so four blocks fit a CU's 160 KiB, and the 32 VGPRs saved
// (133 -> 103) lift the kernel from three to four waves per SIMD: 0.0854 vs 0.0882 ms at
// (512,1024), bs = 65536 (profiles/r02s_sc_ab_ch_lds.txt).  At n = 64 ... 512 the kernel already
// ran at that occupancy and the LDS round trip only costs (+4 ... +39 %), so they keep VGPRs.
template <class C>
struct Ch {
    static constexpr int CHL = (PL_SC_CH_LDS && C::NS == 64 && C::LOG_N == 10) ? 1 : 0;
};

template <class C>
constexpr int nt(int s, int p) {
    return C::NT[(C::N >> s) + (p >> s)];
}
// The stage-s node at position p is the left child of its parent: its input is the parent's f
// output, bounded by llr_max in magnitude.
template <class C>
constexpr bool lchild(int s, int p) {
    return s < C::LOG_N && ((p >> s) & 1) == 0;
}

template <int E>
__device__ __forceinline__ Beta<E> ones() {
    return (Beta<E>)(~(Beta<E>)0 >> (8 * sizeof(Beta<E>) - E));
}

__device__ __forceinline__ uint32_t fu(float x) { return __float_as_uint(x); }
__device__ __forceinline__ float uf(uint32_t x) { return __uint_as_float(x); }

// Output rows are written once: with the non-temporal hint (PL_SC_NT bit 1) they do not push
// the channel rows out of L2 / the Infinity Cache.  Measured with every launch streaming a batch
// the Infinity Cache does not hold (sc_ab.py --rotate 3): 0.0809 vs 0.0841 ms; non-temporal channel
// loads (bit 0) were slower here (0.0875 ms) although a load/store-only kernel of the same shapes
// gains with both hints (5.78 vs 5.38 TB/s, tools/micro/load_pattern.hip).
__device__ __forceinline__ float ld_ch(const float* p) {
#if PL_SC_NT & 1
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_out4(float* p, float4 v) {
#if PL_SC_NT & 2
    const f4v w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<f4v*>(p));
#else
    *reinterpret_cast<float4*>(p) = v;
#endif
}

// Mirror inside aligned blocks of S lanes: lane q reads lane q ^ (S-1).  One DPP op.
template <int S>
__device__ __forceinline__ uint32_t mir(uint32_t v) {
    static_assert(S == 2 || S == 4 || S == 8 || S == 16, "mirror block");
    constexpr int ctrl = S == 2 ? 0xB1 : S == 4 ? 0x1B : S == 8 ? 0x141 : 0x140;
    // mov_dpp (no "old" operand, bound_ctrl) lets the DPP combiner fold the move into its user.
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xF, 0xF, true);
}
template <int S>
__device__ __forceinline__ float mirf(float v) {
    return uf(mir<S>(fu(v)));
}

__device__ __forceinline__ float flip31(float x, uint32_t t);

// f: polar_sc.py:46 (min-sum of clipped inputs) or my_sn dec.py:39-43 (exact boxplus).
// BND: the inputs are known to satisfy |x|, |y| <= lmax -- they are the f outputs of the parent,
// i.e. the node is a left child (lchild below) -- so the clip is the identity and
//   sign(x) sign(y) min(|x|, |y|) = med3(-|x|, sign(x) y, |x|)
// (y' = y with x's sign applied, clamped to [-|x|, |x|]): one bitop3 + one med3 instead of
// min3 + xor + bitop3.  Exact: both pick an input magnitude; only the sign of a zero result can
// differ, and no decision observes it (every test treats +0 and -0 alike).
template <int FM, bool BND = false>
__device__ __forceinline__ float fop(float x, float y, float lmax) {
    if constexpr (FM == 0) {
#if PL_SC_F_BOUNDED
        if constexpr (BND) return __builtin_amdgcn_fmed3f(-fabsf(x), flip31(y, fu(x)), fabsf(x));
#endif
        const float m = fminf(fminf(fabsf(x), fabsf(y)), lmax);
#if PL_SC_F_BITOP3
        // m | ((x ^ y) & sign): v_min3 + v_xor + v_bitop3 ((S0 & S1) | S2, table 0xEA)
        return uf(__builtin_amdgcn_bitop3_b32(fu(x) ^ fu(y), 0x80000000u, fu(m), 0xEA));
#else
        return uf(fu(m) | ((fu(x) ^ fu(y)) & 0x80000000u));
#endif
    } else {
        return plx::f_exact(x, y, lmax);  // my_sn dec.py:39-43, correctly rounded exp / log (exactf.h)
    }
}
// x[j] = f(a[j], a[j + H]), j < H.  Exact f: element pairs through plx::f_exact2 (half the
// calls, two interleaved evaluations per call).
#ifndef PL_SC_FEX_PAIR
#define PL_SC_FEX_PAIR 1
#endif
#ifndef PL_SC_FEX_LANE
#define PL_SC_FEX_LANE 1  // exact f of lane-level nodes split over the lanes holding the pair (f_lane_exact)
#endif
#ifndef PL_SC_G_NODPP
#define PL_SC_G_NODPP 0  // 1: lane-level g as two flips and a plain add, no DPP read of a fresh value and
                         // no hazard s_nop (A/B r04zl, (512,1024): 1.3 % slower)
#endif
template <int FM, bool BND, int H>
__device__ __forceinline__ void fvec(const float* a, float* x, float lmax) {
    if constexpr (FM == 1 && H >= 2 && PL_SC_FEX_PAIR) {
#pragma unroll
        for (int j = 0; j < H; j += 2) {
            const plx::f2 r = plx::f_exact2(a[j], a[j + H], a[j + 1], a[j + 1 + H], lmax);
            x[j] = r.a;
            x[j + 1] = r.b;
        }
    } else {
#pragma unroll
        for (int j = 0; j < H; ++j) x[j] = fop<FM, BND>(a[j], a[j + H], lmax);
    }
}
// g, polar_sc.py:49-53: (1-2u)x + y == (u ? -x : x) + y, one rounding.  The flip is the sign
// bit (bit 31) of t; bitop3 S1 ^ (S0 & S2) (table 0x6c) applies it in one op.
__device__ __forceinline__ float flip31(float x, uint32_t t) {
    return uf(__builtin_amdgcn_bitop3_b32(t, fu(x), 0x80000000u, 0x6c));
}
__device__ __forceinline__ float gop(float x, float y, uint32_t t) { return flip31(x, t) + y; }
// bit j of packed partial sums w moved to bit 31 with one shift (lower bits are don't-care for
// flip31); j is a compile-time constant after unrolling
template <typename W>
__device__ __forceinline__ uint32_t bit31(W w, int j) {
    uint32_t t = j <= 31 ? (uint32_t)(w << (31 - j)) : (uint32_t)(w >> (j - 31));
#if PL_SC_BIT31_ASM
    asm("" : "+v"(t));  // keep it one v_lshlrev (only bit 31 is demanded: LLVM would fuse shifts into v_mul_lo)
#endif
    return t;
}
// hard decision of a leaf, u = 1 iff !(llr > 0) (polar_sc.py:94-97), as a bit-31 flag.
// PL_SC_LANE31: only bit 31 of a lane-level flag is meaningful (its consumers mask with the
// lo31 lane masks or shift by 31), so the decision is one arithmetic op, no compare, no VCC.
// PL_SC_HD_SUB=0 form: one saturating subtract on the bit pattern -- bits(x) - 1 is negative iff
// bits(x) <= 0 as a signed integer, i.e. x <= +0 or x < 0 (no NaN), and the saturation keeps -0
// (INT_MIN) negative.  The default form is a plain fp32 subtract, which issues faster on gfx950
// (tools/micro/issue_cost*.hip: v_add_f32 ~1.1 ns, v_add_i32 clamp ~1.8 ns per wave-instruction).
#if PL_SC_LANE31 && PL_SC_HD_SUB
// x - 2^-149 (the smallest denormal) is negative exactly when x <= 0: +0 and -0 give -2^-149,
// x = 2^-149 gives +0 (an exact zero rounds to +0), larger x stay positive.  Needs fp32 denormals
// preserved, which both build paths keep (no FTZ flag: .amdhsa_float_denorm_mode_32 3); the
// exact-zero golden sets would catch a flushing build.
__device__ __forceinline__ uint32_t hd31(float x) { return fu(x - 1.40129846e-45f); }
#elif PL_SC_LANE31
__device__ __forceinline__ uint32_t hd31(float x) {
    return (uint32_t)__builtin_elementwise_sub_sat((int32_t)fu(x), (int32_t)1);
}
#else
__device__ __forceinline__ uint32_t hd31(float x) { return (x > 0.0f) ? 0u : 0x80000000u; }
#endif
__device__ __forceinline__ uint32_t hd(float x) { return (x > 0.0f) ? 0u : 1u; }

// wave-wide "any lane": the ballot builtin directly (hiprtc's __any materialises the predicate
// as 0/1 and compares it again: +400 VALU and +300 branches at (512,1024))
__device__ __forceinline__ bool any_lane(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }
__device__ __forceinline__ uint64_t ballot_lanes(bool p) { return __builtin_amdgcn_ballot_w64(p); }

struct Lane {
#if PL_SC_LANE31
    // lo31[t]: 0x80000000 if this lane holds the low element of its pair at
    // level 2^t, else 0 (bitop3 operands; opaque to the compiler, see decode())
    uint32_t lo31[5];
    __device__ __forceinline__ uint32_t lom(int t) const { return (uint32_t)((int32_t)lo31[t] >> 31); }
#else
    uint32_t lom_[5];  // lom[t]: all-ones if this lane holds the low element at level 2^t
    __device__ __forceinline__ uint32_t lom(int t) const { return lom_[t]; }
#endif
    float lmax;
    const float* chl;  // PL_SC_CH_LDS: this lane's first LDS channel word (slot NS/2), stride 64 words
};

// ---------------- reductions over the G lanes of a codeword (all lanes get the result) ----
template <int LG, typename T, typename Op>
__device__ __forceinline__ T grp(T v, Op op) {
    if constexpr (LG >= 4) v = op(v, (T)mir<16>((uint32_t)v));
    if constexpr (LG >= 3) v = op(v, (T)mir<8>((uint32_t)v));
    if constexpr (LG >= 2) v = op(v, (T)mir<4>((uint32_t)v));
    if constexpr (LG >= 1) v = op(v, (T)mir<2>((uint32_t)v));
    return v;
}
// SC-order sum: level 2^t pairs lanes q and q ^ (2^t - 1) (residues r, r + 2^(t-1)).
template <int LG>
__device__ __forceinline__ float grp_sumf(float v) {
    if constexpr (LG >= 4) v = v + mirf<16>(v);
    if constexpr (LG >= 3) v = v + mirf<8>(v);
    if constexpr (LG >= 2) v = v + mirf<4>(v);
    if constexpr (LG >= 1) v = v + mirf<2>(v);
    return v;
}
// wave mask with the lowest lane of every aligned S-lane block set
template <int S>
__device__ __forceinline__ constexpr uint64_t blocklow() {
    return S == 1 ? ~0ull : S == 2 ? 0x5555555555555555ull : S == 4 ? 0x1111111111111111ull
         : S == 8 ? 0x0101010101010101ull : 0x0001000100010001ull;
}
// True if some S-lane block whose lanes are set in `live` has two or more lanes set in `m`
// (m must have at least one lane set in every block): subtracting 1 per block clears each
// block's lowest set lane without borrowing across blocks.
template <int S>
__device__ __forceinline__ bool multi_in_block(uint64_t m, uint64_t live) {
    return ((m & (m - blocklow<S>())) & live) != 0;
}

// ---------------- lane-level nodes: size 2^s <= G, one (replicated) LLR per lane ----------
// Partial sums are returned as bit-31 flags (0 / 0x80000000) so g consumes them directly.
template <class C, int s, int P>
__device__ uint32_t lnode(float a, const Lane& ln);

// Exact f of a lane-level node (FM = 1), the transcendentals split over the lanes that hold the
// same pair.  At a node of size S <= G lane q pairs with q ^ (S-1); below the top lane level
// (S < G) lane q ^ (2S-1) holds a copy of lane q's value (its parent's f / g is symmetric), so
// four lanes evaluate the same f: the low half of each 2S-lane block (role A) takes
// log(1 + exp(x + y)), the high half (role B) log(exp(x) + exp(y)) -- each lane one exp of its
// own argument, the pair's sum e^x + e^y by one mirror DPP, one log -- and the halves swap their
// logs with one more mirror.  At S = G only the two lanes of the pair share the f: both take
// exp of their own value and of x + y, then one log each (role A: the lane holding the pair's
// low element).  Every lane ends with the same bits as f_exact(x, y) -- each sum is commutative,
// each transcendental correctly rounded -- so the replication the layout relies on holds.
// 1 exp + 1 log per lane (S < G) or 2 + 1 (S = G) instead of 3 + 2.
// Inlined, the lane-level f drops its call overhead (argument moves, the ABI's register
// constraints); only with a fixed range (PL_EXF_RANGE != 0), where it has no full-range path.
#ifndef PL_SC_FLANE_INLINE
#define PL_SC_FLANE_INLINE 0
#endif
#if PL_SC_FLANE_INLINE && PL_EXF_RANGE == 0
#error "PL_SC_FLANE_INLINE needs PL_EXF_RANGE 1 or 2"
#endif
#if PL_SC_FLANE_INLINE
#define PL_FLANE_ATTR __attribute__((always_inline))
#else
#define PL_FLANE_ATTR __attribute__((noinline))
#endif
template <int S, bool TOP>
__device__ PL_FLANE_ATTR float f_lane_exact(float a, float y, uint32_t role31, float lmax) {
    lmax = plx::uniform_l(lmax);
    if (plx::wide_range(lmax)) return plx::f_exact_wide(a, y, lmax);
    const float xc = plx::clip_l(a, lmax), yc = plx::clip_l(y, lmax);
    const bool A = (int32_t)role31 < 0;
    float arg;
    if constexpr (TOP) {
#if PL_EXF_LEAN
        // e^(x+y) from the pair's two fp64 exps (exactf.h exp_sum) instead of a third exp
        const double ed = plx::exp_d(xc);
        const unsigned long long eb = (unsigned long long)__double_as_longlong(ed);
        const uint32_t plo = mir<S>((uint32_t)eb), phi = mir<S>((uint32_t)(eb >> 32));
        const double edp = __longlong_as_double((long long)(((unsigned long long)phi << 32) | plo));
        const float e = (float)ed;
        const float es = e + (float)edp;  // e^x + e^y in both lanes of the pair
        const float e1 = plx::exp_sum(ed, edp, xc, yc);
#else
        const float e = plx::exp_cr(xc);
        const float es = e + mirf<S>(e);  // e^x + e^y in both lanes of the pair
        const float e1 = plx::exp_cr(xc + yc);
#endif
        arg = A ? 1.0f + e1 : es;
    } else {
        const float e = plx::exp_cr(A ? xc + yc : xc);
        const float es = e + mirf<S>(e);  // role B: e^x + e^y (its partner is role B too)
        arg = A ? 1.0f + e : es;
    }
    const float l = plx::log_cr(arg);
    float lo;  // the other role's log
    if constexpr (TOP) lo = mirf<S>(l);
    else lo = mirf<2 * S>(l);
    return A ? l - lo : lo - l;
}

template <class C, int s, int P>
__device__ __forceinline__ uint32_t lsplit(float a, const Lane& ln) {
    constexpr int S = 1 << s;
    const float y = mirf<S>(a);
    uint32_t bl = 0;
    if constexpr (nt<C>(s - 1, P) != R0) {
        float x;
        if constexpr (C::FM == 1 && PL_SC_FEX_LANE) {
            // role bit: the pair's low element (S = G), the low half of the 2S-block (S < G)
#if PL_SC_LANE31
            const uint32_t role = s == C::LOG_G ? ln.lo31[s] : ln.lo31[s + 1];
#else
            const uint32_t role = s == C::LOG_G ? ln.lom(s) : ln.lom(s + 1);
#endif
            x = f_lane_exact<S, s == C::LOG_G>(a, y, role, ln.lmax);
        } else {
            x = fop<C::FM, lchild<C>(s, P)>(a, y, ln.lmax);
        }
        bl = lnode<C, s - 1, P>(x, ln);
    }
#if PL_SC_LANE31
    // both lanes of the pair evaluate (1-2u) alpha_lo + alpha_hi: the low lane flips its own
    // value (bitop3 S1 ^ (S0 & S2) with the lane's bit-31 mask), the high lane keeps its own, and
    // one DPP add sums the pair in both lanes (fp32 addition is commutative: same bits)
#if PL_SC_G_NODPP
    // the same sum without reading the just-flipped value across lanes (no DPP hazard wait): the
    // low lane flips its own value, the high lane the partner's copy y (taken before the left
    // subtree), and both add -- the same two operands, so the same bits
    const float x = uf(__builtin_amdgcn_bitop3_b32(bl, fu(a), ln.lo31[s], 0x6c)) +
                    uf(__builtin_amdgcn_bitop3_b32(bl, fu(y), ln.lo31[s] ^ 0x80000000u, 0x6c));
#else
    const float v = uf(__builtin_amdgcn_bitop3_b32(bl, fu(a), ln.lo31[s], 0x6c));
    const float x = v + mirf<S>(v);
#endif
    const uint32_t br = lnode<C, s - 1, P + S / 2>(x, ln);
    return __builtin_amdgcn_bitop3_b32(bl, br, ln.lo31[s], 0x6c);  // br ^ (bl & lo31)
#else
    const uint32_t L = ln.lom(s);
    const float x = uf(__builtin_amdgcn_bitop3_b32(bl, fu(a), L, 0x6c)) +
                    uf(__builtin_amdgcn_bitop3_b32(bl, fu(y), L, 0x9c));
    const uint32_t br = lnode<C, s - 1, P + S / 2>(x, ln);
    return br ^ (bl & L);
#endif
}

template <class C, int s, int P>
__device__ __forceinline__ uint32_t lnode(float a, const Lane& ln) {
    constexpr int T = nt<C>(s, P);
#if PL_SC_DIAG_SKIP_LANE
    if constexpr (s == C::LOG_G) return hd31(a);  // diagnostic only: timing without the lane-level subtrees
#endif
    if constexpr (T == R0) {
        return 0u;
    } else if constexpr (s == 0) {
        return hd31(a);
    } else if constexpr (T == REP) {
        float v = a;
        if constexpr (s >= 4) v = v + mirf<16>(v);
        if constexpr (s >= 3) v = v + mirf<8>(v);
        if constexpr (s >= 2) v = v + mirf<4>(v);
        v = v + mirf<2>(v);
        return hd31(v);
    } else if constexpr (T == R1 && C::FM == 0) {
#if PL_SC_LANE31
        if (!any_lane(a == 0.0f)) return fu(a);  // bit 31 = the decision
#else
        if (!any_lane(a == 0.0f)) return fu(a) & 0x80000000u;
#endif
        return lsplit<C, s, P>(a, ln);
    } else if constexpr (T == SPC && C::FM == 0) {
        // magnitudes compared as integers (non-negative floats order like their bit patterns)
        constexpr int S = 1 << s;
        const uint32_t b = fu(a) & 0x80000000u;
        const uint32_t ab = fu(a) & 0x7FFFFFFFu;
        uint32_t par = b, mn = ab;
        if constexpr (s >= 4) { par ^= mir<16>(par); mn = min(mn, mir<16>(mn)); }
        if constexpr (s >= 3) { par ^= mir<8>(par); mn = min(mn, mir<8>(mn)); }
        if constexpr (s >= 2) { par ^= mir<4>(par); mn = min(mn, mir<4>(mn)); }
        par ^= mir<2>(par);
        mn = min(mn, mir<2>(mn));
        const bool eq = ab == mn;
#if PL_SC_SPC_BALLOT
        const bool bad_lane = (ab == 0u) | ((par != 0u) & (mn >= fu(ln.lmax)));
        const bool bad = any_lane(bad_lane) || multi_in_block<S>(ballot_lanes(eq), ballot_lanes(par != 0u));
#else
        uint32_t cnt = eq ? 1u : 0u;
        if constexpr (s >= 4) cnt += mir<16>(cnt);
        if constexpr (s >= 3) cnt += mir<8>(cnt);
        if constexpr (s >= 2) cnt += mir<4>(cnt);
        cnt += mir<2>(cnt);
        const bool bad = any_lane((ab == 0u) | ((par != 0u) & ((cnt != 1u) | (mn >= fu(ln.lmax)))));
#endif
        if (!bad) return b ^ (eq ? par : 0u);
        return lsplit<C, s, P>(a, ln);
    } else {
        return lsplit<C, s, P>(a, ln);
    }
}

// ---------------- in-lane nodes: size 2^s >= 2G, E = 2^s / G slots per lane ---------------
// Partial sums of a node with E <= PL_SC_WIDE slots per lane are kept "wide": one word per slot
// whose bit 31 is the bit (lower bits are don't-care), so g applies a flag with one bitop3 and the
// combine [bl ^ br, br] is E/2 XORs -- no bit extraction (v_lshlrev) per g element.  Larger nodes
// keep packed words (bit j = slot j), which bounds the registers of the long-lived upper stages.
template <int E>
struct Wide {
    uint32_t w[E];
};
template <int E>
using BV = typename Cond<(E <= PL_SC_WIDE), Wide<E>, Beta<E>>::type;

template <int E>
__device__ __forceinline__ uint32_t flag(const Wide<E>& b, int j) { return b.w[j]; }
__device__ __forceinline__ uint32_t flag(uint32_t b, int j) { return bit31(b, j); }
__device__ __forceinline__ uint32_t flag(uint64_t b, int j) { return bit31(b, j); }

template <int E>
__device__ __forceinline__ BV<E> bzero() {
    BV<E> r;
    if constexpr (E <= PL_SC_WIDE) {
#pragma unroll
        for (int j = 0; j < E; ++j) r.w[j] = 0u;
    } else {
        r = 0;
    }
    return r;
}
// packed words of a wide partial-sum vector: bit j = bit 31 of word j.  One v_alignbit per bit:
// alignbit(acc, w, 31) = (acc << 1) | (w >> 31), inserting from the top slot down.
template <int E>
__device__ __forceinline__ Beta<E> packed(const Wide<E>& b) {
    Beta<E> r = 0;
    if constexpr (E <= 32) {
        uint32_t acc = b.w[E - 1] >> 31;
#pragma unroll
        for (int j = E - 2; j >= 0; --j) acc = __builtin_amdgcn_alignbit(acc, b.w[j], 31);
        r = acc;
    } else {
        uint32_t lo = b.w[31] >> 31, hi = b.w[E - 1] >> 31;
#pragma unroll
        for (int j = 30; j >= 0; --j) lo = __builtin_amdgcn_alignbit(lo, b.w[j], 31);
#pragma unroll
        for (int j = E - 2; j >= 32; --j) hi = __builtin_amdgcn_alignbit(hi, b.w[j], 31);
        r = ((uint64_t)hi << 32) | lo;
    }
    return r;
}
__device__ __forceinline__ uint32_t packed(uint32_t b) { return b; }
__device__ __forceinline__ uint64_t packed(uint64_t b) { return b; }

// [bl ^ br, br] (polar_sc.py:83-89)
template <int H>
__device__ __forceinline__ BV<2 * H> combine(const BV<H>& bl, const BV<H>& br) {
    BV<2 * H> r;
    if constexpr (2 * H <= PL_SC_WIDE) {
#pragma unroll
        for (int j = 0; j < H; ++j) {
            r.w[j] = bl.w[j] ^ br.w[j];
            r.w[j + H] = br.w[j];
        }
    } else {
        using BT = Beta<2 * H>;
        const Beta<H> pl = packed(bl), pr = packed(br);
        r = (BT)(pl ^ pr) | ((BT)pr << H);
    }
    return r;
}

template <class C, int s, int P>
__device__ BV<(1 << s) / C::G> node(const float (&a)[(1 << s) / C::G], const Lane& ln);

template <class C, int s, int P>
__device__ __forceinline__ BV<(1 << (s - 1)) / C::G> child(const float (&x)[(1 << (s - 1)) / C::G], const Lane& ln) {
    if constexpr ((1 << (s - 1)) == C::G) {
#if PL_SC_WIDE >= 1
        return Wide<1>{{lnode<C, s - 1, P>(x[0], ln)}};
#else
        return (Beta<1>)(lnode<C, s - 1, P>(x[0], ln) >> 31);
#endif
    } else {
        return node<C, s - 1, P>(x, ln);
    }
}

typedef float f2v __attribute__((ext_vector_type(2)));
// x[j] = g(a[j], a[j + H], flag j of bl) for j < H (polar_sc.py:49-53), two adds per v_pk_add_f32
template <int H, typename B>
__device__ __forceinline__ void gvec(const float (&a)[2 * H], const B& bl, float (&x)[H]) {
    if constexpr (H >= 2 && PL_SC_PK_G) {
#pragma unroll
        for (int j = 0; j < H; j += 2) {
            const f2v u = {flip31(a[j], flag(bl, j)), flip31(a[j + 1], flag(bl, j + 1))};
            const f2v w = {a[j + H], a[j + 1 + H]};
            const f2v r = u + w;
            x[j] = r.x;
            x[j + 1] = r.y;
        }
    } else {
#pragma unroll
        for (int j = 0; j < H; ++j) x[j] = gop(a[j], a[j + H], flag(bl, j));
    }
}

template <class C, int s, int P>
__device__ __forceinline__ BV<(1 << s) / C::G> split(const float (&a)[(1 << s) / C::G], const Lane& ln) {
    constexpr int E = (1 << s) / C::G, H = E / 2, h = 1 << (s - 1);
    float x[H];
    BV<H> bl = bzero<H>();
    if constexpr (nt<C>(s - 1, P) != R0) {
        fvec<C::FM, lchild<C>(s, P), H>(a, x, ln.lmax);
        bl = child<C, s, P>(x, ln);
        gvec<H>(a, bl, x);
    } else {
#pragma unroll
        for (int j = 0; j < H; ++j) x[j] = a[j] + a[j + H];
    }
    const BV<H> br = child<C, s, P + h>(x, ln);
    return combine<H>(bl, br);
}

template <class C, int E>
__device__ __forceinline__ Beta<E> signs(const float (&a)[E]) {
    Beta<E> b = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) b |= (Beta<E>)(fu(a[j]) >> 31) << j;
    return b;
}
template <int E>
__device__ __forceinline__ BV<E> from_packed(Beta<E> b) {
    if constexpr (E <= PL_SC_WIDE) {
        Wide<E> r;
#pragma unroll
        for (int j = 0; j < E; ++j) r.w[j] = bit31(b, j);
        return r;
    } else {
        return b;
    }
}

template <class C, int s, int P>
__device__ __forceinline__ BV<(1 << s) / C::G> node(const float (&a)[(1 << s) / C::G], const Lane& ln) {
    constexpr int E = (1 << s) / C::G;
    constexpr int T = nt<C>(s, P);
    using BT = Beta<E>;
    constexpr bool WIDE = E <= PL_SC_WIDE;
#if PL_SC_DIAG_SKIP_SPECIAL
    if constexpr (T == REP || T == SPC || T == R1) return from_packed<E>(signs<C, E>(a));  // diagnostic only
#endif
    if constexpr (T == R0) {
        return bzero<E>();
    } else if constexpr (T == REP) {
        float y[E];
#pragma unroll
        for (int j = 0; j < E; ++j) y[j] = a[j];
#pragma unroll
        for (int hh = E / 2; hh >= 1; hh >>= 1)
#pragma unroll
            for (int j = 0; j < hh; ++j) y[j] = y[j] + y[j + hh];
        const float v = grp_sumf<C::LOG_G>(y[0]);
        if constexpr (WIDE) {
            Wide<E> r;
            const uint32_t u = hd31(v);
#pragma unroll
            for (int j = 0; j < E; ++j) r.w[j] = u;
            return r;
        } else {
            return hd(v) ? ones<E>() : (BT)0;
        }
    } else if constexpr (T == R1 && C::FM == 0) {
        bool z = false;
#pragma unroll
        for (int j = 0; j < E; ++j) z |= (a[j] == 0.0f);
        if (!any_lane(z)) {
            if constexpr (WIDE) {
                Wide<E> r;
#pragma unroll
                for (int j = 0; j < E; ++j) r.w[j] = fu(a[j]);  // bit 31 = the decision
                return r;
            } else {
                return signs<C, E>(a);
            }
        }
        return split<C, s, P>(a, ln);
    } else if constexpr (T == SPC && C::FM == 0) {
        bool z = false;
#pragma unroll
        for (int j = 0; j < E; ++j) z |= ((fu(a[j]) & 0x7FFFFFFFu) == 0u);
        BT b = signs<C, E>(a);
        uint32_t par = (uint32_t)__popcll((unsigned long long)b) & 1u;
        par = grp<C::LOG_G>(par, [](uint32_t u, uint32_t v) { return u ^ v; });
        uint32_t mn = fu(a[0]) & 0x7FFFFFFFu;
#pragma unroll
        for (int j = 1; j < E; ++j) mn = min(mn, fu(a[j]) & 0x7FFFFFFFu);
        mn = grp<C::LOG_G>(mn, [](uint32_t u, uint32_t v) { return min(u, v); });
        BT eqm = 0;
#pragma unroll
        for (int j = 0; j < E; ++j) eqm |= (BT)((fu(a[j]) & 0x7FFFFFFFu) == mn) << j;
#if PL_SC_SPC_BALLOT
        // unique minimum: no lane holds two, and no codeword group has two lanes holding one
        const bool two = (eqm & (eqm - 1)) != 0;
        const bool bad_lane = z | ((par != 0u) & (two | (mn >= fu(ln.lmax))));
        const bool bad = any_lane(bad_lane) || multi_in_block<C::G>(ballot_lanes(eqm != 0), ballot_lanes(par != 0u));
#else
        uint32_t cnt = (uint32_t)__popcll((unsigned long long)eqm);
        cnt = grp<C::LOG_G>(cnt, [](uint32_t u, uint32_t v) { return u + v; });
        const bool bad = any_lane(z | ((par != 0u) & ((cnt != 1u) | (mn >= fu(ln.lmax)))));
#endif
        if (!bad) return from_packed<E>(par ? (BT)(b ^ eqm) : b);
        return split<C, s, P>(a, ln);
    } else {
        return split<C, s, P>(a, ln);
    }
}

// ---------------- root --------------------------------------------------------------------
// The root's input is the negated channel (polar_sc.py:122), held in VGPRs (NS slots).  The
// stage LOG_N-1 buffers are "virtual": each of their LLRs is recomputed from two channel values
// when a pass of the stage-(LOG_N-1) node reads it (f for the left half, g with the left half's
// partial sums for the right), so the largest stage buffer never occupies registers.
// Min-sum f(-x,-y) = f(x,y) bit for bit and g(-x,-y) = -g(x,y): the negation of polar_sc.py:122
// costs nothing (the sign of an exact zero is never observable: every decision treats +0 and -0
// alike).  The exact boxplus is only algebraically even -- log(1+e^(x+y)) - log(e^x+e^y) rounds
// differently from the same formula on -x, -y (dec.py:39-43 evaluates it on the negated channel,
// dec.py:147) -- so FM = 1 negates first (source modifiers, no extra instruction).
template <class C>
__device__ __forceinline__ float vfroot(float x, float y, float lmax) {
    if constexpr (C::FM == 0) return fop<0>(x, y, lmax);
    else return fop<C::FM>(-x, -y, lmax);
}
template <class C>
__device__ __forceinline__ float valpha(const float (&ch)[C::NS], int side, uint64_t blr, int j, float lmax) {
    const float x = ch[j], y = ch[j + C::NS / 2];
    return side == 0 ? vfroot<C>(x, y, lmax) : (-flip31(x, bit31(blr, j))) - y;
}

// all NS/2 virtual stage-(LOG_N-1) LLRs of one half
template <class C, int SIDE>
__device__ __forceinline__ void valphas(const float (&ch)[C::NS], uint64_t blr, float (&a)[C::NS / 2], float lmax) {
    constexpr int E = C::NS / 2;
    if constexpr (SIDE == 0 && C::FM == 1 && E >= 2 && PL_SC_FEX_PAIR) {
        // exact f on the negated channel (vfroot), two elements per call
#pragma unroll
        for (int j = 0; j < E; j += 2) {
            const plx::f2 r = plx::f_exact2(-ch[j], -ch[j + E], -ch[j + 1], -ch[j + 1 + E], lmax);
            a[j] = r.a;
            a[j + 1] = r.b;
        }
    } else if constexpr (SIDE == 1 && E >= 2) {
#pragma unroll
        for (int j = 0; j < E; j += 2) {
            const f2v u = {flip31(ch[j], bit31(blr, j)), flip31(ch[j + 1], bit31(blr, j + 1))};
            const f2v w = {ch[j + E], ch[j + 1 + E]};
            const f2v r = -u - w;
            a[j] = r.x;
            a[j + 1] = r.y;
        }
    } else {
#pragma unroll
        for (int j = 0; j < E; ++j) a[j] = valpha<C>(ch, SIDE, blr, j, lmax);
    }
}

struct NoHook {
    __device__ __forceinline__ void operator()() const {}
};

// `after` runs once the channel registers are dead (their last read is done): the pipelined
// decoder refills them with the next batch's channel there.
template <class C, int SIDE, class Hook = NoHook>
__device__ __forceinline__ Beta<C::NS / 2> half(float (&ch)[C::NS], uint64_t blr, const Lane& ln,
                                                const Hook& after = Hook()) {
    constexpr int s = C::LOG_N - 1, P = SIDE << s;
    constexpr int E = C::NS / 2;  // slots of the stage-(LOG_N-1) node per lane
    using BT = Beta<E>;
    constexpr int T = nt<C>(s, P);
    if constexpr (Ch<C>::CHL && T != R0) {
        // the upper channel slots, from LDS: live only while this half's virtual LLRs are formed
        // wait for the LDS-DMA (SIDE 1 too: a rate-0 left half reads nothing, and otherwise nothing
        // is outstanding); the memory clobber also keeps the compiler from merging SIDE 1's reads
        // with SIDE 0's, which would hold the values live across the whole left half
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = C::NS / 2; j < C::NS; ++j) ch[j] = ln.chl[(j - C::NS / 2) * 64];
    }
    if constexpr (T == R0) {
        after();
        return (BT)0;
    } else if constexpr (E == 1) {
        const float a = valpha<C>(ch, SIDE, blr, 0, ln.lmax);
        after();
        return (BT)(lnode<C, s, P>(a, ln) >> 31);
    } else if constexpr (T != GEN) {
        float a[E];
        valphas<C, SIDE>(ch, blr, a, ln.lmax);
        after();
        return packed(node<C, s, P>(a, ln));
    } else {
        constexpr int H = E / 2, h = 1 << (s - 1);
        using BH = BV<H>;
        float x[H];
        BH bl = bzero<H>();
        float va[E];
        valphas<C, SIDE>(ch, blr, va, ln.lmax);
        if constexpr (nt<C>(s - 1, P) != R0) {
            fvec<C::FM, SIDE == 0, H>(va, x, ln.lmax);
            bl = child<C, s, P>(x, ln);
#if PL_SC_VA_RECOMPUTE
            // recompute the virtual LLRs for the g pass instead of keeping them live across the
            // left subtree (32 VGPRs at n = 1024): the opaque copy keeps the compiler from reusing
            // the f-pass values
#pragma unroll
            for (int j = 0; j < C::NS; ++j) asm volatile("" : "+v"(ch[j]));
            valphas<C, SIDE>(ch, blr, va, ln.lmax);
#endif
        }
        gvec<H>(va, bl, x);
        after();
        const BH br = child<C, s, P + h>(x, ln);
        return packed(combine<H>(bl, br));
    }
}

// Per-lane constants of the mirror layout.  res(q): residue held by lane q of the group;
// lom[t]: lane holds the low element of its pair at level 2^t (in its canonical frame).
template <int LG>
__device__ __forceinline__ void lane_layout(int q, int& res, uint32_t (&lom)[5]) {
    int c = q;
    res = 0;
#pragma unroll
    for (int t = 4; t >= 1; --t) lom[t] = 0u;
#pragma unroll
    for (int t = LG; t >= 1; --t) {
        const int S = 1 << t;
        const bool lo = (c & (S / 2)) == 0;
        lom[t] = lo ? 0xFFFFFFFFu : 0u;
        if (!lo) {
            res += S / 2;
            c ^= (S - 1);
        }
    }
}


// u = x * G_n (G_n is an involution; the same transform encodes, x = u * G_n): in-lane spans on
// the packed slots, then the cross-lane spans with the mirror DPP (the low element of each pair
// takes the XOR).  w[0 .. WPL) = this lane's words (slot j = bit j % 32 of word j / 32).
template <class C>
__device__ __forceinline__ void butterfly(uint64_t lo, uint64_t hi, const Lane& ln, uint32_t (&w)[4]) {
    constexpr int NS = C::NS, LG = C::LOG_G, WPL = (NS + 31) / 32;
    constexpr uint64_t M[6] = {0x5555555555555555ull, 0x3333333333333333ull, 0x0f0f0f0f0f0f0f0full,
                               0x00ff00ff00ff00ffull, 0x0000ffff0000ffffull, 0x00000000ffffffffull};
#pragma unroll
    for (int t = 0; t < 6; ++t) {
        if ((1 << t) < NS) {
            lo ^= (lo >> (1 << t)) & M[t];
            hi ^= (hi >> (1 << t)) & M[t];
        }
    }
    if constexpr (NS > 64) lo ^= hi;
    w[0] = (uint32_t)lo;
    w[1] = (uint32_t)(lo >> 32);
    w[2] = (uint32_t)hi;
    w[3] = (uint32_t)(hi >> 32);
#pragma unroll
    for (int i = 0; i < WPL; ++i) {
        if constexpr (LG >= 4) w[i] ^= mir<16>(w[i]) & ln.lom(4);
        if constexpr (LG >= 3) w[i] ^= mir<8>(w[i]) & ln.lom(3);
        if constexpr (LG >= 2) w[i] ^= mir<4>(w[i]) & ln.lom(2);
        if constexpr (LG >= 1) w[i] ^= mir<2>(w[i]) & ln.lom(1);
    }
}

// The root's partial sums -> this lane's u words in its LDS slot.
template <class C>
__device__ __forceinline__ void to_u(uint64_t lo, uint64_t hi, const Lane& ln, uint32_t* __restrict__ mine) {
    constexpr int WPL = (C::NS + 31) / 32;
    uint32_t w[4];
    butterfly<C>(lo, hi, ln, w);
#pragma unroll
    for (int i = 0; i < WPL; ++i) mine[i] = w[i];
}

// Information bits of the wave's CW codewords (info_pos ascending, polar_sc.py:127) from its
// LDS u words to coalesced output rows.  info_loc[m] = (byte offset of the word holding info bit
// m in codeword 0's u area) << 5 | bit (jit.cpp attach_static): one v_bfe_u32 extracts the bit
// (its offset operand only reads bits 0-4), consecutive codewords are an immediate LDS offset
// apart, and the K of the code is a compile-time constant (loops unrolled).  `il` holds this
// lane's float4-path table entries when the caller preloaded them (PRE = true).
template <class C>
struct Emit {
    static constexpr int CW = 64 / C::G, WPL = (C::NS + 31) / 32, CWB = C::G * WPL * 4;
    static constexpr int KQ = C::K / 4, IT4 = (KQ + 63) / 64, IT1 = (C::K + 63) / 64;
    static constexpr bool PRE = PL_SC_EMIT_PRE && (C::K & 3) == 0 && IT4 <= 2;  // table entries kept in VGPRs
};

// bit (e & 31) of the u word at byte address wa + row_off
__device__ __forceinline__ float bitf(const unsigned char* wa, int e, int row_off) {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(wa + row_off);
    return (float)__builtin_amdgcn_ubfe(w, (uint32_t)e, 1u);
}

template <class C, int OUT>
__device__ __forceinline__ void emit(const uint32_t* __restrict__ ubase, int64_t cw0, int64_t bs, void* __restrict__ out,
                                     const int32_t* __restrict__ info_loc, const int4 (&il)[2], int lane) {
    using E = Emit<C>;
    constexpr int K = C::K, CW = E::CW, CWB = E::CWB;
    const unsigned char* ub = reinterpret_cast<const unsigned char*>(ubase);
    const bool full = cw0 + CW <= bs;  // wave-uniform
    if (OUT == OUT_F32 && (K & 3) == 0 && ((reinterpret_cast<uintptr_t>(out) & 15) == 0)) {
        // 16-byte stores: lane writes info bits 4c..4c+3 of a row (1 KiB per wave-instruction)
        float* o = static_cast<float*>(out) + cw0 * K;
        if constexpr (E::PRE) {
            // every table entry is consumed before the first store: waiting for the preloaded
            // entries then never waits for this wave's own output stores
            const unsigned char* a[2][4];
#pragma unroll
            for (int it = 0; it < E::IT4; ++it) {
                int off[4] = {il[it].x >> 5, il[it].y >> 5, il[it].z >> 5, il[it].w >> 5};
                // materialise now (the scheduler would sink the second iteration's offsets, and
                // their wait, behind the first iteration's stores)
                asm volatile("" : "+v"(off[0]), "+v"(off[1]), "+v"(off[2]), "+v"(off[3]));
#pragma unroll
                for (int i = 0; i < 4; ++i) a[it][i] = ub + off[i];
            }
#pragma unroll
            for (int it = 0; it < E::IT4; ++it) {
                const int c = lane + 64 * it;
                if (E::KQ % 64 == 0 || c < E::KQ) {
#pragma unroll
                    for (int g = 0; g < CW; ++g) {
                        if (full || cw0 + g < bs) {
                            float4 v;
                            v.x = bitf(a[it][0], il[it].x, g * CWB);
                            v.y = bitf(a[it][1], il[it].y, g * CWB);
                            v.z = bitf(a[it][2], il[it].z, g * CWB);
                            v.w = bitf(a[it][3], il[it].w, g * CWB);
                            st_out4(o + g * K + 4 * c, v);
                        }
                    }
                }
            }
        } else {
#pragma unroll
            for (int it = 0; it < E::IT4; ++it) {
                const int c = lane + 64 * it;
                if (E::KQ % 64 == 0 || c < E::KQ) {
                    const int4 l4 = reinterpret_cast<const int4*>(info_loc)[c];
#pragma unroll
                    for (int g = 0; g < CW; ++g) {
                        if (full || cw0 + g < bs) {
                            float4 v;
                            v.x = bitf(ub + (l4.x >> 5), l4.x, g * CWB);
                            v.y = bitf(ub + (l4.y >> 5), l4.y, g * CWB);
                            v.z = bitf(ub + (l4.z >> 5), l4.z, g * CWB);
                            v.w = bitf(ub + (l4.w >> 5), l4.w, g * CWB);
                            st_out4(o + g * K + 4 * c, v);
                        }
                    }
                }
            }
        }
    } else {
#pragma unroll
        for (int it = 0; it < E::IT1; ++it) {
            const int m = lane + 64 * it;
            if (K % 64 == 0 || m < K) {
                const int e = info_loc[m];
#pragma unroll
                for (int g = 0; g < CW; ++g) {
                    if (full || cw0 + g < bs) {
                        const float b = bitf(ub + (e >> 5), e, g * CWB);
                        if constexpr (OUT == OUT_F32) static_cast<float*>(out)[(cw0 + g) * K + m] = b;
                        else static_cast<uint8_t*>(out)[(cw0 + g) * K + m] = (uint8_t)b;
                    }
                }
            }
        }
    }
}

// OUT_CNT (the Monte-Carlo harness fused into the decoder, my_sn/sim.py:7-18 count_errors /
// count_block_errors): instead of writing the [bs, k] bit rows, compare the decoded information
// bits with the reference bits (packed, bit m of row r = bit m % 32 of ref[r * NQ + m / 32]) and
// store the wave's [bit errors, block errors] at part[2 * wave id] (int32; pl_sc_decode_count sums
// them).  Every wave of the grid stores its pair, rows past bs count nothing.
template <class C>
__device__ __forceinline__ void count_emit(const uint32_t* __restrict__ ubase, int64_t cw0, int64_t bs,
                                           const uint32_t* __restrict__ ref, int32_t* __restrict__ part,
                                           const int32_t* __restrict__ info_loc, int lane, int wid) {
    // Lane l takes information bits m = l + 64 it; a ballot over the wave packs bits 64 it .. 64 it
    // + 63 of a codeword into the same two words the reference row holds there, so the comparison
    // is a scalar XOR + popcount against a wave-uniform (scalar) load of those words.
    using E = Emit<C>;
    constexpr int K = C::K, CW = E::CW, CWB = E::CWB, NQ = (K + 31) / 32;
    const unsigned char* ub = reinterpret_cast<const unsigned char*>(ubase);
    uint32_t bits = 0, blocks = 0;
    int loc[E::IT1 > 0 ? E::IT1 : 1];
#pragma unroll
    for (int it = 0; it < E::IT1; ++it) {
        const int m = lane + 64 * it;
        loc[it] = (K % 64 == 0 || m < K) ? info_loc[m] : -1;
    }
#pragma unroll
    for (int g = 0; g < CW; ++g) {
        if (cw0 + g >= bs) break;  // wave-uniform
        const uint32_t* rrow = ref + (cw0 + g) * NQ;
        uint64_t diff = 0;
#pragma unroll
        for (int it = 0; it < E::IT1; ++it) {
            uint32_t b = 0;
            if (loc[it] >= 0) {
                const uint32_t w = *reinterpret_cast<const uint32_t*>(ub + (loc[it] >> 5) + g * CWB);
                b = __builtin_amdgcn_ubfe(w, (uint32_t)loc[it], 1u);
            }
            const uint64_t dec = __builtin_amdgcn_ballot_w64(b != 0u);
            const uint64_t want = (uint64_t)rrow[2 * it] | (2 * it + 1 < NQ ? (uint64_t)rrow[2 * it + 1] << 32 : 0ull);
            const uint64_t x = dec ^ want;
            bits += (uint32_t)__builtin_popcountll(x);
            diff |= x;
        }
        blocks += diff != 0 ? 1u : 0u;
    }
    if (lane == 0) {
        part[2 * wid] = (int32_t)bits;
        part[2 * wid + 1] = (int32_t)blocks;
    }
}

// ---------------- OUT_SIM: the Monte-Carlo producer fused in front of the decoder ----------
// One iteration of System_AWGN_model.forward (awgn_model.py:33-41: BinarySource, polar encoder,
// QPSK, AWGN, demapper) generated in the decoder's own lane layout, decoded, and compared with the
// information bits in registers (my_sn/sim.py:7-18): no LLR or bit row touches HBM.  Codes with
// 64 slots per lane (C::NS == 64); the lane holding residue r of a codeword holds positions
// r + G j, j < 64.  Random streams (Philox4x32-10, key = seed, counter (row, row >> 32,
// iteration, word 3)), distinct from pl_awgn_qpsk_llr's by bit 30 of word 3:
//   information bits  word 3 = 0x40000000 | r >> 1: position r + G j (if not frozen) = bit j % 32
//                     of component 2 (r & 1) + j / 32 (even residues x, y; odd z, w);
//   noise             word 3 = 0xC0000000 | (16 r + t): slots 4t .. 4t+3 of residue r, the same
//                     Box-Muller and logit map as channel_kernel.hip logits4.
struct SimArgs {
    int64_t row0;  // stream row of the launch's codeword 0
    uint32_t k0, k1, it;
    float no;
    float* llr_dump;  // nullable: [bs, N] fp32 logits as generated (tests)
    float* u_dump;    // nullable: [bs, K] fp32 information bits as generated (tests)
};

struct U4s {
    uint32_t x, y, z, w;
};

// Random123 philox4x32_R(10, ...), as channel_kernel.hip philox
__device__ __forceinline__ U4s philox10(U4s c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        c = U4s{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// channel_kernel.hip logits4: four logits from one Philox block and four code bits (bits 0..3);
// la = scale / sqrt(2), rsc = scale * sqrt(no / 2) * sqrt(2 ln 2), scale = -2 sqrt(2) / no
__device__ __forceinline__ void logits4(const U4s& rnd, uint32_t bits, float la, float rsc, float (&l)[4]) {
    const float rs0 = rsc * __builtin_amdgcn_sqrtf(32.0f - __builtin_amdgcn_logf((float)(rnd.x | 1u)));
    const float rs1 = rsc * __builtin_amdgcn_sqrtf(32.0f - __builtin_amdgcn_logf((float)(rnd.z | 1u)));
    const float t0 = uf(0x3F800000u | (rnd.y >> 9)), t1 = uf(0x3F800000u | (rnd.w >> 9));
    const uint32_t au = fu(la);
    l[0] = __builtin_fmaf(rs0, __builtin_amdgcn_cosf(t0), uf(au ^ ((bits << 31) & 0x80000000u)));
    l[1] = __builtin_fmaf(rs0, __builtin_amdgcn_sinf(t0), uf(au ^ ((bits << 30) & 0x80000000u)));
    l[2] = __builtin_fmaf(rs1, __builtin_amdgcn_cosf(t1), uf(au ^ ((bits << 29) & 0x80000000u)));
    l[3] = __builtin_fmaf(rs1, __builtin_amdgcn_sinf(t1), uf(au ^ ((bits << 28) & 0x80000000u)));
}

// information mask of residue `res` (bit j = position res + G j is not frozen), from the code's
// compile-time table
template <class C, int R = 0>
__device__ __forceinline__ uint64_t info_lane(int res) {
    if constexpr (R == C::G) {
        return 0;
    } else {
        constexpr uint64_t m = C::INFO_LANE[R];
        return res == R ? m : info_lane<C, R + 1>(res);
    }
}

// The channel slots of this lane (slots >= NS/2 into its LDS rows when Ch<C>::CHL) and its
// information bits g (slot words), generated as described above.
template <class C>
__device__ __forceinline__ void gen_channel(float (&chv)[C::NS], const Lane& ln, float* chl_lane, const SimArgs& sa,
                                            int64_t cw0, int64_t bs, int lane, int res, uint32_t (&g)[2]) {
    static_assert(C::NS == 64, "OUT_SIM: 64 slots per lane");
    constexpr int G = C::G;
    const int64_t cw = cw0 + (lane >> C::LOG_G);
    const uint64_t row = (uint64_t)(sa.row0 + cw);
    const uint32_t rlo = (uint32_t)row, rhi = (uint32_t)(row >> 32);
    const uint64_t info = info_lane<C>(res);
    const U4s b = philox10(U4s{rlo, rhi, sa.it, 0x40000000u | (uint32_t)(res >> 1)}, sa.k0, sa.k1);
    g[0] = ((res & 1) ? b.z : b.x) & (uint32_t)info;
    g[1] = ((res & 1) ? b.w : b.y) & (uint32_t)(info >> 32);
    uint32_t x[4];
    butterfly<C>((uint64_t)g[0] | ((uint64_t)g[1] << 32), 0, ln, x);  // code bits x = u G_n
    const float scale = -2.8284271f / sa.no;
    const float la = scale * 0.70710677f, rsc = scale * __builtin_sqrtf(sa.no) * (0.70710677f * 1.17741002f);
    const bool dump = sa.llr_dump != nullptr && cw < bs;
    float* drow = dump ? sa.llr_dump + cw * C::N + res : nullptr;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const U4s rnd = philox10(U4s{rlo, rhi, sa.it, 0xC0000000u | (uint32_t)(res * 16 + t)}, sa.k0, sa.k1);
        float l[4];
        logits4(rnd, x[t >> 3] >> ((t & 7) * 4), la, rsc, l);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = 4 * t + i;
            if (Ch<C>::CHL && j >= C::NS / 2) chl_lane[(j - C::NS / 2) * 64] = l[i];
            else chv[j] = l[i];
        }
        if (dump) {
#pragma unroll
            for (int i = 0; i < 4; ++i) drow[(4 * t + i) * G] = l[i];
        }
    }
}

// [bit errors, block errors] of the wave's codewords: decoded u words (from the root's partial
// sums) against the generated ones; lane 0 stores the pair at part[2 * wid].
template <class C>
__device__ __forceinline__ void sim_count(uint64_t lo, uint64_t hi, const Lane& ln, const uint32_t (&g)[2], int64_t cw0,
                                          int64_t bs, int lane, int32_t* __restrict__ part, int wid) {
    constexpr int G = C::G, CW = 64 / G;
    uint32_t w[4];
    butterfly<C>(lo, hi, ln, w);
    const bool live = cw0 + (lane >> C::LOG_G) < bs;
    uint32_t e = live ? (uint32_t)(__builtin_popcount(w[0] ^ g[0]) + __builtin_popcount(w[1] ^ g[1])) : 0u;
    const uint64_t bad = __builtin_amdgcn_ballot_w64(e != 0u);
    uint32_t blocks = 0;
    if constexpr (G == 1) {
        blocks = (uint32_t)__builtin_popcountll(bad);
    } else {
#pragma unroll
        for (int c = 0; c < CW; ++c) blocks += ((bad >> (c * G)) & ((1ull << G) - 1ull)) != 0 ? 1u : 0u;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) e += (uint32_t)__shfl_xor((int)e, off, 64);
    if (lane == 0) {
        part[2 * wid] = (int32_t)e;
        part[2 * wid + 1] = (int32_t)blocks;
    }
}

// this lane's float4-path table entries, loaded early (their latency hides behind the channel)
template <class C>
__device__ __forceinline__ void preload_info(const int32_t* __restrict__ info_loc, int4 (&il)[2], int lane) {
    using E = Emit<C>;
    il[0] = il[1] = int4{0, 0, 0, 0};
    if constexpr (E::PRE) {
#pragma unroll
        for (int it = 0; it < E::IT4; ++it) {
            const int c = lane + 64 * it;
            if (E::KQ % 64 == 0 || c < E::KQ) il[it] = reinterpret_cast<const int4*>(info_loc)[c];
        }
    }
}

// LDS hand-off between the lanes of ONE wave (each wave owns its LDS slots): LDS executes a
// wave's accesses in order, so only the compiler has to be kept from reordering them.
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

template <class C>
__device__ __forceinline__ void load_channel(float (&chv)[C::NS], const float* __restrict__ llr, int64_t cw0,
                                             int64_t bs, int lane, int res, float* chl_wave = nullptr) {
    const int64_t cw = cw0 + (lane >> C::LOG_G);
    const float* ch = llr + (size_t)(cw < bs ? cw : bs - 1) * C::N;
    if constexpr (Ch<C>::CHL) {
        // slots [0, NS/2) into VGPRs; slots [NS/2, NS) by LDS-DMA, one 256-byte LDS row per slot
        // (lane l's word at l * 4), so no VGPR holds them while the left half is decoded
#pragma unroll
        for (int j = 0; j < C::NS / 2; ++j) chv[j] = ld_ch(ch + j * C::G + res);
#if PL_SC_DMA_ASM
        // saddr form: wave-uniform row base in an SGPR pair (slot offset j * 64 B as the 12-bit
        // immediate would also move the LDS address, so the base steps in SALU), this lane's
        // 32-bit byte offset in a VGPR; M0 = the slot's LDS row.  No VALU per instruction.  The
        // compiler does not track these loads: the reader waits with s_waitcnt vmcnt(0) (half()).
        // base row: the wave's lowest (clamped) row, so every lane's offset is >= 0 and < 16 KiB
        const int64_t row0 = cw0 < bs ? cw0 : bs - 1;
        const uint32_t voff = (uint32_t)(((ch - llr) - row0 * C::N + res) * 4);
        const uint64_t sbase = (uint64_t)(uintptr_t)(llr + row0 * C::N);
        const uint32_t lbase = (uint32_t)(uintptr_t)chl_wave;  // LDS offset (low word of the flat address)
#pragma unroll
        for (int j = C::NS / 2; j < C::NS; ++j) {
            const uint64_t a = sbase + (uint64_t)(j * C::G * 4);
            const uint64_t sb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a) |
                                ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32);
            const uint32_t lb = (uint32_t)__builtin_amdgcn_readfirstlane((int)(lbase + (j - C::NS / 2) * 256));
#if PL_SC_NT & 1
            asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dword %0, %1 nt" ::"v"(voff), "s"(sb), "s"(lb) : "memory", "m0");
#else
            asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dword %0, %1" ::"v"(voff), "s"(sb), "s"(lb) : "memory", "m0");
#endif
        }
#else
#pragma unroll
        for (int j = C::NS / 2; j < C::NS; ++j)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(ch + j * C::G + res),
                                             (__attribute__((address_space(3))) void*)(chl_wave + (j - C::NS / 2) * 64),
                                             4, 0, (PL_SC_NT & 1) ? 2 : 0);
#endif
    } else {
#pragma unroll
        for (int j = 0; j < C::NS; ++j) chv[j] = ld_ch(ch + j * C::G + res);
    }
}

// Hook for half<1>: reload the channel registers with the next batch once they are dead.
template <class C>
struct Refill {
    float (&chv)[C::NS];
    const float* __restrict__ llr;
    int64_t ncw0, bs;
    int lane, res;
    __device__ __forceinline__ void operator()() const {
        // keep the scheduler from hoisting the refill above the last reads of the old values;
        // unconditional (past the end every lane re-reads row bs-1, a cache hit) so the old
        // values are dead here on every path
        __builtin_amdgcn_sched_barrier(0);
        load_channel<C>(chv, llr, ncw0, bs, lane, res);
        __builtin_amdgcn_sched_barrier(0);
    }
};

template <class C, class Hook>
__device__ __forceinline__ void root_virtual(float (&chv)[C::NS], const Lane& ln, uint64_t& lo, uint64_t& hi,
                                             const Hook& after) {
    constexpr int NS = C::NS;
    using BH = Beta<NS / 2>;
    const BH bl = half<C, 0>(chv, 0, ln);
    const BH br = half<C, 1>(chv, (uint64_t)bl, ln, after);
    if constexpr (NS / 2 >= 64) {
        lo = (uint64_t)(bl ^ br);
        hi = (uint64_t)br;
    } else {
        lo = (uint64_t)(bl ^ br) | ((uint64_t)br << (NS / 2));
        hi = 0;
    }
}

template <class C, int OUT>
__device__ __forceinline__ void decode(const float* __restrict__ llr, int64_t bs, void* __restrict__ out,
                                       const int32_t* __restrict__ info_loc, int k, float lmax,
                                       uint32_t* __restrict__ ulds, const uint32_t* __restrict__ ref = nullptr,
                                       const SimArgs* sa = nullptr) {
    static_assert(OUT < OUT_CNT || (!PL_SC_PERSIST && !PL_SC_STAMPS && (PL_SC_ROOT_MODE == 0 || OUT == OUT_CNT)),
                  "OUT_CNT / OUT_SIM: plain decoder only (OUT_CNT also with the stage-(n/2) root of PL_SC_ROOT_MODE 1)");
    constexpr int N = C::N, G = C::G, LG = C::LOG_G, NS = C::NS, CW = 64 / G;
    constexpr int WPL = (NS + 31) / 32;
    // the wave index is wave-uniform: as an SGPR value all batch/row address math is scalar
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane & (G - 1);
    Lane ln;
    int res;
#if PL_SC_LANE31
    {
        uint32_t lom[5];
        lane_layout<LG>(q, res, lom);
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            ln.lo31[t] = t ? lom[t] & 0x80000000u : 0u;
            // keep them VGPR values: a mask the compiler knows to be 0/~0 per lane becomes an
            // SGPR lane mask and each combine a v_cndmask + v_xor instead of one v_bitop3
            asm volatile("" : "+v"(ln.lo31[t]));
        }
    }
#else
    lane_layout<LG>(q, res, ln.lom_);
    ln.lom_[0] = 0u;
#endif
    ln.lmax = lmax;
    if constexpr (C::FM == 1) plx::load_tables(threadIdx.x, blockDim.x);  // the exact f's exp / log tables
    // PL_SC_CH_LDS: each wave's LDS is its channel rows; its u words reuse their first 64 * WPL
    // words once the right half has read them (same wave, LDS in order)
    constexpr int WLDS = Ch<C>::CHL ? (NS / 2) * 64 : 64 * WPL;  // LDS words per wave
    uint32_t* ubase = ulds + wave * WLDS;
    uint32_t* mine = ubase + lane * WPL;
    float* chl_wave = reinterpret_cast<float*>(ulds + wave * WLDS);
    ln.chl = chl_wave + lane;
    static_assert(!Ch<C>::CHL || (!PL_SC_PERSIST && PL_SC_ROOT_MODE == 0 && NS / 2 >= WPL), "PL_SC_CH_LDS: plain decoder only");

#if PL_SC_PERSIST
    // Persistent, software-pipelined: each wave walks batches of CW codewords with a stride of
    // the whole grid; the next batch's channel is loaded into the channel registers as soon as
    // their last read is done (3/4 through the tree), so its HBM latency overlaps the rest of
    // the tree and the output of this batch instead of stalling every wave at the same instant.
    const int64_t stride = (int64_t)gridDim.x * kWaves * CW;
    int64_t cw0 = ((int64_t)blockIdx.x * kWaves + wave) * CW;
    int4 il[2];
    preload_info<C>(info_loc, il, lane);
    float chv[NS];
    load_channel<C>(chv, llr, cw0, bs, lane, res);
    for (; cw0 < bs; cw0 += stride) {
        const int64_t ncw0 = cw0 + stride;
        uint64_t lo, hi;
        root_virtual<C>(chv, ln, lo, hi, Refill<C>{chv, llr, ncw0, bs, lane, res});
        to_u<C>(lo, hi, ln, mine);
        wave_lds_fence();
        emit<C, OUT>(ubase, cw0, bs, out, info_loc, il, lane);
        wave_lds_fence();
    }
#else
    const int64_t cw0 = ((int64_t)blockIdx.x * kWaves + wave) * CW;
#if PL_SC_STAMPS
    // diagnostic build: per-wave clock stamps into the output's tail (tools/static_probe.py)
    uint64_t st0 = __builtin_amdgcn_s_memtime();
    uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    uint64_t lo = 0, hi = 0;
    int4 il[2];
    if constexpr (OUT != OUT_SIM) preload_info<C>(info_loc, il, lane);
#if PL_SC_ROOT_MODE == 0
    float chv[NS];
    uint32_t gsim[2] = {0u, 0u};  // OUT_SIM: the generated information bits (slot words)
#if PL_SC_DIAG_NO_LOAD  // diagnostic only (wrong results): the tree without the channel loads
#pragma unroll
    for (int j = 0; j < NS; ++j) chv[j] = (float)((lane * 7 + j * 13) % 61) - 30.5f;
    asm volatile("" ::"v"(llr));
#else
    if constexpr (OUT == OUT_SIM) gen_channel<C>(chv, ln, chl_wave + lane, *sa, cw0, bs, lane, res, gsim);
    else load_channel<C>(chv, llr, cw0, bs, lane, res, chl_wave);
#endif
#if PL_SC_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
    for (int j = 0; j < NS; ++j) asm volatile("" : "+v"(chv[j]));
    uint64_t st1 = __builtin_amdgcn_s_memtime();
#endif
#if PL_SC_DIAG_NO_TREE  // diagnostic only (wrong results): loads and output without the tree
    {
        uint32_t acc = 0;
#pragma unroll
        for (int j = 0; j < NS; ++j) acc ^= fu(chv[j]) << (j & 31);
        lo = acc;
        hi = acc >> 1;
    }
#else
    root_virtual<C>(chv, ln, lo, hi, NoHook());
#endif
    if constexpr (OUT == OUT_SIM) {
        sim_count<C>(lo, hi, ln, gsim, cw0, bs, lane, static_cast<int32_t*>(out), blockIdx.x * kWaves + wave);
        if (sa->u_dump != nullptr) {  // tests: the generated bits as fp32 rows, through the emit path
            wave_lds_fence();
            mine[0] = gsim[0];
            mine[1] = gsim[1];
            wave_lds_fence();
            preload_info<C>(info_loc, il, lane);
            emit<C, OUT_F32>(ubase, cw0, bs, sa->u_dump, info_loc, il, lane);
        }
        return;
    }
#else
    // Stage LOG_N-1 held in VGPRs; the channel is read once per half (the second read is
    // served by the caches) and is never live across a half's subtree.
#if PL_SC_STAMPS
    uint64_t st1 = st0;
#endif
    {
        const int64_t cw = cw0 + (lane >> LG);
        const float* ch = llr + (size_t)(cw < bs ? cw : bs - 1) * N;
        using BH = Beta<NS / 2>;
        constexpr int E = NS / 2;
        BH bl = 0, br = 0;
        if constexpr (nt<C>(C::LOG_N - 1, 0) != R0) {
            float a[E];
#pragma unroll
            for (int j = 0; j < E; ++j) a[j] = vfroot<C>(ch[j * G + res], ch[(j + E) * G + res], lmax);
            if constexpr (E == 1) bl = lnode<C, C::LOG_N - 1, 0>(a[0], ln) >> 31;
            else bl = packed(node<C, C::LOG_N - 1, 0>(a, ln));
        }
        {
            const float* chp = ch;
            asm volatile("" : "+v"(chp) : "v"(bl));
            float a[E];
#pragma unroll
            for (int j = 0; j < E; ++j)
                a[j] = (-flip31(chp[j * G + res], bit31(bl, j))) - chp[(j + E) * G + res];
            if constexpr (E == 1) br = lnode<C, C::LOG_N - 1, N / 2>(a[0], ln) >> 31;
            else br = packed(node<C, C::LOG_N - 1, N / 2>(a, ln));
        }
        if constexpr (NS / 2 >= 64) {
            lo = (uint64_t)(bl ^ br);
            hi = (uint64_t)br;
        } else {
            lo = (uint64_t)(bl ^ br) | ((uint64_t)br << (NS / 2));
        }
    }
#endif
    to_u<C>(lo, hi, ln, mine);
#if PL_SC_STAMPS
    uint64_t st2 = __builtin_amdgcn_s_memtime();
#endif
    wave_lds_fence();
#if PL_SC_STAMPS
    uint64_t st3 = __builtin_amdgcn_s_memtime();
#endif
    if constexpr (OUT == OUT_CNT)
        count_emit<C>(ubase, cw0, bs, ref, static_cast<int32_t*>(out), info_loc, lane, blockIdx.x * kWaves + wave);
    else
        emit<C, OUT>(ubase, cw0, bs, out, info_loc, il, lane);
#if PL_SC_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
    uint64_t st4 = __builtin_amdgcn_s_memtime();
    uint64_t rt = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        uint64_t* d = reinterpret_cast<uint64_t*>(static_cast<float*>(out) + bs * k) + (blockIdx.x * kWaves + wave) * 8;
        d[0] = st0; d[1] = st1; d[2] = st2; d[3] = st3; d[4] = st4;
        d[5] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_REG_HW_ID
        d[6] = rt0;
        d[7] = rt;
    }
#endif
#endif
}


#if PL_SC_PERSIST == 2
// LDS layout of the staged kernel (one __shared__ array: a second LDS object can make the
// compiler drain the copies early): [kWaves][64 lanes][WPL] u words, then per wave CW channel
// rows of N floats + a 16-float pad (rows r and r + 1 start in opposite halves of the 32 banks,
// so the ds_read_b32 of the residue layout is conflict-free).
template <class C>
struct Staged {
    static constexpr int CW = 64 / C::G, WPL = (C::NS + 31) / 32, ROW = C::N + 16;
    static constexpr int U_WORDS = kWaves * 64 * WPL;
    static constexpr int WORDS = U_WORDS + kWaves * CW * ROW;
    static constexpr int COPIES = CW * (C::N / 256);  // 1-KiB copies per batch
    static constexpr int KQ = C::K / 4;               // float4 output chunks per row
    static constexpr int IT4 = (KQ + 63) / 64, IT1 = (C::K + 63) / 64;
    // store instructions one batch's emit issues after the next batch's copies (full batches):
    // the counted wait before reading the staging buffer leaves exactly these outstanding
    static constexpr int ST_VEC = IT4 * CW, ST_SCALAR = IT1 * CW;
};

template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0, "");
    if constexpr (N >= 63) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Rows cw0 .. cw0+CW-1 (clamped to bs-1) into the wave's staging rows, 1 KiB per instruction.
template <class C>
__device__ __forceinline__ void stage_copy(const float* __restrict__ llr, int64_t cw0, int64_t bs, float* rows,
                                           int lane) {
    using S = Staged<C>;
#pragma unroll
    for (int r = 0; r < S::CW; ++r) {
        const int64_t cw = cw0 + r < bs ? cw0 + r : bs - 1;
        const float* src = llr + (size_t)cw * C::N + lane * 4;
#pragma unroll
        for (int i = 0; i < C::N / 256; ++i)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + i * 256),
                                             (__attribute__((address_space(3))) void*)(rows + r * S::ROW + i * 256),
                                             16, 0, 0);
    }
}

template <class C, int OUT>
__device__ __forceinline__ void decode_staged(const float* __restrict__ llr, int64_t bs, void* __restrict__ out,
                                              const int32_t* __restrict__ info_loc, int k, float lmax,
                                              uint32_t* __restrict__ lds) {
    using S = Staged<C>;
    constexpr int G = C::G, LG = C::LOG_G, NS = C::NS, CW = S::CW, WPL = S::WPL;
    static_assert(C::N >= 256 && C::N % 256 == 0, "staged channel rows are whole 1-KiB copies");
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane & (G - 1);
    Lane ln;
    int res;
#if PL_SC_LANE31
    {
        uint32_t lom[5];
        lane_layout<LG>(q, res, lom);
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            ln.lo31[t] = t ? lom[t] & 0x80000000u : 0u;
            asm volatile("" : "+v"(ln.lo31[t]));
        }
    }
#else
    lane_layout<LG>(q, res, ln.lom_);
    ln.lom_[0] = 0u;
#endif
    ln.lmax = lmax;
    // exact f would add the tables' LDS object next to the single Staged array (see above: the
    // compiler may then drain the copies early); the staged kernel is a rejected min-sum A/B
    static_assert(C::FM == 0, "PL_SC_PERSIST == 2 (staged kernel): min-sum codes only");
    uint32_t* ubase = lds + wave * 64 * WPL;
    uint32_t* mine = lds + (wave * 64 + lane) * WPL;
    float* rows = reinterpret_cast<float*>(lds + S::U_WORDS) + wave * CW * S::ROW;
    const float* myrow = rows + (lane >> LG) * S::ROW + res;
    const bool vec = OUT == OUT_F32 && (C::K & 3) == 0 && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);

    const int64_t stride = (int64_t)gridDim.x * kWaves * CW;
    int64_t cw0 = ((int64_t)blockIdx.x * kWaves + wave) * CW;
    if (cw0 >= bs) return;  // wave-uniform; no block-wide barrier below
    int4 il[2];
    preload_info<C>(info_loc, il, lane);
    stage_copy<C>(llr, cw0, bs, rows, lane);
    wait_vm<0>();
    for (;;) {
        float chv[NS];
#pragma unroll
        for (int j = 0; j < NS; ++j) chv[j] = myrow[j * G];
        // the reads must have returned before the next copy overwrites the rows
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int64_t ncw0 = cw0 + stride;
        const bool more = ncw0 < bs;
        if (more) stage_copy<C>(llr, ncw0, bs, rows, lane);
        uint64_t lo = 0, hi = 0;
        root_virtual<C>(chv, ln, lo, hi, NoHook());
        to_u<C>(lo, hi, ln, mine);
        wave_lds_fence();
        emit<C, OUT>(ubase, cw0, bs, out, info_loc, il, lane);
        wave_lds_fence();
        if (!more) break;
        // this batch was full (a partial batch is the last one): its emit issued exactly
        // ST_VEC / ST_SCALAR stores after the copies
        if (vec) wait_vm<S::ST_VEC>();
        else wait_vm<S::ST_SCALAR>();
        cw0 = ncw0;
    }
    (void)k;
}
#endif

}  // namespace pls

// Entry points instantiated per code: the including translation unit defines PlCode first.
#if PL_SC_PERSIST == 2
#define PL_SC_ENTRY(CODE, NAME, OUTK)                                                                        \
    extern "C" __global__ __launch_bounds__(64 * pls::kWaves, 2) void NAME(                                  \
        const float* __restrict__ llr, int64_t bs, void* __restrict__ out, const int32_t* __restrict__ info_loc, \
        int k, float lmax) {                                                                                  \
        __shared__ uint32_t lds[pls::Staged<CODE>::WORDS];                                                   \
        pls::decode_staged<CODE, OUTK>(llr, bs, out, info_loc, k, lmax, lds);                                \
    }
#else
#define PL_SC_ENTRY(CODE, NAME, OUTK)                                                                        \
    extern "C" __global__ __launch_bounds__(64 * pls::kWaves, PL_SC_MINW) void NAME(                         \
        const float* __restrict__ llr, int64_t bs, void* __restrict__ out, const int32_t* __restrict__ info_loc, \
        int k, float lmax) {                                                                                  \
        __shared__ uint32_t ulds[pls::Ch<CODE>::CHL ? pls::kWaves * 64 * (CODE::NS / 2)                       \
                                                    : pls::kWaves * 64 * ((CODE::NS + 31) / 32)];              \
        pls::decode<CODE, OUTK>(llr, bs, out, info_loc, k, lmax, ulds);                                      \
    }
#endif
#ifndef PL_SC_PERSIST_BPC
#define PL_SC_PERSIST_BPC 2  // resident blocks per CU the launcher gives a persistent kernel
#endif
// decode + error count against packed reference bits (pl_sc_decode_count); plain decoder only
#if PL_SC_PERSIST || PL_SC_STAMPS
#define PL_SC_CNT_ENTRY(CODE)
#else
#define PL_SC_CNT_ENTRY(CODE)                                                                                \
    extern "C" __global__ __launch_bounds__(64 * pls::kWaves, PL_SC_MINW) void pl_sc_static_cnt(             \
        const float* __restrict__ llr, int64_t bs, int32_t* __restrict__ part, const int32_t* __restrict__ info_loc, \
        int k, float lmax, const uint32_t* __restrict__ ref) {                                               \
        __shared__ uint32_t ulds[pls::Ch<CODE>::CHL ? pls::kWaves * 64 * (CODE::NS / 2)                       \
                                                    : pls::kWaves * 64 * ((CODE::NS + 31) / 32)];              \
        pls::decode<CODE, pls::OUT_CNT>(llr, bs, part, info_loc, k, lmax, ulds, ref);                        \
    }
#endif
// producer + decode + error count (pl_sc_sim_count); codes with 64 slots per lane (jit.cpp
// defines PL_SC_SIM for those and emits the code's INFO_LANE table)
#ifndef PL_SC_SIM
#define PL_SC_SIM 0
#endif
#if !PL_SC_SIM || PL_SC_PERSIST || PL_SC_STAMPS || PL_SC_ROOT_MODE
#define PL_SC_SIM_ENTRY(CODE)
#else
#define PL_SC_SIM_ENTRY(CODE)                                                                                \
    extern "C" __global__ __launch_bounds__(64 * pls::kWaves, PL_SC_MINW) void pl_sc_static_sim(             \
        int64_t bs, int64_t row0, uint32_t k0, uint32_t k1, uint32_t it, float no, int32_t* __restrict__ part, \
        const int32_t* __restrict__ info_loc, int k, float lmax, float* __restrict__ llr_dump,               \
        float* __restrict__ u_dump) {                                                                         \
        __shared__ uint32_t ulds[pls::Ch<CODE>::CHL ? pls::kWaves * 64 * (CODE::NS / 2)                       \
                                                    : pls::kWaves * 64 * ((CODE::NS + 31) / 32)];              \
        const pls::SimArgs sa{row0, k0, k1, it, no, llr_dump, u_dump};                                       \
        pls::decode<CODE, pls::OUT_SIM>(nullptr, bs, part, info_loc, k, lmax, ulds, nullptr, &sa);           \
    }
#endif
#define PL_SC_STATIC_KERNELS(CODE)                                                                           \
    extern "C" __device__ const int pl_sc_persistent = PL_SC_PERSIST;                                       \
    extern "C" __device__ const int pl_sc_blocks_per_cu = PL_SC_PERSIST_BPC;                                \
    extern "C" __device__ const int pl_sc_waves = PL_SC_KWAVES;                                            \
    PL_SC_ENTRY(CODE, pl_sc_static_f32, pls::OUT_F32)                                                        \
    PL_SC_ENTRY(CODE, pl_sc_static_u8, pls::OUT_U8)                                                          \
    PL_SC_CNT_ENTRY(CODE)                                                                                    \
    PL_SC_SIM_ENTRY(CODE)

#endif  // PL_SC_STATIC_H
