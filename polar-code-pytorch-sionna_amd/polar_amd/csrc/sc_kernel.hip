// sc_kernel.hip -- successive-cancellation (SC) polar decoder for gfx950 (MI355X).
//
// Reference semantics: x_run_sn_polar/polar/polar_sc.py (SC_Dec, min-sum f forced at :46,
// g :49-53, leaf rule :90-98, partial sums :83-89) and, for f_mode=PL_F_EXACT, the exact boxplus
// of my_sn/fec/polar/dec.py:33-46.  Min-sum results are bit-identical to the reference.
//
// Design ("register tree"): a wave64 decodes C = 64/G codewords at once, G lanes per codeword.
// Element i of a stage buffer lives in lane (i mod G) of its codeword's lane group, slot i/G, so
// every f/g of a node of size >= 2G pairs elements that sit in the SAME lane: the upper stages
// run entirely in VGPRs with no LDS and no cross-lane traffic.  G = max(1, n/128) keeps the
// deepest live set of stage buffers near 128 VGPRs.  Partial sums (beta) are bit-packed per lane.
// The tree walk is generated at compile time (templates on the stage); above a small depth each
// node runs its two children in a runtime 2-trip loop, so code size stays O(n/G).
//
// Exact node shortcuts (what the reference's recursion would compute, derived, not approximated):
//   rate-0 (all frozen)        beta = 0                                   (polar_sc.py:92)
//   repetition (only last info) u = HD(pairwise tree sum of the node LLRs in SC's g order), beta = u
//   rate-1 (all info)          beta = HD(alpha)            if no node LLR is exactly 0
//   SPC (only first frozen)    beta = HD(alpha), parity fixed at the unique min |alpha| < llr_max,
//                                                          if no LLR is 0 and that min is unique
// HD(x) = 1 iff !(x > 0) (polar_sc.py:94-97).  The rate-1 / SPC proofs hold for min-sum only
// (signs of f are exact there), so those two shortcuts are compiled only for f_mode = min-sum;
// when their preconditions fail for any codeword of the wave (exact zeros, ties, saturation) the
// wave runs the full recursion for that node.  Decided bits are never tracked per leaf: the
// root's partial sums are the re-encoded codeword x = u*G_n, and u = x*G_n (G_n is an
// involution), one butterfly at the end.  A node of size G that has no shortcut gathers its G
// LLRs into every lane of the group (ds_bpermute) and is decoded redundantly in-lane.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../../include/polar_mi355x.h"
#include "exactf.h"
#include "plan.h"

namespace {

#ifndef PL_SC_SHORTCUTS
#define PL_SC_SHORTCUTS 13  // bit 0 rep, bit 1 rate-1, bit 2 SPC, bit 3 skip-f of rate-0 left children
#endif
constexpr int kShortcuts = PL_SC_SHORTCUTS;
#ifndef PL_SC_MIN_WAVES
#define PL_SC_MIN_WAVES 2  // waves per SIMD the register allocation must allow (occupancy target)
#endif
#ifndef PL_SC_SHORTCUT_MAX_E
#define PL_SC_SHORTCUT_MAX_E 8  // shortcuts only on nodes with <= this many elements per lane
#endif
#ifndef PL_SC_ROOT_STORED
#define PL_SC_ROOT_STORED 0  // 1: hold stage n/2 in VGPRs; 0: recompute it from the channel
#endif
#ifndef PL_SC_CH_REGS
#define PL_SC_CH_REGS 0  // 1: load this lane's n/G channel values into VGPRs once at the root
#endif
#ifndef PL_SC_LAUNDER_CH
#define PL_SC_LAUNDER_CH 0  // 1: re-load the channel from L2 per pass instead of holding it in VGPRs
#endif
#ifndef PL_SC_DPP_GATHER
#define PL_SC_DPP_GATHER 1  // gather a G-node's LLRs with DPP (VALU) instead of ds_bpermute
#endif
#ifndef PL_SC_LAUNDER_BL
#define PL_SC_LAUNDER_BL 0
#endif
#ifndef PL_SC_ROOT_CHUNK
#define PL_SC_ROOT_CHUNK 8  // root f/g outputs per scheduling chunk (bounds loads in flight)
#endif
constexpr int kWavesPerBlock = 4;
#ifndef PL_SC_DIAG_SAMEROW
#define PL_SC_DIAG_SAMEROW 0  // diagnostic builds only (tools/variants.py)
#endif
#ifndef PL_SC_DIAG_NOSTORE
#define PL_SC_DIAG_NOSTORE 0
#endif
#if !PL_DEV && (PL_SC_DIAG_SAMEROW || PL_SC_DIAG_NOSTORE)
#error "PL_SC_DIAG_* macros give wrong results: development builds (-DPL_DEV=1) only"
#endif
#ifndef PL_SC_LOOP_DEPTH
#define PL_SC_LOOP_DEPTH 3  // nodes with >= 2^depth elements per lane run their children in a loop
#endif
constexpr int kLoopDepth = PL_SC_LOOP_DEPTH;

template <int E>
using BetaT = typename std::conditional<(E <= 32), uint32_t, uint64_t>::type;

enum : int { T_GEN = 0, T_R0 = 1, T_R1 = 2, T_REP = 3, T_SPC = 4 };

struct Ctx {
    uint32_t vfrozen;  // lane l: frozen-mask word l
    uint32_t vr0, vr1, vrep, vspc;  // lane l: word l of the per-node type flags
    int lane, lig;     // lane in wave, lane in codeword group
    float lmax;
};

__device__ __forceinline__ uint32_t rl(uint32_t v, int idx) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, idx);
}

template <int FM>
__device__ __forceinline__ float fop(float x, float y, float lmax) {
    if constexpr (FM == 0) {  // polar_sc.py:46
        const float m = fminf(fminf(fabsf(x), fabsf(y)), lmax);
        const uint32_t sg = (__float_as_uint(x) ^ __float_as_uint(y)) & 0x80000000u;
        return __uint_as_float(__float_as_uint(m) | sg);
    } else {  // my_sn/fec/polar/dec.py:39-43, correctly rounded exp / log (exactf.h)
        return plx::f_exact(x, y, lmax);
    }
}
// g, polar_sc.py:49-53: (1-2u)x + y == (u ? -x : x) + y, one rounding.
__device__ __forceinline__ float gop(float x, float y, uint32_t bit) {
    return __uint_as_float(__float_as_uint(x) ^ (bit << 31)) + y;
}
template <typename T>
__device__ __forceinline__ uint32_t bitof(T w, int j) {
    return (uint32_t)(w >> j) & 1u;
}
__device__ __forceinline__ uint32_t hd(float x) { return (x > 0.0f) ? 0u : 1u; }  // polar_sc.py:94-97

// Node type of the stage-s node at position p (p wave-uniform).  Flag bit OFF(s) + (p >> s),
// OFF(s) = n - (n >> (s-1)).
template <int LOG_N, int s>
__device__ __forceinline__ int node_type(const Ctx& c, int p) {
    constexpr int off = (1 << LOG_N) - ((1 << LOG_N) >> (s - 1));
    const int idx = off + (p >> s);
    const int w = idx >> 5, b = idx & 31;
    if ((rl(c.vr0, w) >> b) & 1u) return T_R0;
    if ((rl(c.vrep, w) >> b) & 1u) return T_REP;
    if ((rl(c.vr1, w) >> b) & 1u) return T_R1;
    if ((rl(c.vspc, w) >> b) & 1u) return T_SPC;
    return T_GEN;
}
template <int LOG_N, int s>
__device__ __forceinline__ bool is_r0(const Ctx& c, int p) {
    constexpr int off = (1 << LOG_N) - ((1 << LOG_N) >> (s - 1));
    const int idx = off + (p >> s);
    return (rl(c.vr0, idx >> 5) >> (idx & 31)) & 1u;
}

// ---- cross-lane ops inside a G-lane codeword group, on DPP (VALU latency, no LDS pipe) ----
// dpp_ctrl: quad_perm 0x00-0xFF, row_shr:k 0x110+k, row_ror:k 0x120+k, row_mirror 0x140,
// row_half_mirror 0x141.  Groups of G <= 16 lanes never straddle a 16-lane DPP row.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __uint_as_float(dpp<CTRL>(__float_as_uint(v)));
}
// all-reduce over the group (every lane gets the result); commutative ops only
template <int G, typename T, typename Op>
__device__ __forceinline__ T grp_reduce(T v, Op op) {
    static_assert(G <= 16, "group wider than a DPP row");
    auto mv = [](T x, auto ctrl_tag) {
        constexpr int C = decltype(ctrl_tag)::value;
        if constexpr (sizeof(T) == 4 && std::is_same<T, float>::value) return dppf<C>(x);
        else return (T)dpp<C>((uint32_t)x);
    };
    if constexpr (G >= 2) v = op(v, mv(v, std::integral_constant<int, 0xB1>{}));   // quad_perm [1,0,3,2]
    if constexpr (G >= 4) v = op(v, mv(v, std::integral_constant<int, 0x4E>{}));   // quad_perm [2,3,0,1]
    if constexpr (G >= 8) v = op(v, mv(v, std::integral_constant<int, 0x141>{}));  // row_half_mirror
    if constexpr (G >= 16) v = op(v, mv(v, std::integral_constant<int, 0x140>{})); // row_mirror
    return v;
}
template <int G>
__device__ __forceinline__ float grp_min(float v) {
    return grp_reduce<G>(v, [](float a, float b) { return fminf(a, b); });
}
template <int G>
__device__ __forceinline__ uint32_t grp_xor(uint32_t v) {
    return grp_reduce<G>(v, [](uint32_t a, uint32_t b) { return a ^ b; });
}
template <int G>
__device__ __forceinline__ uint32_t grp_sum(uint32_t v) {
    return grp_reduce<G>(v, [](uint32_t a, uint32_t b) { return a + b; });
}
// value of lane (lig + H) of the group, for lig < H (row_ror by 16-H)
template <int H>
__device__ __forceinline__ float from_up(float v) {
    return dppf<0x120 + (16 - H)>(v);
}
// broadcast lane 0 of each G-lane group to the whole group
template <int G>
__device__ __forceinline__ float grp_bcast0(float v, int lig) {
    if constexpr (G == 1) {
        return v;
    } else {
        float t = G == 2 ? dppf<0xA0>(v) : dppf<0x00>(v);  // quad_perm [0,0,2,2] / [0,0,0,0]
        if constexpr (G >= 8) {
            const float u = dppf<0x114>(t);  // row_shr:4
            t = (lig & 4) ? u : t;
        }
        if constexpr (G >= 16) {
            const float u = dppf<0x118>(t);  // row_shr:8
            t = (lig & 8) ? u : t;
        }
        return t;
    }
}

// ---- shortcuts on a node of E = 2^s / G elements per lane ----
template <int E>
__device__ __forceinline__ bool any_zero(const float (&a)[E]) {
    bool z = false;
#pragma unroll
    for (int j = 0; j < E; ++j) z |= (a[j] == 0.0f);
    return z;
}
template <int E>
__device__ __forceinline__ BetaT<E> hd_bits(const float (&a)[E]) {
    BetaT<E> b = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) b |= (BetaT<E>)hd(a[j]) << j;
    return b;
}
// Repetition node: SC reduces it to u = HD(sum) with the sum taken in g's pairwise order.
template <int G, int E>
__device__ __forceinline__ BetaT<E> rep_node(const float (&a)[E], const Ctx& c) {
    float y[E];
#pragma unroll
    for (int j = 0; j < E; ++j) y[j] = a[j];
#pragma unroll
    for (int h = E / 2; h >= 1; h >>= 1)
#pragma unroll
        for (int j = 0; j < h; ++j) y[j] = y[j] + y[j + h];
    float v = y[0];
    if constexpr (G >= 16) v = v + from_up<8>(v);  // SC order: y_l + y_{l+h}, valid for lig < h
    if constexpr (G >= 8) v = v + from_up<4>(v);
    if constexpr (G >= 4) v = v + from_up<2>(v);
    if constexpr (G >= 2) v = v + from_up<1>(v);
    v = grp_bcast0<G>(v, c.lig);
    return hd(v) ? (BetaT<E>)(~(BetaT<E>)0 >> (8 * sizeof(BetaT<E>) - E)) : (BetaT<E>)0;
}
// SPC node (Wagner rule).  Returns false (wave-uniform) when the exactness preconditions fail.
template <int G, int E>
__device__ __forceinline__ bool spc_node(const float (&a)[E], const Ctx& c, BetaT<E>& out) {
    const bool zero = any_zero<E>(a);
    BetaT<E> b = hd_bits<E>(a);
    uint32_t par = (uint32_t)__popcll((unsigned long long)b) & 1u;
    par = grp_xor<G>(par);
    float mn = fabsf(a[0]);
#pragma unroll
    for (int j = 1; j < E; ++j) mn = fminf(mn, fabsf(a[j]));
    mn = grp_min<G>(mn);
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < E; ++j) cnt += (fabsf(a[j]) == mn);
    cnt = grp_sum<G>(cnt);
    const bool bad = zero || (par && (cnt != 1 || !(mn < c.lmax)));
    if (__any(bad)) return false;
    if (par) {
#pragma unroll
        for (int j = 0; j < E; ++j) b ^= (BetaT<E>)(fabsf(a[j]) == mn) << j;
    }
    out = b;
    return true;
}

// In-lane generic SC decode of a 2^t-leaf subtree whose LLRs are all in v (bit q of fw = frozen
// flag of subtree leaf q).  Returns the subtree's partial sums (bit j = beta_j).
template <int t, int q, int FM>
__device__ __forceinline__ uint32_t inl(const float (&v)[1 << t], uint32_t fw, float lmax) {
    if constexpr (t == 0) {
        return ((fw >> q) & 1u) ? 0u : hd(v[0]);
    } else {
        constexpr int H = 1 << (t - 1);
        constexpr uint32_t M = (t == 5) ? 0xffffffffu : ((1u << (1 << t)) - 1u);
        if (((fw >> q) & M) == M) return 0u;
        float x[H];
        uint32_t bl = 0u;
        constexpr uint32_t MH = (1u << H) - 1u;
        if (((fw >> q) & MH) != MH) {
#pragma unroll
            for (int j = 0; j < H; ++j) x[j] = fop<FM>(v[j], v[j + H], lmax);
            bl = inl<t - 1, q, FM>(x, fw, lmax);
        }
#pragma unroll
        for (int j = 0; j < H; ++j) x[j] = gop(v[j], v[j + H], bitof(bl, j));
        const uint32_t br = inl<t - 1, q + H, FM>(x, fw, lmax);
        return (bl ^ br) | (br << H);
    }
}

// v[j] = LLR held by lane j of this lane's group (all G of them, in every lane).
template <int G>
__device__ __forceinline__ void gather(float a, const Ctx& c, float (&v)[G]) {
#if PL_SC_DPP_GATHER
    if constexpr (G == 2) {
        v[0] = dppf<0xA0>(a);  // quad_perm [0,0,2,2]
        v[1] = dppf<0xF5>(a);  // quad_perm [1,1,3,3]
        return;
    } else if constexpr (G == 4) {
        v[0] = dppf<0x00>(a);
        v[1] = dppf<0x55>(a);
        v[2] = dppf<0xAA>(a);
        v[3] = dppf<0xFF>(a);
        return;
    } else if constexpr (G == 8) {
        const bool hi = (c.lig & 4) != 0;
        float t[4];
        t[0] = dppf<0x00>(a);  // quad_perm broadcast of quad lane j: a_j (low quad) / a_{4+j} (high)
        t[1] = dppf<0x55>(a);
        t[2] = dppf<0xAA>(a);
        t[3] = dppf<0xFF>(a);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float down = dppf<0x114>(t[j]);  // row_shr:4 -> high quad sees low quad
            const float up = dppf<0x104>(t[j]);    // row_shl:4 -> low quad sees high quad
            v[j] = hi ? down : t[j];
            v[4 + j] = hi ? t[j] : up;
        }
        return;
    }
#endif
    const int base = c.lane & ~(G - 1);
#pragma unroll
    for (int j = 0; j < G; ++j) v[j] = __shfl(a, base + j, 64);
}

// Node of size G at position p (one LLR per lane).  Returns this lane's partial-sum bit.
template <int LOG_N, int LOG_G, int FM>
__device__ __forceinline__ uint32_t bottom(float a, int p, const Ctx& c) {
    constexpr int G = 1 << LOG_G;
    if constexpr (G == 1) {
        return ((rl(c.vfrozen, p >> 5) >> (p & 31)) & 1u) ? 0u : hd(a);
    } else {
        const int ty = node_type<LOG_N, LOG_G>(c, p);
        if (ty == T_R0) return 0u;
        const float av[1] = {a};
        if ((kShortcuts & 1) && ty == T_REP) return rep_node<G, 1>(av, c);
        if constexpr (FM == 0) {
            if ((kShortcuts & 2) && ty == T_R1 && !__any(a == 0.0f)) return hd(a);
            if ((kShortcuts & 4) && ty == T_SPC) {
                uint32_t b;
                if (spc_node<G, 1>(av, c, b)) return b;
            }
        }
        constexpr uint32_t GM = (1u << G) - 1u;
        const uint32_t fw = (rl(c.vfrozen, p >> 5) >> (p & 31)) & GM;
        float v[G];
        gather<G>(a, c, v);
        const uint32_t beta = inl<LOG_G, 0, FM>(v, fw, c.lmax);
        return bitof(beta, c.lig);
    }
}

template <int LOG_N, int LOG_G, int s, int FM>
__device__ BetaT<(1 << (s - LOG_G))> node(const float (&a)[1 << (s - LOG_G)], int p, const Ctx& c);

template <int LOG_N, int LOG_G, int s, int FM>
__device__ __forceinline__ BetaT<(1 << (s - LOG_G))> child(const float (&x)[1 << (s - LOG_G)], int p, const Ctx& c) {
    if constexpr (s == LOG_G) {
        return bottom<LOG_N, LOG_G, FM>(x[0], p, c);
    } else {
        return node<LOG_N, LOG_G, s, FM>(x, p, c);
    }
}

// Left child all-frozen?  (then its f pass is skipped; leaves of G=1 codes use the frozen mask)
template <int LOG_N, int s>
__device__ __forceinline__ bool child_r0(const Ctx& c, int p) {
    if constexpr (s == 0) {
        return (rl(c.vfrozen, p >> 5) >> (p & 31)) & 1u;
    } else {
        return is_r0<LOG_N, s>(c, p);
    }
}

// Two children of a node whose LLRs are a[] (E per lane): polar_sc.py:54-89 on registers.
template <int LOG_N, int LOG_G, int s, int FM>
__device__ __forceinline__ BetaT<(1 << (s - LOG_G))> split(const float (&a)[1 << (s - LOG_G)], int p, const Ctx& c) {
    constexpr int E = 1 << (s - LOG_G), H = E / 2, h = 1 << (s - 1);
    using BT = BetaT<E>;
    using BH = BetaT<H>;
    float x[H];
    BH bl = 0, br = 0;
    const bool left_r0 = (kShortcuts & 8) && child_r0<LOG_N, s - 1>(c, p);
    if constexpr (E >= (1 << kLoopDepth)) {
#pragma unroll 1
        for (int side = left_r0 ? 1 : 0; side < 2; ++side) {
            if (side == 0) {
#pragma unroll
                for (int j = 0; j < H; ++j) x[j] = fop<FM>(a[j], a[j + H], c.lmax);
            } else {
#pragma unroll
                for (int j = 0; j < H; ++j) x[j] = gop(a[j], a[j + H], bitof(bl, j));
            }
            const BH b = child<LOG_N, LOG_G, s - 1, FM>(x, p + side * h, c);
            if (side == 0) bl = b; else br = b;
        }
    } else {
        if (!left_r0) {
#pragma unroll
            for (int j = 0; j < H; ++j) x[j] = fop<FM>(a[j], a[j + H], c.lmax);
            bl = child<LOG_N, LOG_G, s - 1, FM>(x, p, c);
        }
#pragma unroll
        for (int j = 0; j < H; ++j) x[j] = gop(a[j], a[j + H], bitof(bl, j));
        br = child<LOG_N, LOG_G, s - 1, FM>(x, p + h, c);
    }
    return (BT)(bl ^ br) | ((BT)br << H);
}

// Node at stage s (size 2^s) starting at position p.
template <int LOG_N, int LOG_G, int s, int FM>
__device__ __forceinline__ BetaT<(1 << (s - LOG_G))> node(const float (&a)[1 << (s - LOG_G)], int p, const Ctx& c) {
    constexpr int E = 1 << (s - LOG_G), G = 1 << LOG_G;
    using BT = BetaT<E>;
    if constexpr (E <= PL_SC_SHORTCUT_MAX_E) {
        const int ty = node_type<LOG_N, s>(c, p);
        if (ty == T_R0) return (BT)0;
        if ((kShortcuts & 1) && ty == T_REP) return rep_node<G, E>(a, c);
        if constexpr (FM == 0) {
            if ((kShortcuts & 2) && ty == T_R1 && !__any(any_zero<E>(a))) return hd_bits<E>(a);
            if ((kShortcuts & 4) && ty == T_SPC) {
                BT b;
                if (spc_node<G, E>(a, c, b)) return b;
            }
        }
    } else {
        if (is_r0<LOG_N, s>(c, p)) return (BT)0;
    }
    return split<LOG_N, LOG_G, s, FM>(a, p, c);
}

// u = x * G_n on this lane's packed slots: x[a+j] ^= x[a+h+j] for every span (polar transform,
// an involution).  Slot j of lane l is position j*G + l; spans >= G are in-lane, < G cross-lane.
template <int G>
__device__ __forceinline__ void butterfly(uint64_t& lo, uint64_t& hi, int nslots, int lig) {
    constexpr uint64_t M[6] = {0x5555555555555555ull, 0x3333333333333333ull, 0x0f0f0f0f0f0f0f0full,
                               0x00ff00ff00ff00ffull, 0x0000ffff0000ffffull, 0x00000000ffffffffull};
#pragma unroll
    for (int t = 0; t < 6; ++t) {
        const int hs = 1 << t;
        if (hs < nslots) {
            lo ^= (lo >> hs) & M[t];
            hi ^= (hi >> hs) & M[t];
        }
    }
    if (nslots > 64) lo ^= hi;
#pragma unroll
    for (int h = 1; h < G; h <<= 1) {
        const uint64_t olo = (uint64_t)__shfl_xor((long long)lo, h, 64);
        const uint64_t ohi = (uint64_t)__shfl_xor((long long)hi, h, 64);
        if ((lig & h) == 0) {
            lo ^= olo;
            hi ^= ohi;
        }
    }
}

// Root.  Stage LOG_N is the negated channel (polar_sc.py:122), read from HBM/L2, never held.
// Stage LOG_N-1 is not held either ("virtual"): each of its LLRs is recomputed from two channel
// values when the stage-(LOG_N-1) node needs it (f for the left half, g with the left half's
// partial sums for the right half), which keeps the largest stage buffer (n/2G floats per lane)
// out of the register file.  Loads are issued in chunks so the scheduler cannot hoist them all.
template <int LOG_N, int LOG_G, int FM>
__device__ __forceinline__ float root_alpha(const float* __restrict__ chl, const Ctx& c, int side, uint64_t bl_root,
                                            int j) {
    constexpr int N = 1 << LOG_N, G = 1 << LOG_G;
    const float x = -chl[j * G + c.lig], y = -chl[j * G + c.lig + N / 2];
    return side == 0 ? fop<FM>(x, y, c.lmax) : gop(x, y, bitof(bl_root, j));
}

template <int LOG_N, int LOG_G, int FM>
__device__ __forceinline__ float root_alpha_r(const float (&chv)[(1 << LOG_N) >> LOG_G], const Ctx& c, int side,
                                              uint64_t bl_root, int j) {
    constexpr int NS = (1 << LOG_N) >> LOG_G;
    const float x = -chv[j], y = -chv[j + NS / 2];
    return side == 0 ? fop<FM>(x, y, c.lmax) : gop(x, y, bitof(bl_root, j));
}

template <int LOG_N, int LOG_G, int FM>
__device__ __forceinline__ BetaT<((1 << LOG_N) >> LOG_G) / 2> half_node_r(const float (&chv)[(1 << LOG_N) >> LOG_G],
                                                                          const Ctx& c, int side, uint64_t bl_root) {
    constexpr int s = LOG_N - 1, E = (1 << s) >> LOG_G, H = E / 2, h = 1 << (s - 1);
    using BT = BetaT<E>;
    using BH = BetaT<H>;
    const int p = side * (1 << s);
    if (is_r0<LOG_N, s>(c, p)) return (BT)0;
    float x[H];
    BH bl = 0, br = 0;
    const bool left_r0 = (kShortcuts & 8) && child_r0<LOG_N, s - 1>(c, p);
#pragma unroll 1
    for (int sd = left_r0 ? 1 : 0; sd < 2; ++sd) {
        uint64_t blr = bl_root;
        asm volatile("" : "+v"(blr));
#pragma unroll
        for (int j = 0; j < H; ++j) {
            const float a0 = root_alpha_r<LOG_N, LOG_G, FM>(chv, c, side, blr, j);
            const float a1 = root_alpha_r<LOG_N, LOG_G, FM>(chv, c, side, blr, j + H);
            x[j] = sd == 0 ? fop<FM>(a0, a1, c.lmax) : gop(a0, a1, bitof(bl, j));
        }
        const BH b = child<LOG_N, LOG_G, s - 1, FM>(x, p + sd * h, c);
        if (sd == 0) bl = b; else br = b;
    }
    return (BT)(bl ^ br) | ((BT)br << H);
}

template <int LOG_N, int LOG_G, int FM>
__device__ __forceinline__ BetaT<((1 << LOG_N) >> LOG_G) / 2> half_node(const float* __restrict__ ch, const Ctx& c,
                                                                        int side, uint64_t bl_root) {
    constexpr int s = LOG_N - 1, E = (1 << s) >> LOG_G, H = E / 2, h = 1 << (s - 1);
    using BT = BetaT<E>;
    using BH = BetaT<H>;
    const int p = side * (1 << s);
    if (is_r0<LOG_N, s>(c, p)) return (BT)0;
    float x[H];
    BH bl = 0, br = 0;
    const bool left_r0 = (kShortcuts & 8) && child_r0<LOG_N, s - 1>(c, p);
    constexpr int CH = PL_SC_ROOT_CHUNK < H ? PL_SC_ROOT_CHUNK : H;
#pragma unroll 1
    for (int sd = left_r0 ? 1 : 0; sd < 2; ++sd) {
        // Launder the channel pointer per pass: the loads are loop-invariant, and LICM would
        // otherwise hoist all of them and keep the whole stage in VGPRs (the thing avoided here).
#pragma unroll
        for (int j0 = 0; j0 < H; j0 += CH) {
#if PL_SC_LAUNDER_CH
            const float* chp = ch;
            asm volatile("" : "+v"(chp));
#else
            const float* chp = ch;  // loads hoisted by LICM: the channel stays in VGPRs (one HBM pass)
#endif
            uint64_t blr = bl_root;
#if PL_SC_LAUNDER_BL
            asm volatile("" : "+v"(blr));  // keeps LICM from hoisting its 2H sign masks into VGPRs
#endif
#pragma unroll
            for (int j = j0; j < j0 + CH; ++j) {
                const float a0 = root_alpha<LOG_N, LOG_G, FM>(chp, c, side, blr, j);
                const float a1 = root_alpha<LOG_N, LOG_G, FM>(chp, c, side, blr, j + H);
                x[j] = sd == 0 ? fop<FM>(a0, a1, c.lmax) : gop(a0, a1, bitof(bl, j));
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        const BH b = child<LOG_N, LOG_G, s - 1, FM>(x, p + sd * h, c);
        if (sd == 0) bl = b; else br = b;
    }
    return (BT)(bl ^ br) | ((BT)br << H);
}

// Returns the packed re-encoded codeword slots of this lane (x = u*G_n).
template <int LOG_N, int LOG_G, int FM>
__device__ __forceinline__ void root(const float* __restrict__ ch, const Ctx& c, uint64_t& lo, uint64_t& hi) {
    constexpr int N = 1 << LOG_N, G = 1 << LOG_G, H = (N / G) / 2;
    using BH = BetaT<H>;
    BH bl = 0, br = 0;
    if constexpr (LOG_N - 1 == LOG_G) {
        // two-leaf-group codes (n = 2G): the halves are bottoms, fed straight from the channel
        const float x = -ch[c.lig], y = -ch[c.lig + N / 2];
        bl = bottom<LOG_N, LOG_G, FM>(fop<FM>(x, y, c.lmax), 0, c);
        br = bottom<LOG_N, LOG_G, FM>(gop(x, y, bl), N / 2, c);
    } else if constexpr (PL_SC_CH_REGS) {
        constexpr int NS = N / G;
        float chv[NS];
#pragma unroll
        for (int j = 0; j < NS / 2; ++j) {
            chv[j] = ch[j * G + c.lig];
            chv[j + NS / 2] = ch[j * G + c.lig + N / 2];
        }
#pragma unroll 1
        for (int side = 0; side < 2; ++side) {
            const BH b = half_node_r<LOG_N, LOG_G, FM>(chv, c, side, (uint64_t)bl);
            if (side == 0) bl = b; else br = b;
        }
    } else if constexpr (PL_SC_ROOT_STORED) {
        // stage LOG_N-1 held in VGPRs: the channel is read once per half (two HBM/L2 passes)
        float a[H];
        constexpr int CH = PL_SC_ROOT_CHUNK < H ? PL_SC_ROOT_CHUNK : H;
#pragma unroll 1
        for (int side = 0; side < 2; ++side) {
#pragma unroll
            for (int j0 = 0; j0 < H; j0 += CH) {
                const float* chp = ch;
                uint64_t blr = (uint64_t)bl;
                asm volatile("" : "+v"(chp), "+v"(blr));
#pragma unroll
                for (int j = j0; j < j0 + CH; ++j) a[j] = root_alpha<LOG_N, LOG_G, FM>(chp, c, side, blr, j);
                __builtin_amdgcn_sched_barrier(0);
            }
            const BH b = child<LOG_N, LOG_G, LOG_N - 1, FM>(a, side * (N / 2), c);
            if (side == 0) bl = b; else br = b;
        }
    } else {
#pragma unroll 1
        for (int side = 0; side < 2; ++side) {
            const float* chp = ch;
#if PL_SC_LAUNDER_CH
            asm volatile("" : "+v"(chp));
#endif
            const BH b = half_node<LOG_N, LOG_G, FM>(chp, c, side, (uint64_t)bl);
            if (side == 0) bl = b; else br = b;
        }
    }
    // root partial sums x = [bl ^ br, br]: H slots each
    if constexpr (H >= 64) {
        lo = (uint64_t)(bl ^ br);
        hi = (uint64_t)br;
    } else {
        lo = (uint64_t)(bl ^ br) | ((uint64_t)br << H);
        hi = 0;
    }
}

template <int LOG_N, int FM, int OUTK>
__global__ __launch_bounds__(64 * kWavesPerBlock, PL_SC_MIN_WAVES) void sc_decode_kernel(
    const float* __restrict__ llr, int64_t bs, void* __restrict__ out, const uint32_t* __restrict__ frozen_words,
    const uint32_t* __restrict__ type_words, int type_stride, const int32_t* __restrict__ info_pos, int k,
    float lmax) {
    constexpr int LOG_G = (LOG_N > 7) ? (LOG_N - 7) : 0;
    constexpr int N = 1 << LOG_N, G = 1 << LOG_G, C = 64 / G;
    constexpr int NSL = N / G;                       // slots per lane (<= 128)
    constexpr int WPL = (NSL + 31) / 32;             // u words per lane
    constexpr int WPC = (N + 31) / 32;               // frozen words
    __shared__ uint32_t ulds[kWavesPerBlock * 64 * WPL];

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int grp = lane >> LOG_G;
    const int64_t cw0 = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * C;
    const int64_t cw = cw0 + grp;
#if PL_SC_DIAG_SAMEROW
    const float* ch = llr + (size_t)((cw < bs ? cw : bs - 1) & 255) * N;  // diagnostic: L2-resident input
#else
    const float* ch = llr + (size_t)(cw < bs ? cw : bs - 1) * N;
#endif

    Ctx c;
    c.vfrozen = lane < WPC ? frozen_words[lane] : 0u;
    c.vr0 = type_words[0 * type_stride + lane];
    c.vr1 = type_words[1 * type_stride + lane];
    c.vrep = type_words[2 * type_stride + lane];
    c.vspc = type_words[3 * type_stride + lane];
    c.lane = lane;
    c.lig = lane & (G - 1);
    c.lmax = lmax;
    if constexpr (FM == 1) plx::load_tables(threadIdx.x, blockDim.x);  // the exact f's exp / log tables

    uint64_t lo, hi;
    root<LOG_N, LOG_G, FM>(ch, c, lo, hi);
    butterfly<G>(lo, hi, NSL, c.lig);

    uint32_t* mine = ulds + (wave * 64 + lane) * WPL;
    mine[0] = (uint32_t)lo;
    if constexpr (WPL > 1) mine[1] = (uint32_t)(lo >> 32);
    if constexpr (WPL > 2) {
        mine[2] = (uint32_t)hi;
        mine[3] = (uint32_t)(hi >> 32);
    }
    __syncthreads();

#if PL_SC_DIAG_NOSTORE
    if (lo == 0x123456789ull && hi == 7) static_cast<float*>(out)[cw] = 1.0f;  // diagnostic: keep the tree live
    return;
#endif
    // Gather the k information bits (info_pos ascending, polar_sc.py:127) -> coalesced rows.
    const uint32_t* ubase = ulds + wave * 64 * WPL;
    for (int g = 0; g < C; ++g) {
        const int64_t row = cw0 + g;
        if (row >= bs) break;
        for (int m = lane; m < k; m += 64) {
            const int pos = info_pos[m];
            const int l = pos & (G - 1), slot = pos >> LOG_G;
            const uint32_t bit = (ubase[(g * G + l) * WPL + (slot >> 5)] >> (slot & 31)) & 1u;
            if constexpr (OUTK == PL_OUT_F32) {
                static_cast<float*>(out)[row * k + m] = bit ? 1.0f : 0.0f;
            } else {
                static_cast<uint8_t*>(out)[row * k + m] = (uint8_t)bit;
            }
        }
    }
}

template <int LOG_N, int FM, int OUTK>
void launch_one(const pl_plan* p, const float* llr, int64_t bs, void* out, hipStream_t st) {
    constexpr int LOG_G = (LOG_N > 7) ? (LOG_N - 7) : 0;
    constexpr int C = 64 >> LOG_G;
    const int64_t per_block = (int64_t)kWavesPerBlock * C;
    const int64_t blocks = (bs + per_block - 1) / per_block;
    hipLaunchKernelGGL((sc_decode_kernel<LOG_N, FM, OUTK>), dim3((unsigned)blocks), dim3(64 * kWavesPerBlock), 0, st,
                       llr, bs, out, p->d_frozen_words, p->d_type_words, p->type_stride, p->d_info_pos, p->k,
                       p->llr_max);
}

template <int LOG_N>
void dispatch_fm(const pl_plan* p, const float* llr, int64_t bs, void* out, int out_kind, hipStream_t st) {
    if (p->f_mode == PL_F_MINSUM) {
        if (out_kind == PL_OUT_F32) launch_one<LOG_N, 0, PL_OUT_F32>(p, llr, bs, out, st);
        else launch_one<LOG_N, 0, PL_OUT_U8>(p, llr, bs, out, st);
    } else {
        if (out_kind == PL_OUT_F32) launch_one<LOG_N, 1, PL_OUT_F32>(p, llr, bs, out, st);
        else launch_one<LOG_N, 1, PL_OUT_U8>(p, llr, bs, out, st);
    }
}

}  // namespace

namespace pl {
int launch_sc(const pl_plan* p, const float* llr, int64_t bs, void* out, int out_kind, hipStream_t st) {
    if (bs == 0 || p->k == 0) return PL_OK;
    switch (p->log_n) {
        case 1: dispatch_fm<1>(p, llr, bs, out, out_kind, st); break;
        case 2: dispatch_fm<2>(p, llr, bs, out, out_kind, st); break;
        case 3: dispatch_fm<3>(p, llr, bs, out, out_kind, st); break;
        case 4: dispatch_fm<4>(p, llr, bs, out, out_kind, st); break;
        case 5: dispatch_fm<5>(p, llr, bs, out, out_kind, st); break;
        case 6: dispatch_fm<6>(p, llr, bs, out, out_kind, st); break;
        case 7: dispatch_fm<7>(p, llr, bs, out, out_kind, st); break;
        case 8: dispatch_fm<8>(p, llr, bs, out, out_kind, st); break;
        case 9: dispatch_fm<9>(p, llr, bs, out, out_kind, st); break;
        case 10: dispatch_fm<10>(p, llr, bs, out, out_kind, st); break;
        case 11: dispatch_fm<11>(p, llr, bs, out, out_kind, st); break;
        default: set_error("SC decode: n must be a power of two in [2, 2048]"); return PL_ENOTSUP;
    }
    return check_hip(hipGetLastError(), "SC decode launch");
}
}  // namespace pl
