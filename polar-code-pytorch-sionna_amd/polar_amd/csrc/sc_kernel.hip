// sc_kernel.hip -- successive-cancellation (SC) polar decoder for gfx950 (MI355X).
//
// Reference semantics: x_run_sn_polar/polar/polar_sc.py (SC_Dec, min-sum f forced at :46,
// g :49-53, leaf rule :90-98, partial sums :83-89) and, for f_mode=PL_F_EXACT, the exact boxplus
// of my_sn/fec/polar/dec.py:33-46.  Results are bit-identical to the reference for min-sum
// (f is sign/min, g is one fp32 add; both are exact restatements).
//
// Design ("register tree"): a wave64 decodes C = 64/G codewords at once, G lanes per codeword.
// Element i of a stage buffer lives in lane (i mod G) of its codeword's lane group, slot i/G, so
// every f/g of a node of size >= 2G pairs elements that sit in the SAME lane: the upper stages
// run entirely in VGPRs with no LDS and no cross-lane traffic.  A node of size G (one element
// per lane) is finished by gathering its G LLRs into every lane of the group (ds_bpermute) and
// decoding that small subtree redundantly in-lane.  G = max(1, n/128) keeps the deepest live
// set of stage buffers (about n/G floats per lane) near 128 VGPRs.  Partial sums (beta) are
// bit-packed per lane.  The tree walk is generated at compile time (templates on the stage);
// above a small depth each node runs its two children in a runtime 2-trip loop so code size
// stays O(n/G) rather than O(n).  The frozen pattern is runtime data: a per-lane copy of the
// frozen bitmask and of the rate-0 node bitmask (one 32-bit word per lane) is queried with
// v_readlane on wave-uniform positions, and all-frozen (rate-0) subtrees are skipped, which is
// exact (the reference just writes zeros there).  Decided bits are packed into LDS (n/8 bytes
// per codeword) and written out coalesced at the end (gathered at info_pos).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../../include/polar_mi355x.h"
#include "plan.h"

namespace {

constexpr int kWavesPerBlock = 4;
constexpr int kLoopDepth = 3;  // nodes with >= 2^kLoopDepth elements per lane use the side loop

template <int E>
using BetaT = typename std::conditional<(E <= 32), uint32_t, uint64_t>::type;

struct Ctx {
    uint32_t vfrozen;  // lane l: frozen-mask word l
    uint32_t vrate0;   // lane l: rate-0 node-flag word l
    uint32_t ucur;     // decided bits of the current 32-position word
    uint32_t* ulds;    // this lane group's codeword: packed decided bits in LDS
    int lane, lig;     // lane in wave, lane in codeword group
    float lmax;
};

__device__ __forceinline__ uint32_t rl(uint32_t v, int idx) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, idx);
}

// f, polar_sc.py:33-48 (min-sum; clip only bounds the magnitude) / dec.py:33-46 (exact).
template <int FM>
__device__ __forceinline__ float fop(float x, float y, float lmax) {
    if constexpr (FM == 0) {
        const float m = fminf(fminf(fabsf(x), fabsf(y)), lmax);
        const uint32_t sg = (__float_as_uint(x) ^ __float_as_uint(y)) & 0x80000000u;
        return __uint_as_float(__float_as_uint(m) | sg);
    } else {
        const float xc = fminf(fmaxf(x, -lmax), lmax), yc = fminf(fmaxf(y, -lmax), lmax);
        float o = logf(1.0f + expf(xc + yc));
        o -= logf(expf(xc) + expf(yc));
        return o;
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

// Rate-0 flag of the stage-s node starting at position p (p wave-uniform).
template <int LOG_N, int s>
__device__ __forceinline__ bool is_rate0(const Ctx& c, int p) {
    constexpr int off = (1 << LOG_N) - ((1 << LOG_N) >> (s - 1));
    const int idx = off + (p >> s);
    return (rl(c.vrate0, idx >> 5) >> (idx & 31)) & 1u;
}

// In-lane SC decode of a 2^t-leaf subtree whose LLRs are all in v (bit q of fw = frozen flag of
// subtree leaf q).  Returns the subtree's partial sums (bit j = beta_j); info decisions are OR-ed
// into ub at their leaf offset.  Leaf rule polar_sc.py:90-98: u = 1 iff !(llr > 0).
template <int t, int q, int FM>
__device__ __forceinline__ uint32_t inl(const float (&v)[1 << t], uint32_t fw, uint32_t& ub, float lmax) {
    if constexpr (t == 0) {
        uint32_t u = (v[0] > 0.0f) ? 0u : 1u;
        u = ((fw >> q) & 1u) ? 0u : u;
        ub |= u << q;
        return u;
    } else {
        constexpr int H = 1 << (t - 1);
        constexpr uint32_t M = (t == 5) ? 0xffffffffu : ((1u << (1 << t)) - 1u);
        if (((fw >> q) & M) == M) return 0u;
        float x[H];
#pragma unroll
        for (int j = 0; j < H; ++j) x[j] = fop<FM>(v[j], v[j + H], lmax);
        const uint32_t bl = inl<t - 1, q, FM>(x, fw, ub, lmax);
#pragma unroll
        for (int j = 0; j < H; ++j) x[j] = gop(v[j], v[j + H], bitof(bl, j));
        const uint32_t br = inl<t - 1, q + H, FM>(x, fw, ub, lmax);
        return (bl ^ br) | (br << H);
    }
}

// Decided bits are collected 32 positions at a time and stored when a word is complete.  A
// skipped (rate-0) node that ends a word must still store it.
__device__ __forceinline__ void end_of_range(int p_end, Ctx& c) {
    if ((p_end & 31) == 0) {
        if (c.lig == 0) c.ulds[(p_end - 1) >> 5] = c.ucur;
        c.ucur = 0u;
    }
}

// Node of size G at position p: one LLR per lane.  Returns this lane's partial-sum bit.
template <int LOG_G, int FM>
__device__ __forceinline__ uint32_t bottom(float a, int p, Ctx& c) {
    constexpr int G = 1 << LOG_G;
    constexpr uint32_t GM = (G == 32) ? 0xffffffffu : ((1u << G) - 1u);
    const uint32_t fw = (rl(c.vfrozen, p >> 5) >> (p & 31)) & GM;
    uint32_t beta = 0u, ub = 0u;
    if (fw != GM) {
        float v[G];
        if constexpr (G == 1) {
            v[0] = a;
        } else {
            const int base = c.lane & ~(G - 1);
#pragma unroll
            for (int j = 0; j < G; ++j) v[j] = __shfl(a, base + j, 64);
        }
        beta = inl<LOG_G, 0, FM>(v, fw, ub, c.lmax);
    }
    c.ucur |= ub << (p & 31);
    end_of_range(p + G, c);
    return bitof(beta, c.lig);
}

template <int LOG_N, int LOG_G, int s, int FM>
__device__ BetaT<(1 << (s - LOG_G))> node(const float (&a)[1 << (s - LOG_G)], int p, Ctx& c);

template <int LOG_N, int LOG_G, int s, int FM>
__device__ __forceinline__ BetaT<(1 << (s - LOG_G))> child(const float (&x)[1 << (s - LOG_G)], int p, Ctx& c) {
    if constexpr (s == LOG_G) {
        return bottom<LOG_G, FM>(x[0], p, c);
    } else {
        return node<LOG_N, LOG_G, s, FM>(x, p, c);
    }
}

// Node at stage s (size 2^s) starting at position p: polar_sc.py:54-89 on registers.
template <int LOG_N, int LOG_G, int s, int FM>
__device__ __forceinline__ BetaT<(1 << (s - LOG_G))> node(const float (&a)[1 << (s - LOG_G)], int p, Ctx& c) {
    constexpr int E = 1 << (s - LOG_G), H = E / 2, h = 1 << (s - 1);
    using BT = BetaT<E>;
    using BH = BetaT<H>;
    if (is_rate0<LOG_N, s>(c, p)) {
        // all positions frozen: bits stay 0 (polar_sc.py:92); nodes >= 32 are word-aligned
        if constexpr ((1 << s) < 32) end_of_range(p + (1 << s), c);
        return (BT)0;
    }
    float x[H];
    BH bl = 0, br = 0;
    if constexpr (E >= (1 << kLoopDepth)) {
#pragma unroll 1
        for (int side = 0; side < 2; ++side) {
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
#pragma unroll
        for (int j = 0; j < H; ++j) x[j] = fop<FM>(a[j], a[j + H], c.lmax);
        bl = child<LOG_N, LOG_G, s - 1, FM>(x, p, c);
#pragma unroll
        for (int j = 0; j < H; ++j) x[j] = gop(a[j], a[j + H], bitof(bl, j));
        br = child<LOG_N, LOG_G, s - 1, FM>(x, p + h, c);
    }
    return (BT)(bl ^ br) | ((BT)br << H);
}

// Root: stage-LOG_N LLRs are the negated channel logits (polar_sc.py:122), read from HBM in
// both passes instead of being held in registers.
template <int LOG_N, int LOG_G, int FM>
__device__ __forceinline__ void root(const float* __restrict__ ch, Ctx& c) {
    constexpr int N = 1 << LOG_N, G = 1 << LOG_G, H = (N / G) / 2;
    using BH = BetaT<H>;
    float x[H];
    BH bl = 0;
#pragma unroll 1
    for (int side = 0; side < 2; ++side) {
        if (side == 0) {
#pragma unroll
            for (int j = 0; j < H; ++j) {
                const int i = j * G + c.lig;
                x[j] = fop<FM>(-ch[i], -ch[i + N / 2], c.lmax);
            }
        } else {
#pragma unroll
            for (int j = 0; j < H; ++j) {
                const int i = j * G + c.lig;
                x[j] = gop(-ch[i], -ch[i + N / 2], bitof(bl, j));
            }
        }
        const BH b = child<LOG_N, LOG_G, LOG_N - 1, FM>(x, side * (N / 2), c);
        if (side == 0) bl = b;
    }
}

template <int LOG_N, int FM, int OUTK>
__global__ __launch_bounds__(64 * kWavesPerBlock) void sc_decode_kernel(
    const float* __restrict__ llr, int64_t bs, void* __restrict__ out,
    const uint32_t* __restrict__ frozen_words, const uint32_t* __restrict__ rate0_words,
    const int32_t* __restrict__ info_pos, int k, float lmax) {
    constexpr int LOG_G = (LOG_N > 7) ? (LOG_N - 7) : 0;
    constexpr int N = 1 << LOG_N, G = 1 << LOG_G, C = 64 / G;
    constexpr int WPC = (N + 31) / 32;       // packed-bit words per codeword
    constexpr int NW = (N - 1 + 31) / 32;    // rate-0 flag words
    __shared__ uint32_t ulds[kWavesPerBlock * C * WPC];

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int grp = lane >> LOG_G;
    const int64_t cw0 = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * C;
    const int64_t cw = cw0 + grp;
    const float* ch = llr + (size_t)(cw < bs ? cw : bs - 1) * N;

    Ctx c;
    c.vfrozen = lane < WPC ? frozen_words[lane] : 0u;
    c.vrate0 = lane < NW ? rate0_words[lane] : 0u;
    c.ucur = 0u;
    c.ulds = ulds + (wave * C + grp) * WPC;
    c.lane = lane;
    c.lig = lane & (G - 1);
    c.lmax = lmax;

    root<LOG_N, LOG_G, FM>(ch, c);
    if constexpr (N < 32) {
        if (c.lig == 0) c.ulds[0] = c.ucur;
    }
    __syncthreads();

    // Gather the k information bits (info_pos ascending, polar_sc.py:127) -> coalesced rows.
    const uint32_t* ubase = ulds + wave * C * WPC;
    for (int g = 0; g < C; ++g) {
        const int64_t row = cw0 + g;
        if (row >= bs) break;
        const uint32_t* U = ubase + g * WPC;
        for (int m = lane; m < k; m += 64) {
            const int pos = info_pos[m];
            const uint32_t bit = (U[pos >> 5] >> (pos & 31)) & 1u;
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
                       llr, bs, out, p->d_frozen_words, p->d_rate0_words, p->d_info_pos, p->k, p->llr_max);
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
