// scl_tree_kernel.hip -- SC-list polar decoder for gfx950 (MI355X), "register subtree" form.
//
// Same decoder as scl_kernel.hip (x_run_sn_polar/polar/polar_scl.py SCL_Dec, :49-234; and the
// exact-f variant of my_sn/fec/polar/dec.py:330-339 without fast-SCL pruning), restructured for
// latency: the reference walks the tree leaf by leaf with a sort + full-row copy of all 2L paths
// at every information leaf (:86-120); here
//
//  * the bottom of the tree runs LANE-PER-PATH: lane p (< L) decodes path p's stage-R node
//    (R = 5, 32 leaves) entirely in its VGPRs -- stage buffers 0..R-1 (31 fp64), the node's
//    partial sums as one bit word, the path metric.  f/g, the per-leaf metric update
//    (:69-85) and, at information leaves, the 2L-candidate selection (:86-92) run without LDS
//    traffic: candidates are ranked by v_readlane broadcasts (stable (metric, candidate index)
//    order, candidate c < L = (state c, u=0), c >= L = (state c-L, u=1) -- the reference's
//    logical order after _update_single_bit_np :49-68), and a fork (:109-120) pulls the parent's
//    LIVE stage buffers with ds_bpermute (a stage-s buffer is live iff the leaf is in the left
//    half of its stage-s node; dead ones are never copied);
//  * forks only move register state: each lane records the path it descends from at subtree
//    entry ("origin"); the LDS state of the upper tree (stage-buffer owner pointers, partial
//    sums of finished nodes) is re-pointed once per subtree, from the origins, instead of once
//    per information leaf;
//  * the upper stages run WAVE-PARALLEL over (path, element) from LDS, with lazy copies (per
//    path per stage owner pointers, as scl_kernel.hip);
//  * the top V stages below the channel are never stored: a node reading one recomputes its
//    input from the channel and the path's partial sums (f/g are pure functions of those), so a
//    codeword needs ~11 KB of LDS at n=1024, L=8 (14 codewords per CU instead of 4);
//  * decided bits are not tracked: the root's partial sums are x = u G_n and u = x G_n (G_n is
//    an involution over GF(2)), recovered by one butterfly per path at the end.
//
// Every f, g and metric value is computed by the same fp64 expressions, in the same order, as
// scl_kernel.hip, so the two kernels agree bit for bit (tests/test_scl_gpu.py runs both).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/polar_mi355x.h"
#include "plan.h"

namespace {

// Tuning macros (A/B variants: tools/scl_variants.py)
#ifndef PL_SCL_R
#define PL_SCL_R 4  // stage of the lane-local subtree (4 or 5; A/B on MI355X: 4 is 19 % faster)
#endif
#ifndef PL_SCL_LOADGRP
#define PL_SCL_LOADGRP 0  // > 0: stage-R input read in groups of this many pairs (caps VGPRs)
#endif
#ifndef PL_SCL_WPE
#define PL_SCL_WPE 0  // > 0: amdgpu_waves_per_eu minimum
#endif

constexpr int R = PL_SCL_R;  // stage of the lane-local subtree
constexpr int T = 1 << R;    // leaves per lane-local subtree (<= one partial-sum word)

__host__ __device__ inline int align16(int x) { return (x + 15) & ~15; }

struct Lay {
    int W;    // partial-sum words per path
    int SS;   // top stored stage (R..SS in LDS); SS == R == S: the channel is the subtree input,
              // kept as fp64 in A[0, T) and shared by every path (per = 0)
    int per;  // doubles per path of stored stages
    int off_A, off_ch, off_beta, off_sptr, off_org, off_ps, off_pm, off_fail, bytes;
};

__host__ __device__ inline Lay make_layout(int n, int S, int L, int V) {
    Lay y;
    y.W = n / 32;
    y.SS = S == R ? R : S - 1 - V;
    y.per = S == R ? 0 : (1 << (y.SS + 1)) - (1 << R);
    int o = 0;
    y.off_A = o; o = align16(o + (S == R ? T : L * y.per) * 8);
    y.off_ch = o; o = align16(o + n * 4);
    y.off_beta = o; o = align16(o + L * y.W * 4);
    y.off_sptr = o; o = align16(o + L * (S + 1));
    y.off_org = o; o = align16(o + L * 4);
    y.off_ps = o; o = align16(o + L * 4);
    y.off_pm = o; o = align16(o + L * 8);
    y.off_fail = o; o = align16(o + L * 4);
    y.bytes = o;
    return y;
}

__device__ __forceinline__ double f_ms(double x, double y, double lmax) {  // polar_scl.py:93-106
    const double m = fmin(fmin(fabs(x), fabs(y)), lmax);
    const bool neg = (__double_as_longlong(x) ^ __double_as_longlong(y)) < 0;
    return neg ? -m : m;
}
__device__ __forceinline__ double f_ex(double x, double y, double lmax) {  // my_sn dec.py:330-339
    const double xc = fmax(fmin(x, lmax), -lmax), yc = fmax(fmin(y, lmax), -lmax);
    double o = log(1.0 + exp(xc + yc));
    o -= log(exp(xc) + exp(yc));
    return o;
}
template <int FM>
__device__ __forceinline__ double f_op(double x, double y, double lmax) {
    if constexpr (FM == 0) return f_ms(x, y, lmax);
    else return f_ex(x, y, lmax);
}
__device__ __forceinline__ double g_op(double x, double y, uint32_t bit) {  // :107-108
    return (bit ? -x : x) + y;
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

// Element j of the stage-s node at position pos of one path, D stages below the channel,
// recomputed from the channel and the path's partial sums (virtual stages).
template <int D, int FM>
__device__ __forceinline__ double vread(const float* ch, const uint32_t* beta, int s, int pos, int j, double lmax) {
    if constexpr (D == 0) {
        return (double)ch[j];
    } else {
        const int h = 1 << s, pp = pos & ~(2 * h - 1);
        const double x = vread<D - 1, FM>(ch, beta, s + 1, pp, j, lmax);
        const double y = vread<D - 1, FM>(ch, beta, s + 1, pp, j + h, lmax);
        return pos == pp ? f_op<FM>(x, y, lmax) : g_op(x, y, getbit(beta, pp + j));
    }
}

struct St {
    double* A;        // [L][per] stage s (R <= s <= SS) of buffer b at A[b*per + 2^s - 2^R + j]
    float* ch;        // [n] negated channel LLRs (stage S)
    uint32_t* beta;   // [L][W] partial sums by absolute position
    uint8_t* sptr;    // [L][S+1] owner buffer of stage s
    int* org_s;       // [L] subtree exchange: origin path
    uint32_t* ps_s;   // [L] subtree exchange: partial-sum word
    int n, S, W, SS, per;
    double lmax;
};

// Element j + M 2^s of the stage-(s+T) node on the path to the channel, for the stage-s node at
// pos (D = S - s stages below the channel).  c[m] = channel element j + m 2^s; base[t] =
// start of the stage-(s+t+1) node + j (g at level t reads bit base[t] + M 2^s of the path).
template <int D, int T, int M, int FM>
__device__ __forceinline__ double vtree(const double* c, const uint32_t* bp, const int* base, uint32_t gmask, int hs,
                                        double lmax) {
    if constexpr (T == D) {
        return c[M];
    } else {
        const double x = vtree<D, T + 1, M, FM>(c, bp, base, gmask, hs, lmax);
        const double y = vtree<D, T + 1, M + (1 << T), FM>(c, bp, base, gmask, hs, lmax);
        if ((gmask >> T) & 1u) return g_op(x, y, getbit(bp, base[T] + M * hs));
        return f_op<FM>(x, y, lmax);
    }
}

// Upper-tree node at stage s (> R), position pos: f (or g) of its input into the stage-(s-1)
// buffers of every path (s-1 <= SS), wave-parallel over (path, element).  When the input is
// virtual (s = SS + 1, V stages below the channel) each lane keeps one element j and loops over
// the paths, so the 2 x 2^V channel values it needs are read once, not once per path.
template <int L, int V, int FM>
__device__ void node_fg(const St& t, int s, int pos, bool is_g, int lane) {
    const int ls = s - 1, h = 1 << ls;
    if (s <= t.SS || h < 64) {
        const int total = L * h;
        for (int idx = lane; idx < total; idx += 64) {
            const int p = idx >> ls, j = idx & (h - 1);
            const uint32_t* bp = t.beta + p * t.W;
            double x, y;
            if (s <= t.SS) {
                const double* in = t.A + t.sptr[p * (t.S + 1) + s] * t.per + (1 << s) - (1 << R);
                x = in[j];
                y = in[j + h];
            } else {  // s == SS + 1: V stages below the channel
                x = vread<V, FM>(t.ch, bp, s, pos, j, t.lmax);
                y = vread<V, FM>(t.ch, bp, s, pos, j + h, t.lmax);
            }
            const double r = is_g ? g_op(x, y, getbit(bp, pos + j)) : f_op<FM>(x, y, t.lmax);
            t.A[p * t.per + (1 << ls) - (1 << R) + j] = r;
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
        for (int j = lane; j < h; j += 64) {
            double cx[NC], cy[NC];
#pragma unroll
            for (int m = 0; m < NC; ++m) {
                cx[m] = (double)t.ch[j + m * hs];
                cy[m] = (double)t.ch[j + h + m * hs];
            }
            int basex[V > 0 ? V : 1], basey[V > 0 ? V : 1];
#pragma unroll
            for (int q = 0; q < V; ++q) {
                basex[q] = bx[q] + j;
                basey[q] = by[q] + j;
            }
            for (int p = 0; p < L; ++p) {
                const uint32_t* bp = t.beta + p * t.W;
                const double x = vtree<V, 0, 0, FM>(cx, bp, basex, gmask, hs, t.lmax);
                const double y = vtree<V, 0, 0, FM>(cy, bp, basey, gmask, hs, t.lmax);
                const double r = is_g ? g_op(x, y, getbit(bp, pos + j)) : f_op<FM>(x, y, t.lmax);
                t.A[p * t.per + (1 << ls) - (1 << R) + j] = r;
            }
        }
    }
    if (lane < L) t.sptr[lane * (t.S + 1) + ls] = (uint8_t)lane;
    __syncthreads();
}

// beta[pos, pos+h) ^= beta[pos+h, pos+2h) for every path, h = 2^(s-1): word XORs for h >= 32,
// in-word bit ops below.
template <int L>
__device__ void combine_upper(const St& t, int s, int pos, int lane) {
    const int h = 1 << (s - 1);
    if (h >= 32) {
        const int hw = h >> 5, w0 = pos >> 5;
        for (int idx = lane; idx < L * hw; idx += 64) {
            const int p = idx / hw, w = idx - p * hw;
            uint32_t* b = t.beta + p * t.W;
            b[w0 + w] ^= b[w0 + hw + w];
        }
    } else if (lane < L) {
        uint32_t* b = t.beta + lane * t.W + (pos >> 5);
        *b ^= (*b >> h) & (((1u << h) - 1u) << (pos & 31));
    }
    __syncthreads();
}

// ---- lane-local subtree --------------------------------------------------------------------
// st[2^s - 1 + j] = element j of the stage-s buffer (s < R).
constexpr int IDX(int s) { return (1 << s) - 1; }

template <int s, int FM>
__device__ __forceinline__ void f_down(double* st, double lmax) {
    if constexpr (s >= 1) {
        constexpr int h = 1 << (s - 1);
#pragma unroll
        for (int j = 0; j < h; ++j) st[IDX(s - 1) + j] = f_op<FM>(st[IDX(s) + j], st[IDX(s) + j + h], lmax);
        f_down<s - 1, FM>(st, lmax);
    }
}

// stage-R input element j of a lane's subtree (the origin's stored buffer, or the channel)
__device__ __forceinline__ double in_R(const St&, const double* inA, int j) { return inA[j]; }

__device__ __forceinline__ void load_group_fence(int j) {
#if PL_SCL_LOADGRP > 0
    if ((j + 1) % PL_SCL_LOADGRP == 0) __builtin_amdgcn_sched_barrier(0);
#else
    (void)j;
#endif
}

// Leaf i (> 0) with tz = ctz(i) trailing zeros: g at stage tz+1 into stage tz, then f down.
template <int tz, int FM>
__device__ __forceinline__ void g_step(const St& t, const double* inA, double* st, uint32_t ps, int i) {
    constexpr int h = 1 << tz;
    const int p0 = i - h;  // start of the left sibling, whose partial sums g consumes
#pragma unroll
    for (int j = 0; j < h; ++j) {
        double x, y;
        if constexpr (tz + 1 == R) {
            x = in_R(t, inA, j);
            y = in_R(t, inA, j + h);
        } else {
            x = st[IDX(tz + 1) + j];
            y = st[IDX(tz + 1) + j + h];
        }
        st[IDX(tz) + j] = g_op(x, y, (ps >> (p0 + j)) & 1u);
        if constexpr (tz + 1 == R) load_group_fence(j);
    }
    f_down<tz, FM>(st, t.lmax);
}

template <int FM>
__device__ __forceinline__ void leaf_llr(const St& t, const double* inA, double* st, uint32_t ps, int i) {
    if (i == 0) {
        constexpr int h = T / 2;
#pragma unroll
        for (int j = 0; j < h; ++j) {
            st[IDX(R - 1) + j] = f_op<FM>(in_R(t, inA, j), in_R(t, inA, j + h), t.lmax);
            load_group_fence(j);
        }
        f_down<R - 1, FM>(st, t.lmax);
        return;
    }
    switch (__builtin_ctz(i)) {
        case 0: g_step<0, FM>(t, inA, st, ps, i); break;
        case 1: g_step<1, FM>(t, inA, st, ps, i); break;
        case 2: g_step<2, FM>(t, inA, st, ps, i); break;
        case 3: g_step<3, FM>(t, inA, st, ps, i); break;
        default: g_step<R - 1, FM>(t, inA, st, ps, i); break;
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

// Decode the stage-R node at absolute position i0 for every path (lanes < L own paths; the
// other lanes shadow lane % L and are ignored).  pm, org: the lane's metric and origin.
template <int L, int FM>
__device__ void subtree(const St& t, int i0, uint32_t fz, double& pm, int& org, uint32_t& ps, int lane) {
    double st[T - 1];
    ps = 0u;
    org = lane & (L - 1);
    const double* inA = t.A + org * t.per;  // stage R sits at offset 0 of a path's region
    for (int i = 0; i < T; ++i) {
        if (i > 0) {  // nodes that ended at leaf i-1 (stages 1..ctz(i)): [uL ^ uR, uR] (:147-153)
            const int tz = __builtin_ctz(i);
            for (int s = 1; s <= tz; ++s) {
                const int h = 1 << (s - 1), pos = i - (1 << s);
                ps ^= (ps >> h) & (((1u << h) - 1u) << pos);
            }
            if (tz + 1 == R) inA = t.A + org * t.per;  // the origin may have changed
        }
        leaf_llr<FM>(t, inA, st, ps, i);
        const double l = fmax(fmin(st[0], t.lmax), -t.lmax);
        // metric update (:83): pen = log(1 + exp(-(1-2u) l)).  At an information leaf lanes
        // c >= L (shadows of state c & (L-1)) evaluate u = 1, lanes c < L u = 0: one exp/log per
        // lane gives all 2L candidates.  Same expression as the reference, so same rounding.
        const bool info = ((fz >> i) & 1u) == 0u;
        const bool hi = (lane & L) != 0;
        const double sl = (info && hi) ? -1.0 * l : 1.0 * l;
        const double pen = log(1.0 + exp(-sl));
        if (!info) {  // frozen leaf: metric update only (u = 0)
            pm = pm + pen;
            continue;
        }
        // Lane c < 2L holds candidate c: c < L = (state c, u=0), c >= L = (state c-L, u=1).  Its
        // rank in the stable (metric, index) order comes from 2L readlane broadcasts; one
        // ds_permute then sends every candidate to the lane of its rank (ranks are a permutation
        // of [0, 2L); lanes >= 2L send to themselves, so every lane is written exactly once), and
        // slots >= L re-shadow slot & (L-1).
        const double cv = pm + pen;
        int rk = 0;
#pragma unroll
        for (int c = 0; c < 2 * L; ++c) {
            const double v = readlane_d(cv, c);
            rk += (v < cv || (v == cv && c < lane)) ? 1 : 0;
        }
        const int dst = lane < 2 * L ? rk : lane;
        const int code = (lane & (L - 1)) | (hi ? 256 : 0);
        const long long cb = __double_as_longlong(cv);
        int rcode = __builtin_amdgcn_ds_permute(dst << 2, code);
        int rlo = __builtin_amdgcn_ds_permute(dst << 2, (int)(cb & 0xffffffffLL));
        int rhi = __builtin_amdgcn_ds_permute(dst << 2, (int)(cb >> 32));
        const int me = lane & (L - 1);
        rcode = bperm_i(rcode, me);
        rlo = bperm_i(rlo, me);
        rhi = bperm_i(rhi, me);
        const int par = rcode & 255;
        const uint32_t bit = (uint32_t)rcode >> 8;
        const double npm = __longlong_as_double(((long long)rhi << 32) | (unsigned int)rlo);
        pm = npm;
        ps = (uint32_t)bperm_i((int)ps, par) | (bit << i);
        org = bperm_i(org, par);
        inA = t.A + org * t.per;
        pull_live<R - 1>(st, i, par);
    }
    for (int s = 1; s <= R; ++s) {  // the nodes ending at the last leaf, up to stage R
        const int h = 1 << (s - 1), pos = T - (1 << s);
        ps ^= (ps >> h) & (((1u << h) - 1u) << pos);
    }
}

template <int L, int V, int FM>
__global__ __launch_bounds__(64)
#if PL_SCL_WPE > 0
__attribute__((amdgpu_waves_per_eu(PL_SCL_WPE)))
#endif
void scl_tree_kernel(const float* __restrict__ llr, int64_t bs, void* __restrict__ out,
                                                      int out_kind, double* __restrict__ out_pm,
                                                      const uint32_t* __restrict__ frozen_words,
                                                      const int32_t* __restrict__ info_pos, int n, int S, int k,
                                                      double lmax, int crc_deg, uint32_t crc_g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Lay y = make_layout(n, S, L, V);
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    St t;
    t.A = reinterpret_cast<double*>(smem + y.off_A);
    t.ch = reinterpret_cast<float*>(smem + y.off_ch);
    t.beta = reinterpret_cast<uint32_t*>(smem + y.off_beta);
    t.sptr = smem + y.off_sptr;
    t.org_s = reinterpret_cast<int*>(smem + y.off_org);
    t.ps_s = reinterpret_cast<uint32_t*>(smem + y.off_ps);
    t.n = n;
    t.S = S;
    t.W = y.W;
    t.SS = y.SS;
    t.per = y.per;
    t.lmax = lmax;
    double* pm_s = reinterpret_cast<double*>(smem + y.off_pm);
    int* fail_s = reinterpret_cast<int*>(smem + y.off_fail);

    {
        const float4* x4 = reinterpret_cast<const float4*>(llr + b * n);
        float4* c4 = reinterpret_cast<float4*>(t.ch);
        for (int i = lane; i < n / 4; i += 64) {
            const float4 v = x4[i];
            c4[i] = make_float4(-1.0f * v.x, -1.0f * v.y, -1.0f * v.z, -1.0f * v.w);  // polar_scl.py:219
        }
    }
    for (int i = lane; i < L * y.W; i += 64) t.beta[i] = 0u;
    for (int i = lane; i < L * (S + 1); i += 64) t.sptr[i] = (uint8_t)(i / (S + 1));
    if (S == R)  // the whole tree is one lane-local subtree: its input is the channel, as fp64
        for (int i = lane; i < T; i += 64) t.A[i] = (double)t.ch[i];
    __syncthreads();

    double pm = (lane & (L - 1)) == 0 ? 0.0 : lmax;  // :192-194 ([0, 30 x (L-1)] per half)
    const int nsub = n >> R;
    for (int q = 0; q < nsub; ++q) {
        const int i0 = q << R;
        // input of the stage-R node at i0: g of the node that ends the finished left sibling,
        // then f down to stage R (stored stages only; virtual ones are recomputed on read)
        if (q == 0) {
            for (int s = S; s > R; --s)
                if (s - 1 <= t.SS) node_fg<L, V, FM>(t, s, 0, false, lane);
        } else {
            const int tz = __builtin_ctz(i0);
            if (tz <= t.SS) node_fg<L, V, FM>(t, tz + 1, i0 & ~((2 << tz) - 1), true, lane);
            for (int s = tz; s > R; --s)
                if (s - 1 <= t.SS) node_fg<L, V, FM>(t, s, i0, false, lane);
        }
        int org;
        uint32_t ps;
        subtree<L, FM>(t, i0, frozen_words[i0 >> 5] >> (i0 & 31), pm, org, ps, lane);
        // re-point the upper-tree state of every path to its origin's, then store the
        // subtree's partial sums: partial-sum words before i0 and stage owners R..SS
        if (lane < L) {
            t.org_s[lane] = org;
            t.ps_s[lane] = ps;
        }
        __syncthreads();
        const int w_i = i0 >> 5, w_lim = (i0 + 31) >> 5, off = i0 & 31;
        constexpr int RB = (L * 32 + 63) / 64;  // <= L*W/64 words per lane (n <= 1024)
        uint32_t vb[RB];
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            const int idx = r * 64 + lane;
            const int np = idx >> 5, w = idx & 31;
            if (np < L && w < w_lim) vb[r] = t.beta[t.org_s[np] * y.W + w];
        }
        constexpr int RS = (L * 11 + 63) / 64;
        uint8_t vs[RS];
        const int S1 = S + 1;
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            const int idx = r * 64 + lane;
            if (idx < L * S1) vs[r] = t.sptr[t.org_s[idx / S1] * S1 + idx % S1];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            const int idx = r * 64 + lane;
            const int np = idx >> 5, w = idx & 31;
            if (np < L && w < w_lim) t.beta[np * y.W + w] = vb[r];
        }
#pragma unroll
        for (int r = 0; r < RS; ++r) {
            const int idx = r * 64 + lane;
            if (idx < L * S1) t.sptr[idx] = vs[r];
        }
        if (T < 32 && off != 0) __syncthreads();  // the word's low part was just copied
        if (lane < L) {
            uint32_t* bw = t.beta + lane * y.W + w_i;
            *bw = off == 0 ? ps : ((*bw & ((1u << off) - 1u)) | (ps << off));
        }
        __syncthreads();
        // nodes above R that end with this subtree
        const int nxt = i0 + T;
        const int top = nxt < n ? __builtin_ctz(nxt) : S;
        for (int s = R + 1; s <= top; ++s) combine_upper<L>(t, s, nxt - (1 << s), lane);
    }
    if (lane < L) pm_s[lane] = pm;

    // u = x G_n per path (x = the root's partial sums): in-word spans, then word spans
    for (int idx = lane; idx < L * y.W; idx += 64) {
        uint32_t w = t.beta[idx];
        w ^= (w >> 1) & 0x55555555u;
        w ^= (w >> 2) & 0x33333333u;
        w ^= (w >> 4) & 0x0f0f0f0fu;
        w ^= (w >> 8) & 0x00ff00ffu;
        w ^= (w >> 16) & 0x0000ffffu;
        t.beta[idx] = w;
    }
    __syncthreads();
    for (int m = 1; m < y.W; m <<= 1) {
        for (int idx = lane; idx < L * y.W; idx += 64)
            if ((idx & m) == 0) t.beta[idx] ^= t.beta[idx + m];
        __syncthreads();
    }

    // CRC check per path (my_sn dec.py:507-518), final stable sort of the 2L logical rows
    // (row r < L = state r, row r >= L its copy), penalty per failing row, first argmin (:224)
    if (lane < L) {
        int f = 0;
        if (crc_deg > 0) {
            const uint32_t* U = t.beta + lane * y.W;
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
        fail_s[lane] = f;
    }
    __syncthreads();
    int best = 0;
    {
        int row[64];
        for (int r = 0; r < 2 * L; ++r) row[r] = r;
        for (int a = 1; a < 2 * L; ++a) {
            const int v = row[a];
            int c = a - 1;
            while (c >= 0 && pm_s[row[c] % L] > pm_s[v % L]) {
                row[c + 1] = row[c];
                --c;
            }
            row[c + 1] = v;
        }
        double bestv = 0.0;
        for (int r = 0; r < 2 * L; ++r) {
            const int p = row[r] % L;
            const double v = pm_s[p] + (fail_s[p] ? 30.0 * (double)k : 0.0);
            if (out_pm != nullptr && lane == 0) out_pm[b * 2 * L + r] = v;
            if (r == 0 || v < bestv) {
                best = p;
                bestv = v;
            }
        }
    }
    const uint32_t* U = t.beta + best * y.W;
    for (int m = lane; m < k; m += 64) {
        const int pos = info_pos[m];
        const uint32_t bit = (U[pos >> 5] >> (pos & 31)) & 1u;
        if (out_kind == PL_OUT_F32) static_cast<float*>(out)[b * k + m] = bit ? 1.0f : 0.0f;
        else static_cast<uint8_t*>(out)[b * k + m] = (uint8_t)bit;
    }
}

}  // namespace

// Instantiations are split over translation units, one per list size (the build compiles this
// file once per PL_SCL_TREE_L in parallel, plus once with PL_SCL_TREE_DISPATCH for the launcher).
namespace pl {
template <int L>
const void* scl_tree_fn(int v, bool exact);
}

#ifdef PL_SCL_TREE_L
namespace pl {
template <>
const void* scl_tree_fn<PL_SCL_TREE_L>(int v, bool exact) {
    constexpr int L = PL_SCL_TREE_L;
#define PL_FM(V) (exact ? (const void*)scl_tree_kernel<L, V, 1> : (const void*)scl_tree_kernel<L, V, 0>)
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
    int vmax = 3;
    if (const char* e = getenv("PL_SCL_VIRTUAL")) vmax = atoi(e);
    int v = S - 1 - R;
    if (v > vmax) v = vmax;
    return v < 0 ? 0 : v;
}
}  // namespace

namespace pl {

// Eligible plans: 2 <= L <= 32, 32 <= n <= 1024, no fast-SCL pruning.
bool scl_tree_eligible(const pl_plan* p) {
    if (p->flags & (PL_PLAN_FAST_SCL | PL_PLAN_GENERIC)) return false;
    if (const char* e = getenv("PL_SCL_TREE"))
        if (e[0] == '0') return false;
    return p->list_size >= 2 && p->list_size <= 32 && p->log_n >= 5 && p->log_n <= 10;
}

int launch_scl_tree(const pl_plan* p, const float* llr, int64_t bs, void* out, int out_kind, double* out_pm,
                    hipStream_t st) {
    if (bs == 0) return PL_OK;
    if (bs > 0x7fffffffLL) {
        set_error("SCL decode: batch too large for one launch");
        return PL_EINVAL;
    }
    const int S = p->log_n, L = p->list_size, V = pick_v(S);
    const bool exact = p->f_mode == PL_F_EXACT;
    const void* fn = nullptr;
#ifdef PL_SCL_VARIANT_ONLY_L8  // development variant libraries (tools/scl_variants.py)
    if (L != 8) {
        set_error("variant library: L = 8 only");
        return PL_ENOTSUP;
    }
    fn = scl_tree_fn<8>(V, exact);
#else
    switch (L) {
        case 2: fn = scl_tree_fn<2>(V, exact); break;
        case 4: fn = scl_tree_fn<4>(V, exact); break;
        case 8: fn = scl_tree_fn<8>(V, exact); break;
        case 16: fn = scl_tree_fn<16>(V, exact); break;
        default: fn = scl_tree_fn<32>(V, exact); break;
    }
#endif
    const Lay y = make_layout(p->n, S, L, V);
    if (y.bytes > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, y.bytes);
        if (e != hipSuccess) return check_hip(e, "SCL decode: LDS attribute");
    }
    int n = p->n, k = p->k, cdeg = p->crc_deg;
    double lmax = (double)p->llr_max;
    uint32_t cg = p->crc_g;
    const uint32_t* fw = p->d_frozen_words;
    const int32_t* ip = p->d_info_pos;
    void* args[] = {(void*)&llr, (void*)&bs, (void*)&out, (void*)&out_kind, (void*)&out_pm, (void*)&fw,
                    (void*)&ip, (void*)&n, (void*)&S, (void*)&k, (void*)&lmax, (void*)&cdeg, (void*)&cg};
    hipError_t e = hipLaunchKernel(fn, dim3((unsigned)bs), dim3(64), args, y.bytes, st);
    if (e != hipSuccess) return check_hip(e, "SCL decode launch (subtree kernel)");
    return check_hip(hipGetLastError(), "SCL decode launch (subtree kernel)");
}

}  // namespace pl
#endif  // PL_SCL_TREE_DISPATCH
