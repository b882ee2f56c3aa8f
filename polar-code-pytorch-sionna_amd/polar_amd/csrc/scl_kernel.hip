// scl_kernel.hip -- successive-cancellation LIST (SCL) polar decoder for gfx950 (MI355X).
//
// Reference semantics: x_run_sn_polar/polar/polar_scl.py (SCL_Dec): min-sum f on clipped LLRs
// (:93-106), g (:107-108), per-leaf path-metric update pm += log(1+exp(-(1-2u)*clip(llr)))
// (:69-85), at information leaves a sort of the 2L candidates (:86-92) and duplication of the
// best L (:109-120), dead paths initialised at +30 (:193-194), final argmin (:224).  The
// reference keeps every state in float64; so does this kernel (LLRs and path metrics), which
// makes every f/g value identical and the path metrics equal up to the last-ulp differences of
// exp/log.  Tie order: the reference's np.argsort is unstable (host-dependent); this kernel
// sorts by the stable (metric, candidate index) order.
//
// Equivalence used: the reference's 2L physical rows always hold two identical copies of L
// states (row j and j+L), so L states suffice: candidate c < L is (state c, u=0), c >= L is
// (state c-L, u=1), exactly the reference's logical order after _update_single_bit_np.
//
// Layout: one wave64 per codeword (no barriers are real: a single-wave workgroup), all state in
// LDS: per path the stage buffers s = 0..S-2 (fp64, n/2 per path) addressed through per-path
// per-stage pointers (lazy copy: a forked path inherits its parent's pointers and only
// writes its own buffers when it descends), bit-packed partial sums and decided bits (copied at
// each fork, n/32 words each), the fp32 channel (stage S).  Stage S-1 is never stored: it is
// recomputed from the channel (f for the left half, g with the path's own partial sums for the
// right half), which halves the footprint (about 38 KB per codeword at n=1024, L=8).
//
// my_sn variant (my_sn/fec/polar/dec.py SCL_Dec :158-537), selected per plan:
//   FM = 1    exact boxplus f on clipped inputs, float64 (dec.py:330-339)
//   FAST      fast-SCL tree pruning (dec.py:367-376): a rate-0 node adds, per path, the sum of
//             log(1+exp(-clip(llr))) over the node (:269-280); a repetition node forks once on
//             the two node sums (:281-306).  Sums follow numpy's pairwise order (np.sum over the
//             last axis) so path metrics match to rounding.
//   CRC       CRC-aided pick (:507-518): every path failing the CRC gets +llr_max*k, first argmin; the
//             penalty also lands in the returned metrics (it aliases msg_pm in the reference).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/polar_mi355x.h"
#include "plan.h"
#include "softplus.h"

#include <string>

namespace {

struct Lay {
    int n, S, L, W;
    int off_alpha, off_ch, off_beta, off_u, off_pm, off_fork_par, off_fork_bit, off_fork_pm, off_sptr, bytes;
};

__host__ __device__ inline int align16(int x) { return (x + 15) & ~15; }

__host__ __device__ inline Lay make_layout(int n, int log_n, int L) {
    Lay y;
    y.n = n;
    y.S = log_n;
    y.L = L;
    y.W = n >= 32 ? n / 32 : 1;
    int o = 0;
    // L stage regions of n/2 doubles; at least n doubles, the staging area of the node terms of a
    // pruned root (node_softplus_sums, one path at a time)
    const int na = L * (n / 2 > 0 ? n / 2 : 1);
    y.off_alpha = o; o = align16(o + (na > n ? na : n) * 8);
    y.off_ch = o; o = align16(o + n * 4);
    y.off_beta = o; o = align16(o + L * y.W * 4);
    y.off_u = o; o = align16(o + L * y.W * 4);
    y.off_pm = o; o = align16(o + L * 8);
    y.off_fork_pm = o; o = align16(o + L * 8);
    y.off_fork_par = o; o = align16(o + L * 4);
    y.off_fork_bit = o; o = align16(o + L * 4);
    y.off_sptr = o; o = align16(o + L * (log_n > 0 ? log_n : 1));
    y.bytes = o;
    return y;
}

struct St {
    double* A;        // [L][n/2]   stage s (s <= S-2) of path p at A[p*(n/2) + 2^s + j]
    float* ch;        // [n]        negated channel LLRs (stage S)
    uint32_t* beta;   // [L][W]     partial sums by absolute position
    uint32_t* u;      // [L][W]     decided bits by absolute position
    double* pm;       // [L]
    double* fpm;      // [L]        fork table: new metric
    int* fpar;        // [L]        fork table: parent state
    int* fbit;        // [L]        fork table: decided bit
    uint8_t* sptr;    // [L][S]     stage-buffer owner
    int n, S, L, W, half;
    double lmax;
};

__device__ __forceinline__ double f_ms(double x, double y, double lmax) {  // polar_scl.py:93-106
    const double m = fmin(fmin(fabs(x), fabs(y)), lmax);
    const bool neg = (__double_as_longlong(x) ^ __double_as_longlong(y)) < 0;
    return neg ? -m : m;
}
// Diagnostic macros (timing ablations with WRONG results) exist only in development builds.
#ifndef PL_DEV
#define PL_DEV 0
#endif
#if !PL_DEV && defined(PL_SCL_DIAG_FMS_ALL) && PL_SCL_DIAG_FMS_ALL
#error "PL_SCL_DIAG_FMS_ALL gives wrong results: development builds (-DPL_DEV=1) only"
#endif
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
template <int FM>
__device__ __forceinline__ double f_op(double x, double y, double lmax) {
    if constexpr (FM == 0) return f_ms(x, y, lmax);
    else return f_ex(x, y, lmax);
}
__device__ __forceinline__ double g_op(double x, double y, uint32_t bit) {  // :107-108
    return (bit ? -x : x) + y;
}
__device__ __forceinline__ uint32_t getbit(const uint32_t* w, int pos) { return (w[pos >> 5] >> (pos & 31)) & 1u; }

// LLR j of the stage-s node at position pos for path p.
template <int FM>
__device__ __forceinline__ double read_alpha(const St& t, int p, int s, int pos, int j) {
    if (s == t.S) return (double)t.ch[j];
    if (s == t.S - 1) {
        const double x = (double)t.ch[j], y = (double)t.ch[j + t.half];
        if (pos == 0) return f_op<FM>(x, y, t.lmax);
        return g_op(x, y, getbit(t.beta + p * t.W, j));
    }
    const int owner = t.sptr[p * t.S + s];
    return t.A[owner * t.half + (1 << s) + j];
}

// f (is_g = false) or g at the stage-s node at position pos, for every path: writes stage s-1.
template <int FM>
__device__ void node_fg(St& t, int s, int pos, bool is_g, int lane) {
    const int ls = s - 1, h = 1 << ls;
    const int total = t.L * h;
    for (int idx = lane; idx < total; idx += 64) {
        const int p = idx >> ls, j = idx & (h - 1);
        const double x = read_alpha<FM>(t, p, s, pos, j);
        const double y = read_alpha<FM>(t, p, s, pos, j + h);
        const double r = is_g ? g_op(x, y, getbit(t.beta + p * t.W, pos + j)) : f_op<FM>(x, y, t.lmax);
        t.A[p * t.half + h + j] = r;
    }
    __syncthreads();
    if (lane < t.L) t.sptr[lane * t.S + ls] = (uint8_t)lane;
    __syncthreads();
}

// beta[pos, pos+h) ^= beta[pos+h, pos+2h) for every path (polar_scl.py:147-153, in place).
__device__ void combine(St& t, int s, int pos, int lane) {
    const int h = 1 << (s - 1);
    if (h >= 32) {
        const int hw = h >> 5, w0 = pos >> 5;
        for (int idx = lane; idx < t.L * hw; idx += 64) {
            const int p = idx / hw, w = idx - p * hw;
            uint32_t* b = t.beta + p * t.W;
            b[w0 + w] ^= b[w0 + hw + w];
        }
    } else if (lane < t.L) {
        uint32_t* b = t.beta + lane * t.W + (pos >> 5);
        const int sh = pos & 31;
        const uint32_t m = (h == 32 ? 0xffffffffu : ((1u << h) - 1u)) << sh;
        *b ^= (*b >> h) & m;
    }
    __syncthreads();
}

__device__ __forceinline__ double shfl_d(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __shfl((int)(b & 0xffffffffLL), src, 64);
    const int hi = __shfl((int)(b >> 32), src, 64);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// 2L-candidate selection and fork (polar_scl.py:86-92 + :109-120): lanes < L hold pm + pen0
// (candidate c = state c, u = 0) and pen1 (candidate L + c = state c, u = 1).  Survivors take
// their parent's partial sums, decisions and stage pointers; a fork on a node [a, a+len) sets
// the node's partial sums to the chosen bit (len = 1: a leaf) and its last decision.
__device__ void select_fork(St& t, double pmv, double pen0, double pen1, int a, int len, int lane) {
    const int L = t.L;
    // candidate c: c < L -> (state c, u=0), c >= L -> (state c-L, u=1)
    const int src = lane < L ? lane : (lane - L);
    const double p_src = shfl_d(pmv, src & 63);
    const double q_src = shfl_d(pen1, src & 63);
    const double cand = lane < L ? (pmv + pen0) : (p_src + q_src);
    int rank = 0;
    for (int c = 0; c < 2 * L; ++c) {
        const double v = shfl_d(cand, c);
        rank += (v < cand) || (v == cand && c < lane);
    }
    if (lane < 2 * L && rank < L) {
        t.fpar[rank] = lane < L ? lane : lane - L;
        t.fbit[rank] = lane < L ? 0 : 1;
        t.fpm[rank] = cand;
    }
    __syncthreads();
    // gather the parents' partial sums, decisions and stage pointers, then scatter (all reads
    // complete before any write: several new states may share one parent)
    const int W = t.W, S = t.S;
    const int per = L * W;  // <= 32 * 32 = 1024 words -> <= 16 per lane
    constexpr int R = 16;
    uint32_t vb[R], vu[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int idx = r * 64 + lane;
        if (idx < per) {
            const int np = idx / W, w = idx - np * W;
            const int par = t.fpar[np];
            vb[r] = t.beta[par * W + w];
            vu[r] = t.u[par * W + w];
        }
    }
    constexpr int RS = 8;  // L * S <= 32 * 10 = 320 bytes -> <= 5 per lane
    uint8_t sp[RS];
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        const int idx = r * 64 + lane;
        if (idx < L * S) sp[r] = t.sptr[t.fpar[idx / S] * S + idx % S];
    }
    __syncthreads();
    const int last = a + len - 1;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int idx = r * 64 + lane;
        if (idx < per) {
            const int np = idx / W, w = idx - np * W;
            uint32_t b = vb[r], uu = vu[r];
            if (t.fbit[np]) {
                // node bits [a, a+len) inside word w
                const int lo = a > (w << 5) ? a - (w << 5) : 0;
                const int hi = (a + len) < ((w + 1) << 5) ? (a + len) - (w << 5) : 32;
                if (lo < hi) b |= (hi - lo == 32 ? 0xffffffffu : (((1u << (hi - lo)) - 1u) << lo));
                if (w == (last >> 5)) uu |= 1u << (last & 31);
            }
            t.beta[np * W + w] = b;
            t.u[np * W + w] = uu;
        }
    }
#pragma unroll
    for (int r = 0; r < RS; ++r) {
        const int idx = r * 64 + lane;
        if (idx < L * S) t.sptr[idx] = sp[r];
    }
    if (lane < L) t.pm[lane] = t.fpm[lane];
    __syncthreads();
}

// Leaf i: path-metric update for every path (polar_scl.py:69-85); at information leaves the
// 2L-candidate selection and fork.
template <int FM>
__device__ void leaf(St& t, int i, bool info, int lane) {
    double pen0 = 0.0, pen1 = 0.0, pmv = 0.0;
    if (lane < t.L) {
        double l = read_alpha<FM>(t, lane, 0, i, 0);
        l = fmax(fmin(l, t.lmax), -t.lmax);
        pmv = t.pm[lane];
        pen0 = pl::softplus_pm(-(1.0 * l));
        pen1 = info ? pl::softplus_pm(-(-1.0 * l)) : 0.0;
    }
    if (!info) {
        if (lane < t.L) t.pm[lane] = pmv + pen0;
        __syncthreads();
        return;
    }
    select_fork(t, pmv, pen0, pen1, i, 1, lane);
}

// Terms log(1+exp(-clip(sg*llr))) of the stage-s node at pos, for paths p0 .. p0+np-1, written
// to base[q * stride + j] (q = p - p0): every lane of the wave computes terms, not one lane per
// path.  The staging area [0, 2^s) of a path's own stage region holds only stages below s, dead
// while the node is pruned.
template <int FM>
__device__ void node_terms(St& t, int s, int pos, double sg, int p0, int np, double* base, int stride, int lane) {
    const int len = 1 << s;
    for (int idx = lane; idx < np * len; idx += 64) {
        const int q = idx >> s, j = idx & (len - 1);
        const double l = fmax(fmin(sg * read_alpha<FM>(t, p0 + q, s, pos, j), t.lmax), -t.lmax);
        base[q * stride + j] = pl::softplus_pm(-l);
    }
    __syncthreads();
}

// Sum of T[0, len) in numpy's pairwise order (np.sum over the last axis: < 8 terms sequentially
// from 0; <= 128 terms with 8 interleaved partial sums combined ((0+1)+(2+3))+((4+5)+(6+7));
// larger halves recursively -- len is a power of two, so blocks of 128 combined pairwise).
__device__ double pairwise_sum(const double* T, int len) {
    if (len < 8) {
        double r = 0.0;
        for (int j = 0; j < len; ++j) r += T[j];
        return r;
    }
    const int blk = len < 128 ? len : 128;
    double lvl[16];
    int nl = 0;
    const int nb = len / blk;  // <= 16 blocks at n <= 2048
    for (int b = 0; b < nb; ++b) {
        const double* a = T + b * blk;
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        for (int i = 8; i < blk; i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        lvl[nl++] = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    }
    while (nl > 1) {
        for (int i = 0; i < nl / 2; ++i) lvl[i] = lvl[2 * i] + lvl[2 * i + 1];
        nl /= 2;
    }
    return lvl[0];
}

// Node sum of every path into pen (lane p < L gets path p's sum).  A node larger than a path's
// region (the root of a rate-0 / repetition code) goes one path at a time through A[0, n): no
// stage buffer is live then.
template <int FM>
__device__ double node_softplus_sums(St& t, int s, int pos, double sg, int lane) {
    const int len = 1 << s;
    double pen = 0.0;
    if (len <= t.half) {
        node_terms<FM>(t, s, pos, sg, 0, t.L, t.A, t.half, lane);
        if (lane < t.L) pen = pairwise_sum(t.A + lane * t.half, len);
        __syncthreads();
    } else {
        for (int p = 0; p < t.L; ++p) {
            node_terms<FM>(t, s, pos, sg, p, 1, t.A, 0, lane);
            if (lane == p) pen = pairwise_sum(t.A, len);
            __syncthreads();
        }
    }
    return pen;
}

// Pruned node (fast-SCL).  Rate-0: pm += node sum (dec.py:269-280).  Repetition: candidates
// pm + sum(u=0) / pm + sum(u=1) -> selection and fork on the whole node (dec.py:281-306).
template <int FM>
__device__ void pruned_node(St& t, int s, int pos, bool rep, int lane) {
    const double pmv = lane < t.L ? t.pm[lane] : 0.0;
    const double pen0 = node_softplus_sums<FM>(t, s, pos, 1.0, lane);
    const double pen1 = rep ? node_softplus_sums<FM>(t, s, pos, -1.0, lane) : 0.0;
    if (!rep) {
        if (lane < t.L) t.pm[lane] = pmv + pen0;
        __syncthreads();
        return;
    }
    select_fork(t, pmv, pen0, pen1, pos, 1 << s, lane);
}

// node type flags of the plan (capi.cpp): bit OFF(s) + (pos >> s), OFF(s) = n - (n >> (s-1))
__device__ __forceinline__ bool type_bit(const uint32_t* __restrict__ words, int n, int s, int pos) {
    const int bit = n - (n >> (s - 1)) + (pos >> s);
    return (words[bit >> 5] >> (bit & 31)) & 1u;
}

template <int OUTK, int FM, bool FAST>
__global__ __launch_bounds__(64) void scl_decode_kernel(const float* __restrict__ llr, int64_t bs, void* __restrict__ out,
                                                         double* __restrict__ out_pm,
                                                         const uint32_t* __restrict__ frozen_words,
                                                         const uint32_t* __restrict__ r0_words,
                                                         const uint32_t* __restrict__ rep_words,
                                                         const int32_t* __restrict__ info_pos, int n, int log_n, int L,
                                                         int k, double lmax, int crc_deg, uint32_t crc_g) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Lay y = make_layout(n, log_n, L);
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    pl::sp_load_tables(lane, 64);  // the penalty's log table (softplus.h, PL_SP_FORM 3)
    pl::fex_load_table<FM == 1>(lane);  // the exact f's 2^(j/64) table (softplus.h fex_exp)
    St t;
    t.A = reinterpret_cast<double*>(smem + y.off_alpha);
    t.ch = reinterpret_cast<float*>(smem + y.off_ch);
    t.beta = reinterpret_cast<uint32_t*>(smem + y.off_beta);
    t.u = reinterpret_cast<uint32_t*>(smem + y.off_u);
    t.pm = reinterpret_cast<double*>(smem + y.off_pm);
    t.fpm = reinterpret_cast<double*>(smem + y.off_fork_pm);
    t.fpar = reinterpret_cast<int*>(smem + y.off_fork_par);
    t.fbit = reinterpret_cast<int*>(smem + y.off_fork_bit);
    t.sptr = smem + y.off_sptr;
    t.n = n;
    t.S = log_n;
    t.L = L;
    t.W = y.W;
    t.half = n / 2 > 0 ? n / 2 : 1;
    t.lmax = lmax;

    const float* x = llr + b * n;
    for (int i = lane; i < n; i += 64) t.ch[i] = -1.0f * x[i];  // polar_scl.py:219
    for (int i = lane; i < L * y.W; i += 64) {
        t.beta[i] = 0u;
        t.u[i] = 0u;
    }
    for (int i = lane; i < L * log_n; i += 64) t.sptr[i] = (uint8_t)(i / log_n);
    if (lane < L) t.pm[lane] = lane == 0 ? 0.0 : lmax;  // :192-194 ([0, 30 x (L-1)] per half)
    __syncthreads();

    // Tree walk in leaf order.  At leaf (or pruned node) start i: combine the nodes that ended
    // at i-1 above the last finished node (stage `done`), compute the input of the node that
    // starts at i (g of its parent), then descend with f, pruning rate-0 / repetition nodes.
    const int S = log_n;
    int i = 0, done = 0;
    while (i < n) {
        int start;
        if (i == 0) {
            start = S;  // the root's input is the channel; stage S-1 is virtual (read_alpha)
        } else {
            const int tz = __builtin_ctz(i);
            for (int s = done + 1; s <= tz; ++s) combine(t, s, (i - 1) & ~((1 << s) - 1), lane);
            if (tz + 1 < S) node_fg<FM>(t, tz + 1, i & ~((1 << (tz + 1)) - 1), true, lane);
            start = tz;
        }
        int s = start;
        bool pruned = false;
        for (; s >= 1; --s) {
            if constexpr (FAST) {
                if (type_bit(r0_words, n, s, i)) {
                    pruned_node<FM>(t, s, i, false, lane);
                    pruned = true;
                    break;
                }
                if (type_bit(rep_words, n, s, i)) {
                    pruned_node<FM>(t, s, i, true, lane);
                    pruned = true;
                    break;
                }
            }
            if (s < S) node_fg<FM>(t, s, i, false, lane);  // stage S-1 of the root is virtual
        }
        if (pruned) {
            done = s;
            i += 1 << s;
        } else {
            const bool info = ((frozen_words[i >> 5] >> (i & 31)) & 1u) == 0u;
            leaf<FM>(t, i, info, lane);
            done = 0;
            i += 1;
        }
    }

    // Final sort of the 2L logical rows (row r < L = state r, row r >= L its copy; stable by
    // pm), CRC penalty per failing row (my_sn dec.py:507-518), first argmin (:224 / :520).
    __shared__ int fail_s[32];
    if (lane < L) {
        int f = 0;
        if (crc_deg > 0) {
            const uint32_t* U = t.u + lane * y.W;
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
            while (c >= 0 && t.pm[row[c] % L] > t.pm[v % L]) {
                row[c + 1] = row[c];
                --c;
            }
            row[c + 1] = v;
        }
        double bestv = 0.0;
        for (int r = 0; r < 2 * L; ++r) {
            const int p = row[r] % L;
            const double v = t.pm[p] + (fail_s[p] ? t.lmax * (double)k : 0.0);
            if (out_pm != nullptr && lane == 0) out_pm[b * 2 * L + r] = v;
            if (r == 0 || v < bestv) {
                best = p;
                bestv = v;
            }
        }
    }
    const uint32_t* U = t.u + best * y.W;
    for (int m = lane; m < k; m += 64) {
        const int pos = info_pos[m];
        const uint32_t bit = (U[pos >> 5] >> (pos & 31)) & 1u;
        if constexpr (OUTK == PL_OUT_F32) static_cast<float*>(out)[b * k + m] = bit ? 1.0f : 0.0f;
        else static_cast<uint8_t*>(out)[b * k + m] = (uint8_t)bit;
    }
}

}  // namespace

namespace pl {
size_t scl_workspace_size(const pl_plan* p, int64_t bs) { return scl_tree_workspace_size(p, bs); }

// Limits of the generic kernel: its state is LDS-resident (one wave per codeword, <= 160 KiB)
// and a fork gathers the L * n/32 partial-sum and decision words in 16 registers per lane
// (select_fork: R = 16), and the L * log n stage owners in 8 (RS = 8).  At n = 2048 that is
// L <= 16 (147.6 KB of LDS at L = 16).  The subtree kernel covers 2 <= L <= 32 up to n = 1024.
bool scl_supported(const pl_plan* p) {
    if (scl_tree_eligible(p)) return true;
    const int L = p->list_size, W = p->n >= 32 ? p->n / 32 : 1;
    const Lay y = make_layout(p->n, p->log_n, L);
    if (L * W > 16 * 64 || L * p->log_n > 8 * 64 || y.bytes > 160 * 1024) {
        set_error("SCL decode: n = " + std::to_string(p->n) + " with list_size " + std::to_string(L) +
                  " is not supported (the list state must fit one CU's LDS: list_size <= 16 at n = 2048)");
        return false;
    }
    return true;
}

int launch_scl(const pl_plan* p, const float* llr, int64_t bs, void* out, int out_kind, double* out_pm, void* ws,
               size_t ws_bytes, hipStream_t st) {
    if (bs == 0) return PL_OK;
    if (scl_tree_eligible(p)) return launch_scl_tree(p, llr, bs, out, out_kind, out_pm, ws, ws_bytes, st);
    if (!scl_supported(p)) return PL_ENOTSUP;
    const Lay y = make_layout(p->n, p->log_n, p->list_size);
    const bool fast = (p->flags & PL_PLAN_FAST_SCL) != 0;
    const bool exact = p->f_mode == PL_F_EXACT;
    const void* fn = nullptr;
#define PL_SCL_PICK(O, F, P) if (out_kind == O && (exact ? 1 : 0) == F && fast == P) fn = (const void*)scl_decode_kernel<O, F, P>;
    PL_SCL_PICK(PL_OUT_F32, 0, false) PL_SCL_PICK(PL_OUT_F32, 0, true) PL_SCL_PICK(PL_OUT_F32, 1, false)
    PL_SCL_PICK(PL_OUT_F32, 1, true) PL_SCL_PICK(PL_OUT_U8, 0, false) PL_SCL_PICK(PL_OUT_U8, 0, true)
    PL_SCL_PICK(PL_OUT_U8, 1, false) PL_SCL_PICK(PL_OUT_U8, 1, true)
#undef PL_SCL_PICK
    if (y.bytes > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, y.bytes);
        if (e != hipSuccess) return check_hip(e, "SCL decode: LDS attribute");
    }
    const uint32_t* r0w = p->d_type_words;
    const uint32_t* repw = p->d_type_words + 2 * p->type_stride;
    const int32_t* ip = p->d_info_pos;
    int n = p->n, log_n = p->log_n, L = p->list_size, k = p->k, cdeg = p->crc_deg;
    double lmax = (double)p->llr_max;
    uint32_t cg = p->crc_g;
    const uint32_t* fw = p->d_frozen_words;
    void* args[] = {(void*)&llr, (void*)&bs, (void*)&out, (void*)&out_pm, (void*)&fw, (void*)&r0w, (void*)&repw,
                    (void*)&ip, (void*)&n, (void*)&log_n, (void*)&L, (void*)&k, (void*)&lmax, (void*)&cdeg, (void*)&cg};
    hipError_t e = hipLaunchKernel(fn, dim3((unsigned)bs), dim3(64), args, y.bytes, st);
    if (e != hipSuccess) return check_hip(e, "SCL decode launch");
    return check_hip(hipGetLastError(), "SCL decode launch");
}
}  // namespace pl
