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
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/polar_mi355x.h"
#include "plan.h"

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
    y.off_alpha = o; o = align16(o + L * (n / 2 > 0 ? n / 2 : 1) * 8);
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
__device__ __forceinline__ double g_op(double x, double y, uint32_t bit) {  // :107-108
    return (bit ? -x : x) + y;
}
__device__ __forceinline__ uint32_t getbit(const uint32_t* w, int pos) { return (w[pos >> 5] >> (pos & 31)) & 1u; }

// LLR j of the stage-s node at position pos for path p.
__device__ __forceinline__ double read_alpha(const St& t, int p, int s, int pos, int j) {
    if (s == t.S) return (double)t.ch[j];
    if (s == t.S - 1) {
        const double x = (double)t.ch[j], y = (double)t.ch[j + t.half];
        if (pos == 0) return f_ms(x, y, t.lmax);
        return g_op(x, y, getbit(t.beta + p * t.W, j));
    }
    const int owner = t.sptr[p * t.S + s];
    return t.A[owner * t.half + (1 << s) + j];
}

// f (is_g = false) or g at the stage-s node at position pos, for every path: writes stage s-1.
__device__ void node_fg(St& t, int s, int pos, bool is_g, int lane) {
    const int ls = s - 1, h = 1 << ls;
    const int total = t.L * h;
    for (int idx = lane; idx < total; idx += 64) {
        const int p = idx >> ls, j = idx & (h - 1);
        const double x = read_alpha(t, p, s, pos, j);
        const double y = read_alpha(t, p, s, pos, j + h);
        const double r = is_g ? g_op(x, y, getbit(t.beta + p * t.W, pos + j)) : f_ms(x, y, t.lmax);
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

// Leaf i: path-metric update for every path; at information leaves the 2L-candidate selection
// and the fork (inherit parent's pointers, partial sums and decisions, then set bit i).
__device__ void leaf(St& t, int i, bool info, int lane) {
    double pen0 = 0.0, pen1 = 0.0, pmv = 0.0;
    if (lane < t.L) {
        double l = read_alpha(t, lane, 0, i, 0);
        l = fmax(fmin(l, t.lmax), -t.lmax);
        pmv = t.pm[lane];
        pen0 = log(1.0 + exp(-(1.0 * l)));
        pen1 = info ? log(1.0 + exp(-(-1.0 * l))) : 0.0;
    }
    if (!info) {
        if (lane < t.L) t.pm[lane] = pmv + pen0;
        __syncthreads();
        return;
    }
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
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int idx = r * 64 + lane;
        if (idx < per) {
            const int np = idx / W, w = idx - np * W;
            uint32_t b = vb[r], uu = vu[r];
            if (w == (i >> 5) && t.fbit[np]) {
                b |= 1u << (i & 31);
                uu |= 1u << (i & 31);
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

template <int OUTK>
__global__ __launch_bounds__(64) void scl_decode_kernel(const float* __restrict__ llr, int64_t bs, void* __restrict__ out,
                                                         double* __restrict__ out_pm,
                                                         const uint32_t* __restrict__ frozen_words,
                                                         const int32_t* __restrict__ info_pos, int n, int log_n, int L,
                                                         int k, double lmax) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Lay y = make_layout(n, log_n, L);
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
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

    const int S = log_n;
    for (int i = 0; i < n; ++i) {
        int start;
        if (i == 0) {
            start = S - 1;  // root f is virtual (stage S-1 recomputed from the channel)
        } else {
            const int tz = __builtin_ctz(i);
            for (int s = 1; s <= tz; ++s) combine(t, s, (i - 1) & ~((1 << s) - 1), lane);
            if (tz + 1 < S) node_fg(t, tz + 1, i & ~((1 << (tz + 1)) - 1), true, lane);
            start = tz;
        }
        for (int s = start; s >= 1; --s) node_fg(t, s, i & ~((1 << s) - 1), false, lane);
        const bool info = ((frozen_words[i >> 5] >> (i & 31)) & 1u) == 0u;
        leaf(t, i, info, lane);
    }

    // best path: first minimum over states in slot order (sorted msg_pm[:, 0], polar_scl.py:224)
    int best = 0;
    for (int p = 1; p < L; ++p)
        if (t.pm[p] < t.pm[best]) best = p;
    const uint32_t* U = t.u + best * y.W;
    for (int m = lane; m < k; m += 64) {
        const int pos = info_pos[m];
        const uint32_t bit = (U[pos >> 5] >> (pos & 31)) & 1u;
        if constexpr (OUTK == PL_OUT_F32) static_cast<float*>(out)[b * k + m] = bit ? 1.0f : 0.0f;
        else static_cast<uint8_t*>(out)[b * k + m] = (uint8_t)bit;
    }
    if (out_pm != nullptr && lane == 0) {
        // final sorted msg_pm: every surviving state appears twice (rows j and j+L)
        double v[32];
        for (int p = 0; p < L; ++p) v[p] = t.pm[p];
        for (int a = 1; a < L; ++a) {
            const double key = v[a];
            int c = a - 1;
            while (c >= 0 && v[c] > key) {
                v[c + 1] = v[c];
                --c;
            }
            v[c + 1] = key;
        }
        for (int p = 0; p < L; ++p) {
            out_pm[b * 2 * L + 2 * p] = v[p];
            out_pm[b * 2 * L + 2 * p + 1] = v[p];
        }
    }
}

}  // namespace

namespace pl {
size_t scl_workspace_size(const pl_plan*, int64_t) { return 0; }

int launch_scl(const pl_plan* p, const float* llr, int64_t bs, void* out, int out_kind, double* out_pm, void*, size_t,
               hipStream_t st) {
    if (bs == 0) return PL_OK;
    if (p->n > 1024) {
        set_error("SCL decode: n must be <= 1024");
        return PL_ENOTSUP;
    }
    const Lay y = make_layout(p->n, p->log_n, p->list_size);
    if (y.bytes > 160 * 1024) {
        set_error("SCL decode: n * list_size too large for LDS");
        return PL_ENOTSUP;
    }
    if (y.bytes > 64 * 1024) {
        hipError_t e = out_kind == PL_OUT_F32
            ? hipFuncSetAttribute((const void*)scl_decode_kernel<PL_OUT_F32>, hipFuncAttributeMaxDynamicSharedMemorySize, y.bytes)
            : hipFuncSetAttribute((const void*)scl_decode_kernel<PL_OUT_U8>, hipFuncAttributeMaxDynamicSharedMemorySize, y.bytes);
        if (e != hipSuccess) return check_hip(e, "SCL decode: LDS attribute");
    }
    if (out_kind == PL_OUT_F32)
        hipLaunchKernelGGL(scl_decode_kernel<PL_OUT_F32>, dim3((unsigned)bs), dim3(64), y.bytes, st, llr, bs, out, out_pm,
                           p->d_frozen_words, p->d_info_pos, p->n, p->log_n, p->list_size, p->k, (double)p->llr_max);
    else
        hipLaunchKernelGGL(scl_decode_kernel<PL_OUT_U8>, dim3((unsigned)bs), dim3(64), y.bytes, st, llr, bs, out, out_pm,
                           p->d_frozen_words, p->d_info_pos, p->n, p->log_n, p->list_size, p->k, (double)p->llr_max);
    return check_hip(hipGetLastError(), "SCL decode launch");
}
}  // namespace pl
