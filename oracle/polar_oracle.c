/*
 * polar_oracle.c -- CPU restatement of the reference SC / SCL polar decoders.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker for the HIP decoders in
 * polar-code-pytorch-sionna_amd/ and the CPU baseline timed by bench.py.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The product path
 * never links or calls it.
 *
 * Pinned: the outputs of this file are checked bit-exactly against the tests/golden fixtures, which
 * tests/golden/make_golden.py generated from the reference itself (see tests/test_oracle.py).
 *
 * Restated reference functions (jaco267/polar-code-pytorch-sionna, /root/reference):
 *   orc_sc_decode   x_run_sn_polar/polar/polar_sc.py   SC_Dec (:33-133); f_mode=1 follows the
 *                   exact-boxplus f of my_sn/fec/polar/dec.py:33-46 instead of min-sum (:46).
 *   orc_scl_decode  x_run_sn_polar/polar/polar_scl.py  SCL_Dec (:49-234): 2L physical rows,
 *                   dec_pointer indirection, full-row path copies, float64 state.  One deliberate
 *                   deviation: np.argsort (:88) is unstable (AVX-512 sort, tie order is
 *                   host-dependent); this oracle uses the stable (pm, index) order.
 *   orc_scl_decode_lazy  the same decoder restated the way the GPU kernel runs it: L states,
 *                   per-stage LLR pointers (lazy copy), bit-packed partial sums.  Cross-checked
 *                   against orc_scl_decode in tests.
 *   orc_polar_encode  x_run_sn_polar/polar/enc.py:30-43 (c[:,info]=u; (c@G)%2) computed by the
 *                   XOR butterfly of my_sn/fec/polar/enc.py:85-96.
 *   orc_crc_encode / orc_crc_check  my_sn/fec/crc.py: CRCEncoder (:6-109, G-matrix form of the
 *                   5G polynomials :38-52) and CRCDecoder (:111-138), restated as the MSB-first
 *                   shift register (equal to the G-matrix form; pinned by tests/golden/crc.npz).
 *   orc_scl_decode_mysn  my_sn/fec/polar/dec.py SCL_Dec (:158-537): exact-boxplus f (:330-339),
 *                   fast-SCL rate-0 (:269-280) and repetition (:281-306) nodes with numpy's
 *                   pairwise summation order for the node sums, CRC-aided pick (:507-518).
 *                   Same stable tie order as orc_scl_decode.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define LLR_MAX 30.0f

static inline float clipf(float x) { return fminf(fmaxf(x, -LLR_MAX), LLR_MAX); }
static inline float clipf_l(float x, float l) { return fminf(fmaxf(x, -l), l); }
static inline float signf_t(float x) { return (float)((x > 0.0f) - (x < 0.0f)); } /* torch.sign */

/* f, polar_sc.py:33-48: min-sum is what runs (line 46 overrides the exact result). */
static inline float f_minsum(float x, float y, float l) {
    float xc = clipf_l(x, l), yc = clipf_l(y, l);
    return signf_t(xc) * signf_t(yc) * fminf(fabsf(xc), fabsf(yc));
}
/* f, my_sn/fec/polar/dec.py:33-46: exact log-domain boxplus on clipped inputs (fp32). */
static inline float f_exact(float x, float y, float l) {
    float xc = clipf_l(x, l), yc = clipf_l(y, l);
    float o = logf(1.0f + expf(xc + yc));
    o -= logf(expf(xc) + expf(yc));
    return o;
}
/* g, polar_sc.py:49-53: (1-2u)x + y on unclipped inputs. */
static inline float g_op(float x, float y, float u) { return (1.0f - 2.0f * u) * x + y; }
/* leaf, polar_sc.py:90-98: u = 0.5(1-sign(llr)), 0.5 -> 1, i.e. 1 iff !(llr > 0). */
static inline float leaf_hd(float llr) { return (llr > 0.0f) ? 0.0f : 1.0f; }

static int ilog2(int n) { int s = 0; while ((1 << s) < n) ++s; return ((1 << s) == n) ? s : -1; }

/* ---------------------------------------------------------------- SC ---- */
typedef struct {
    int n, S, f_mode;
    float lmax;   /* llr_max (the reference: 30) */
    const uint8_t* frozen;
    float* llr;   /* [S+1][n]  msg_llr  (polar_sc.py:108-110) */
    float* uhat;  /* [S+1][n]  msg_uhat */
} sc_ctx;

/* polar_sc.py:54-98, node = positions [a, a + 2^s) */
static void sc_node(sc_ctx* c, int a, int s) {
    const int n = c->n;
    float* L = c->llr;
    float* U = c->uhat;
    if (s > 0) {
        const int h = 1 << (s - 1);
        float* in = L + (size_t)s * n;
        float* out = L + (size_t)(s - 1) * n;
        for (int j = 0; j < h; ++j)
            out[a + j] = c->f_mode ? f_exact(in[a + j], in[a + h + j], c->lmax)
                                : f_minsum(in[a + j], in[a + h + j], c->lmax);
        sc_node(c, a, s - 1);
        const float* ul = U + (size_t)(s - 1) * n;
        for (int j = 0; j < h; ++j) out[a + h + j] = g_op(in[a + j], in[a + h + j], ul[a + j]);
        sc_node(c, a + h, s - 1);
        float* us = U + (size_t)s * n;
        for (int j = 0; j < h; ++j) {
            float l = ul[a + j], r = ul[a + h + j];
            us[a + j] = (l != r) ? 1.0f : 0.0f;
            us[a + h + j] = r;
        }
    } else {
        U[a] = c->frozen[a] ? 0.0f : leaf_hd(L[a]);
    }
}

/* SC_Dec.forward (polar_sc.py:113-133): logits are negated, decoded, gathered at info_pos.
 * orc_sc_decode_lmax: the same with another clipping bound than the reference's 30 (a plan's
 * llr_max; tests of the full-range exact f). */
int orc_sc_decode_lmax(int n, const uint8_t* frozen_mask, int f_mode, float lmax, const float* logits, int64_t bs,
                       float* out_bits, int nthreads) {
    const int S = ilog2(n);
    if (S < 0 || !frozen_mask || !logits || !out_bits || bs < 0) return -1;
    int* info = (int*)malloc(sizeof(int) * (size_t)n);
    int k = 0;
    for (int i = 0; i < n; ++i) if (!frozen_mask[i]) info[k++] = i;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        sc_ctx c;
        c.n = n; c.S = S; c.f_mode = f_mode; c.lmax = lmax; c.frozen = frozen_mask;
        c.llr = (float*)malloc(sizeof(float) * (size_t)(S + 1) * n);
        c.uhat = (float*)malloc(sizeof(float) * (size_t)(S + 1) * n);
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t b = 0; b < bs; ++b) {
            memset(c.uhat, 0, sizeof(float) * (size_t)(S + 1) * n);
            for (int i = 0; i < n; ++i) c.llr[(size_t)S * n + i] = -1.0f * logits[b * n + i];
            sc_node(&c, 0, S);
            for (int m = 0; m < k; ++m) out_bits[b * k + m] = c.uhat[info[m]];
        }
        free(c.llr); free(c.uhat);
    }
    free(info);
    return k;
}
int orc_sc_decode(int n, const uint8_t* frozen_mask, int f_mode, const float* logits, int64_t bs,
                  float* out_bits, int nthreads) {
    return orc_sc_decode_lmax(n, frozen_mask, f_mode, LLR_MAX, logits, bs, out_bits, nthreads);
}

/* --------------------------------------------------------------- SCL ---- */
/* Faithful restatement of polar_scl.py: 2L physical rows of [S+1][n] float64 state. */
typedef struct {
    int n, S, L;
    const uint8_t* frozen;
    double* llr;   /* [2L][S+1][n] */
    double* uhat;  /* [2L][S+1][n] */
    double pm[64];
    int ptr[64];
} scl_ctx;

#define ROW(c, base, p, s) ((base) + ((size_t)(p) * ((c)->S + 1) + (s)) * (c)->n)

static inline double f_minsum_d(double x, double y, double lmax) {  /* polar_scl.py:93-106 (torch on f64) */
    double xc = fmin(fmax(x, -lmax), lmax), yc = fmin(fmax(y, -lmax), lmax);
    double sx = (double)((xc > 0) - (xc < 0)), sy = (double)((yc > 0) - (yc < 0));
    return sx * sy * fmin(fabs(xc), fabs(yc));
}

static void scl_sort(scl_ctx* c) {  /* polar_scl.py:86-92, stable (pm, logical index) order */
    const int M = 2 * c->L;
    for (int i = 1; i < M; ++i) {
        double v = c->pm[i]; int p = c->ptr[i]; int j = i - 1;
        while (j >= 0 && c->pm[j] > v) { c->pm[j + 1] = c->pm[j]; c->ptr[j + 1] = c->ptr[j]; --j; }
        c->pm[j + 1] = v; c->ptr[j + 1] = p;
    }
}

static void scl_node(scl_ctx* c, int a, int s) {  /* polar_scl.py:121-177 */
    const int M = 2 * c->L, n = c->n;
    if (s > 0) {
        const int h = 1 << (s - 1);
        for (int p = 0; p < M; ++p) {
            double* in = ROW(c, c->llr, p, s);
            double* out = ROW(c, c->llr, p, s - 1);
            for (int j = 0; j < h; ++j) out[a + j] = f_minsum_d(in[a + j], in[a + h + j], 30.0);
        }
        scl_node(c, a, s - 1);
        for (int p = 0; p < M; ++p) {
            double* in = ROW(c, c->llr, p, s);
            double* out = ROW(c, c->llr, p, s - 1);
            const double* ul = ROW(c, c->uhat, p, s - 1);
            for (int j = 0; j < h; ++j) out[a + h + j] = (1.0 - 2.0 * ul[a + j]) * in[a + j] + in[a + h + j];
        }
        scl_node(c, a + h, s - 1);
        for (int p = 0; p < M; ++p) {
            const double* ul = ROW(c, c->uhat, p, s - 1);
            double* us = ROW(c, c->uhat, p, s);
            for (int j = 0; j < h; ++j) {
                double l = ul[a + j], r = ul[a + h + j];
                us[a + j] = (l != r) ? 1.0 : 0.0;
                us[a + h + j] = r;
            }
        }
    } else {
        const int info = !c->frozen[a];
        if (info)  /* _update_single_bit_np :49-68 */
            for (int j = c->L; j < M; ++j) ROW(c, c->uhat, c->ptr[j], 0)[a] = 1.0;
        for (int j = 0; j < M; ++j) {  /* _update_pm_np :69-85 */
            const int p = c->ptr[j];
            const double u = ROW(c, c->uhat, p, 0)[a];
            double l = ROW(c, c->llr, p, 0)[a];
            l = fmax(fmin(l, 30.0), -30.0);
            c->pm[j] += log(1.0 + exp(-((1.0 - 2.0 * u) * l)));
        }
        if (info) {
            scl_sort(c);
            for (int m = 0; m < c->L; ++m) {  /* _duplicate_paths_np :109-120 */
                const int lo = c->ptr[m], up = c->ptr[c->L + m];
                memcpy(ROW(c, c->uhat, up, 0), ROW(c, c->uhat, lo, 0), sizeof(double) * (size_t)(c->S + 1) * n);
                memcpy(ROW(c, c->llr, up, 0), ROW(c, c->llr, lo, 0), sizeof(double) * (size_t)(c->S + 1) * n);
            }
            for (int m = 0; m < c->L; ++m) c->pm[c->L + m] = c->pm[m];
        }
    }
}

/* SCL_Dec.forward (polar_scl.py:210-234).  out_pm (nullable) = final sorted msg_pm [bs][2L]. */
int orc_scl_decode(int n, const uint8_t* frozen_mask, int L, const float* logits, int64_t bs,
                   float* out_bits, double* out_pm, int nthreads) {
    const int S = ilog2(n);
    if (S < 0 || L < 1 || L > 32 || (L & (L - 1)) || !frozen_mask || !logits || !out_bits) return -1;
    int* info = (int*)malloc(sizeof(int) * (size_t)n);
    int k = 0;
    for (int i = 0; i < n; ++i) if (!frozen_mask[i]) info[k++] = i;
    const int M = 2 * L;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        scl_ctx c;
        c.n = n; c.S = S; c.L = L; c.frozen = frozen_mask;
        const size_t rowsz = (size_t)(S + 1) * n;
        c.llr = (double*)malloc(sizeof(double) * rowsz * M);
        c.uhat = (double*)malloc(sizeof(double) * rowsz * M);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t b = 0; b < bs; ++b) {
            memset(c.uhat, 0, sizeof(double) * rowsz * M);
            memset(c.llr, 0, sizeof(double) * rowsz * M);
            for (int j = 0; j < M; ++j) {  /* _decode_np_batch :190-200 */
                c.pm[j] = (j % L == 0) ? 0.0 : 30.0;
                c.ptr[j] = j;
                double* top = ROW(&c, c.llr, j, S);
                for (int i = 0; i < n; ++i) top[i] = (double)(-1.0f * logits[b * n + i]);
            }
            scl_node(&c, 0, S);
            scl_sort(&c);  /* :204 */
            /* forward :224-228: argmin over the sorted pm = slot 0 (first minimum) */
            const double* u0 = ROW(&c, c.uhat, c.ptr[0], 0);
            for (int m = 0; m < k; ++m) out_bits[b * k + m] = (float)u0[info[m]];
            if (out_pm) for (int j = 0; j < M; ++j) out_pm[b * M + j] = c.pm[j];
        }
        free(c.llr); free(c.uhat);
    }
    free(info);
    return k;
}

/* ----------------------------------------------- SCL, lazy-copy form ---- */
/* Same decoder as orc_scl_decode (equivalence: logical rows j and j+L are always identical
 * copies, so L states suffice).  Stage-s LLR buffers are per (path, stage) with a per-path
 * pointer to the buffer holding its current stage-s node; the channel stage is shared. */
typedef struct {
    int n, S, L;
    const uint8_t* frozen;
    const double* ch;      /* [n] negated channel LLRs */
    double* alpha;         /* [L][n] : stage s of path p at alpha[p*n + 2^s .. 2^(s+1)) */
    int* sptr;             /* [L][S+1] : which path's stage-s buffer path p reads */
    uint8_t* beta;         /* [L][n] partial sums by absolute position */
    uint8_t* u;            /* [L][n] decided u */
    double pm[32];
    double lmax;           /* clipping bound llr_max (reference: 30) */
    uint8_t* tmp_beta; uint8_t* tmp_u; int* tmp_sptr;
} lz_ctx;

static const double* lz_stage(lz_ctx* c, int p, int s) {
    if (s == c->S) return c->ch;
    return c->alpha + (size_t)c->sptr[p * (c->S + 1) + s] * c->n + (1u << s);
}

static void lz_node(lz_ctx* c, int a, int s) {
    const int n = c->n, L = c->L, S1 = c->S + 1;
    if (s > 0) {
        const int h = 1 << (s - 1);
        for (int p = 0; p < L; ++p) {
            const double* in = lz_stage(c, p, s);
            double* out = c->alpha + (size_t)p * n + (1u << (s - 1));
            for (int j = 0; j < h; ++j) out[j] = f_minsum_d(in[j], in[j + h], c->lmax);
        }
        for (int p = 0; p < L; ++p) c->sptr[p * S1 + s - 1] = p;
        lz_node(c, a, s - 1);
        for (int p = 0; p < L; ++p) {
            const double* in = lz_stage(c, p, s);
            double* out = c->alpha + (size_t)p * n + (1u << (s - 1));
            const uint8_t* bl = c->beta + (size_t)p * n + a;
            for (int j = 0; j < h; ++j) out[j] = (bl[j] ? -in[j] : in[j]) + in[j + h];
        }
        for (int p = 0; p < L; ++p) c->sptr[p * S1 + s - 1] = p;
        lz_node(c, a + h, s - 1);
        for (int p = 0; p < L; ++p) {
            uint8_t* b = c->beta + (size_t)p * n + a;
            for (int j = 0; j < h; ++j) b[j] ^= b[j + h];
        }
    } else {
        const int info = !c->frozen[a];
        double cand[64];
        for (int p = 0; p < L; ++p) {
            const double l = fmax(fmin(lz_stage(c, p, 0)[0], c->lmax), -c->lmax);
            cand[p] = c->pm[p] + log(1.0 + exp(-l));           /* u = 0 */
            cand[L + p] = c->pm[p] + log(1.0 + exp(-(-1.0 * l)));  /* u = 1 */
        }
        if (!info) {
            for (int p = 0; p < L; ++p) { c->pm[p] = cand[p]; c->beta[(size_t)p * n + a] = 0; c->u[(size_t)p * n + a] = 0; }
            return;
        }
        /* stable rank of every candidate; survivors = ranks < L, in rank order */
        int src[32], bit[32];
        double npm[32];
        for (int i = 0; i < 2 * L; ++i) {
            int r = 0;
            for (int j = 0; j < 2 * L; ++j) r += (cand[j] < cand[i]) || (cand[j] == cand[i] && j < i);
            if (r < L) { src[r] = i % L; bit[r] = i / L; npm[r] = cand[i]; }
        }
        memcpy(c->tmp_beta, c->beta, (size_t)L * n);
        memcpy(c->tmp_u, c->u, (size_t)L * n);
        memcpy(c->tmp_sptr, c->sptr, sizeof(int) * (size_t)L * S1);
        for (int m = 0; m < L; ++m) {
            const int q = src[m];
            memcpy(c->beta + (size_t)m * n, c->tmp_beta + (size_t)q * n, (size_t)n);
            memcpy(c->u + (size_t)m * n, c->tmp_u + (size_t)q * n, (size_t)n);
            memcpy(c->sptr + (size_t)m * S1, c->tmp_sptr + (size_t)q * S1, sizeof(int) * S1);
            c->beta[(size_t)m * n + a] = (uint8_t)bit[m];
            c->u[(size_t)m * n + a] = (uint8_t)bit[m];
            c->pm[m] = npm[m];
        }
    }
}

int orc_scl_decode_lazy(int n, const uint8_t* frozen_mask, int L, const float* logits, int64_t bs,
                        float* out_bits, double* out_pm, int nthreads) {
    const int S = ilog2(n);
    if (S < 0 || L < 1 || L > 32 || (L & (L - 1)) || !frozen_mask || !logits || !out_bits) return -1;
    int* info = (int*)malloc(sizeof(int) * (size_t)n);
    int k = 0;
    for (int i = 0; i < n; ++i) if (!frozen_mask[i]) info[k++] = i;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        lz_ctx c;
        c.n = n; c.S = S; c.L = L; c.frozen = frozen_mask; c.lmax = 30.0;
        double* ch = (double*)malloc(sizeof(double) * (size_t)n);
        c.ch = ch;
        c.alpha = (double*)malloc(sizeof(double) * (size_t)L * n);
        c.sptr = (int*)malloc(sizeof(int) * (size_t)L * (S + 1));
        c.beta = (uint8_t*)malloc((size_t)L * n);
        c.u = (uint8_t*)malloc((size_t)L * n);
        c.tmp_beta = (uint8_t*)malloc((size_t)L * n);
        c.tmp_u = (uint8_t*)malloc((size_t)L * n);
        c.tmp_sptr = (int*)malloc(sizeof(int) * (size_t)L * (S + 1));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
        for (int64_t b = 0; b < bs; ++b) {
            for (int i = 0; i < n; ++i) ch[i] = (double)(-1.0f * logits[b * n + i]);
            memset(c.beta, 0, (size_t)L * n);
            memset(c.u, 0, (size_t)L * n);
            for (int p = 0; p < L * (S + 1); ++p) c.sptr[p] = p / (S + 1);
            for (int p = 0; p < L; ++p) c.pm[p] = p == 0 ? 0.0 : c.lmax;
            lz_node(&c, 0, S);
            int best = 0;
            for (int p = 1; p < L; ++p) if (c.pm[p] < c.pm[best]) best = p;
            for (int m = 0; m < k; ++m) out_bits[b * k + m] = (float)c.u[(size_t)best * n + info[m]];
            if (out_pm) {
                /* final msg_pm after the last sort: every survivor appears twice (rows j, j+L) */
                double tmp[64];
                for (int p = 0; p < L; ++p) { tmp[2 * p] = c.pm[p]; tmp[2 * p + 1] = c.pm[p]; }
                for (int i = 1; i < 2 * L; ++i) {
                    double v = tmp[i]; int j = i - 1;
                    while (j >= 0 && tmp[j] > v) { tmp[j + 1] = tmp[j]; --j; }
                    tmp[j + 1] = v;
                }
                memcpy(out_pm + b * 2 * L, tmp, sizeof(double) * 2 * L);
            }
        }
        free(ch); free(c.alpha); free(c.sptr); free(c.beta); free(c.u);
        free(c.tmp_beta); free(c.tmp_u); free(c.tmp_sptr);
    }
    free(info);
    return k;
}

/* ------------------------------------------- my_sn SCL (fast-SCL, CRC) ---- */
/* np.sum over the last axis of a contiguous float64 array: numpy's pairwise summation
 * (blocks of <= 128 with 8 interleaved partial sums, halves above).  Pinned against numpy in
 * tests/test_oracle.py. */
double orc_np_pairwise_sum(const double* a, int n) {
    if (n < 8) {
        double r = 0.0;
        for (int i = 0; i < n; ++i) r += a[i];
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int i = 8;
        for (; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    return orc_np_pairwise_sum(a, n2) + orc_np_pairwise_sum(a + n2, n - n2);
}

/* CRC remainder of bits[0..len) (MSB first) times D^deg modulo g, g given by its coefficient
 * bit mask without the leading term (bit c set = D^c present, c < deg). */
static uint32_t crc_reg(const uint8_t* bits, int len, int deg, uint32_t g) {
    uint32_t reg = 0, mask = (deg == 32) ? 0xffffffffu : ((1u << deg) - 1u);
    for (int i = 0; i < len; ++i) {
        const uint32_t fb = ((reg >> (deg - 1)) & 1u) ^ (bits[i] & 1u);
        reg = (reg << 1) & mask;
        if (fb) reg ^= g;
    }
    return reg;
}

/* CRCEncoder.forward: [bs, k] 0/1 -> [bs, k + deg] (systematic, parity appended MSB first). */
int orc_crc_encode(const float* in, int64_t bs, int k, int deg, uint32_t g, float* out) {
    if (deg < 1 || deg > 31 || k < 0) return -1;
    uint8_t* b = (uint8_t*)malloc((size_t)k + 1);
    for (int64_t r = 0; r < bs; ++r) {
        for (int i = 0; i < k; ++i) b[i] = in[r * k + i] != 0.0f;
        const uint32_t reg = crc_reg(b, k, deg, g);
        for (int i = 0; i < k; ++i) out[r * (k + deg) + i] = (float)b[i];
        for (int i = 0; i < deg; ++i) out[r * (k + deg) + k + i] = (float)((reg >> (deg - 1 - i)) & 1u);
    }
    free(b);
    return 0;
}

/* CRCDecoder.forward validity: re-encoding the whole (info||parity) word gives zero parity. */
int orc_crc_check(const float* in, int64_t bs, int len, int deg, uint32_t g, uint8_t* valid) {
    if (deg < 1 || deg > 31 || len < deg) return -1;
    uint8_t* b = (uint8_t*)malloc((size_t)len + 1);
    for (int64_t r = 0; r < bs; ++r) {
        for (int i = 0; i < len; ++i) b[i] = in[r * len + i] != 0.0f;
        valid[r] = crc_reg(b, len, deg, g) == 0u;
    }
    free(b);
    return 0;
}

static inline double f_exact_d(double x, double y, double lmax) {  /* dec.py:330-339 on float64 */
    const double xc = fmax(fmin(x, lmax), -lmax), yc = fmax(fmin(y, lmax), -lmax);
    double o = log(1.0 + exp(xc + yc));
    o -= log(exp(xc) + exp(yc));
    return o;
}

typedef struct {
    lz_ctx z;
    int fast, exact;
    double* terms;  /* [n] scratch for node sums */
} my_ctx;

/* stable selection of L survivors among 2L candidates + fork (dec.py:315-330, :340-352) */
static void my_select(lz_ctx* c, const double* cand, int a, int len) {
    const int L = c->L, n = c->n, S1 = c->S + 1;
    int src[32], bit[32];
    double npm[32];
    for (int i = 0; i < 2 * L; ++i) {
        int r = 0;
        for (int j = 0; j < 2 * L; ++j) r += (cand[j] < cand[i]) || (cand[j] == cand[i] && j < i);
        if (r < L) { src[r] = i % L; bit[r] = i / L; npm[r] = cand[i]; }
    }
    memcpy(c->tmp_beta, c->beta, (size_t)L * n);
    memcpy(c->tmp_u, c->u, (size_t)L * n);
    memcpy(c->tmp_sptr, c->sptr, sizeof(int) * (size_t)L * S1);
    for (int m = 0; m < L; ++m) {
        const int q = src[m];
        memcpy(c->beta + (size_t)m * n, c->tmp_beta + (size_t)q * n, (size_t)n);
        memcpy(c->u + (size_t)m * n, c->tmp_u + (size_t)q * n, (size_t)n);
        memcpy(c->sptr + (size_t)m * S1, c->tmp_sptr + (size_t)q * S1, sizeof(int) * S1);
        for (int j = a; j < a + len; ++j) c->beta[(size_t)m * n + j] = (uint8_t)bit[m];  /* node partial sums */
        c->u[(size_t)m * n + a + len - 1] = (uint8_t)bit[m];                              /* its info bit */
        c->pm[m] = npm[m];
    }
}

static void my_node(my_ctx* mc, int a, int s) {
    lz_ctx* c = &mc->z;
    const int n = c->n, L = c->L, S1 = c->S + 1, len = 1 << s;
    if (s > 0 && mc->fast) {
        int nfz = 0;
        for (int j = a; j < a + len; ++j) nfz += c->frozen[j] != 0;
        if (nfz == len) {  /* rate-0 (dec.py:269-280): pm += sum softplus(-clip(llr)) */
            for (int p = 0; p < L; ++p) {
                const double* in = lz_stage(c, p, s);
                for (int j = 0; j < len; ++j) mc->terms[j] = log(1.0 + exp(-fmax(fmin(in[j], c->lmax), -c->lmax)));
                c->pm[p] += orc_np_pairwise_sum(mc->terms, len);
                memset(c->beta + (size_t)p * n + a, 0, (size_t)len);
            }
            return;
        }
        if (!c->frozen[a + len - 1] && nfz == len - 1) {  /* repetition (dec.py:281-306) */
            double cand[64];
            for (int p = 0; p < L; ++p) {
                const double* in = lz_stage(c, p, s);
                for (int j = 0; j < len; ++j) mc->terms[j] = log(1.0 + exp(-fmax(fmin(in[j], c->lmax), -c->lmax)));
                cand[p] = c->pm[p] + orc_np_pairwise_sum(mc->terms, len);
                for (int j = 0; j < len; ++j) mc->terms[j] = log(1.0 + exp(-fmax(fmin(-in[j], c->lmax), -c->lmax)));
                cand[L + p] = c->pm[p] + orc_np_pairwise_sum(mc->terms, len);
            }
            my_select(c, cand, a, len);
            return;
        }
    }
    if (s > 0) {
        const int h = 1 << (s - 1);
        for (int p = 0; p < L; ++p) {
            const double* in = lz_stage(c, p, s);
            double* out = c->alpha + (size_t)p * n + (1u << (s - 1));
            for (int j = 0; j < h; ++j) out[j] = mc->exact ? f_exact_d(in[j], in[j + h], c->lmax) : f_minsum_d(in[j], in[j + h], c->lmax);
        }
        for (int p = 0; p < L; ++p) c->sptr[p * S1 + s - 1] = p;
        my_node(mc, a, s - 1);
        for (int p = 0; p < L; ++p) {
            const double* in = lz_stage(c, p, s);
            double* out = c->alpha + (size_t)p * n + (1u << (s - 1));
            const uint8_t* bl = c->beta + (size_t)p * n + a;
            for (int j = 0; j < h; ++j) out[j] = (bl[j] ? -in[j] : in[j]) + in[j + h];
        }
        for (int p = 0; p < L; ++p) c->sptr[p * S1 + s - 1] = p;
        my_node(mc, a + h, s - 1);
        for (int p = 0; p < L; ++p) {
            uint8_t* b = c->beta + (size_t)p * n + a;
            for (int j = 0; j < h; ++j) b[j] ^= b[j + h];
        }
        return;
    }
    /* leaf (dec.py:377-383): pm update every leaf; info leaves select and fork */
    double cand[64];
    for (int p = 0; p < L; ++p) {
        const double l = fmax(fmin(lz_stage(c, p, 0)[0], c->lmax), -c->lmax);
        cand[p] = c->pm[p] + log(1.0 + exp(-l));
        cand[L + p] = c->pm[p] + log(1.0 + exp(-(-1.0 * l)));
    }
    if (c->frozen[a]) {
        for (int p = 0; p < L; ++p) { c->pm[p] = cand[p]; c->beta[(size_t)p * n + a] = 0; c->u[(size_t)p * n + a] = 0; }
        return;
    }
    my_select(c, cand, a, 1);
}

/* SCL_Dec.forward of my_sn (dec.py:476-537).  crc_deg = 0: no CRC.  out_pm = msg_pm as the
 * reference leaves it: sorted by _decode_np_batch, then CRC-penalised in place, [bs][2L]. */
int orc_scl_decode_mysn(int n, const uint8_t* frozen_mask, int L, const float* logits, int64_t bs, float* out_bits,
                        double* out_pm, int fast_scl, int exact_f, int crc_deg, uint32_t crc_g, double llr_max, int nthreads) {
    const int S = ilog2(n);
    if (S < 0 || L < 1 || L > 32 || (L & (L - 1)) || !frozen_mask || !logits || !out_bits) return -1;
    int* info = (int*)malloc(sizeof(int) * (size_t)n);
    int k = 0;
    for (int i = 0; i < n; ++i) if (!frozen_mask[i]) info[k++] = i;
    if (crc_deg > 0 && k < crc_deg) { free(info); return -1; }
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        my_ctx mc;
        lz_ctx* c = &mc.z;
        mc.fast = fast_scl; mc.exact = exact_f;
        c->n = n; c->S = S; c->L = L; c->frozen = frozen_mask; c->lmax = llr_max;
        double* ch = (double*)malloc(sizeof(double) * (size_t)n);
        c->ch = ch;
        c->alpha = (double*)malloc(sizeof(double) * (size_t)L * n);
        c->sptr = (int*)malloc(sizeof(int) * (size_t)L * (S + 1));
        c->beta = (uint8_t*)malloc((size_t)L * n);
        c->u = (uint8_t*)malloc((size_t)L * n);
        c->tmp_beta = (uint8_t*)malloc((size_t)L * n);
        c->tmp_u = (uint8_t*)malloc((size_t)L * n);
        c->tmp_sptr = (int*)malloc(sizeof(int) * (size_t)L * (S + 1));
        mc.terms = (double*)malloc(sizeof(double) * (size_t)n);
        uint8_t* ub = (uint8_t*)malloc((size_t)k + 1);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
        for (int64_t b = 0; b < bs; ++b) {
            for (int i = 0; i < n; ++i) ch[i] = (double)(-1.0f * logits[b * n + i]);
            memset(c->beta, 0, (size_t)L * n);
            memset(c->u, 0, (size_t)L * n);
            for (int p = 0; p < L * (S + 1); ++p) c->sptr[p] = p / (S + 1);
            for (int p = 0; p < L; ++p) c->pm[p] = p == 0 ? 0.0 : c->lmax;
            my_node(&mc, 0, S);
            /* final sort (dec.py:202) of the 2L logical rows (row r < L = state r, row r >= L its
             * copy), stable by pm; CRC penalty llr_max*k per failing row added in place (dec.py:515-518,
             * which also lands in the returned msg_pm: it aliases self.msg_pm); first argmin. */
            int row[64];
            for (int r = 0; r < 2 * L; ++r) row[r] = r;
            for (int i = 1; i < 2 * L; ++i) {
                int v = row[i], j = i - 1;
                while (j >= 0 && c->pm[row[j] % L] > c->pm[v % L]) { row[j + 1] = row[j]; --j; }
                row[j + 1] = v;
            }
            int fail[32] = {0};
            if (crc_deg > 0)
                for (int p = 0; p < L; ++p) {
                    for (int m = 0; m < k; ++m) ub[m] = c->u[(size_t)p * n + info[m]];
                    fail[p] = crc_reg(ub, k, crc_deg, crc_g) != 0u;
                }
            int best = row[0] % L;
            double bestv = 0.0;
            for (int r = 0; r < 2 * L; ++r) {
                const int p = row[r] % L;
                const double v = c->pm[p] + (fail[p] ? c->lmax * (double)k : 0.0);
                if (out_pm) out_pm[b * 2 * L + r] = v;
                if (r == 0 || v < bestv) { best = p; bestv = v; }
            }
            for (int m = 0; m < k; ++m) out_bits[b * k + m] = (float)c->u[(size_t)best * n + info[m]];
        }
        free(ch); free(c->alpha); free(c->sptr); free(c->beta); free(c->u);
        free(c->tmp_beta); free(c->tmp_u); free(c->tmp_sptr); free(mc.terms); free(ub);
    }
    free(info);
    return k;
}

/* ----------------------------------------------------------- encoder ---- */
/* x_run_sn_polar/polar/enc.py:30-43: codeword = (u placed at info_pos) * F2^{(x)m} mod 2. */
int orc_polar_encode(int n, const uint8_t* frozen_mask, const float* u_bits, int64_t bs, float* out_cw) {
    const int S = ilog2(n);
    if (S < 0) return -1;
    int k = 0;
    for (int i = 0; i < n; ++i) k += !frozen_mask[i];
    uint8_t* x = (uint8_t*)malloc((size_t)n);
    for (int64_t b = 0; b < bs; ++b) {
        int m = 0;
        for (int i = 0; i < n; ++i) x[i] = frozen_mask[i] ? 0 : (u_bits[b * k + m++] != 0.0f);
        /* row vector times G = kron^m(F2), F2 = [[1,0],[1,1]]: x[j] ^= x[j+h] for the lower half */
        for (int h = 1; h < n; h <<= 1)
            for (int a = 0; a < n; a += 2 * h)
                for (int j = 0; j < h; ++j) x[a + j] ^= x[a + h + j];
        for (int i = 0; i < n; ++i) out_cw[b * n + i] = (float)x[i];
    }
    free(x);
    return k;
}
