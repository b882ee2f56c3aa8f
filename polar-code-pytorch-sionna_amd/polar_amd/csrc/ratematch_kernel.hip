// ratematch_kernel.hip -- the 5G NR data path around the mother-code decoder:
// CRC attachment, rate matching (gather) and rate recovery, for gfx950.
//
// Reference: my_sn/fec/polar/enc.py Polar5GEncoder.forward :359-392 (CRC encode -> polar encode
// -> c[:, ind_rate_matching]) and dec.py Polar5GDecoder.forward :612-666 (channel de-interleave,
// de-puncture / de-shorten / repetition combine, sub-block de-interleave).  All index tables are
// built once on the host (polar_amd/polar5g.py, 3GPP TS 38.212 Sec. 5.4.1) and passed as device
// pointers; the kernels are HBM-bound gathers: one block per row group, the table in LDS, lanes
// over columns (coalesced stores; loads stay inside the row, which L1/L2 serve).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/polar_mi355x.h"
#include "plan.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxCols = 4096;  // table entries staged in LDS

// out[b, j] = in[b, idx[j]]
__global__ __launch_bounds__(kThreads) void gather_rows_kernel(const float* __restrict__ in, int64_t bs, int n_in,
                                                               const int32_t* __restrict__ idx, int n_out,
                                                               float* __restrict__ out, int rows_per_block) {
    __shared__ int32_t s_idx[kMaxCols];
    for (int j = threadIdx.x; j < n_out; j += kThreads) s_idx[j] = idx[j];
    __syncthreads();
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    for (int r = 0; r < rows_per_block; ++r) {
        const int64_t b = r0 + r;
        if (b >= bs) break;
        const float* x = in + b * n_in;
        float* y = out + b * n_out;
        for (int j = threadIdx.x; j < n_out; j += kThreads) y[j] = x[s_idx[j]];
    }
}

// out[b, j] = a[j] < 0 ? fill[j] : in[b, a[j]] (+ in[b, c[j]] when c[j] >= 0)
__global__ __launch_bounds__(kThreads) void rate_recover_kernel(const float* __restrict__ in, int64_t bs, int e,
                                                                const int32_t* __restrict__ src_a,
                                                                const int32_t* __restrict__ src_b,
                                                                const float* __restrict__ fill, int n,
                                                                float* __restrict__ out, int rows_per_block) {
    __shared__ int32_t s_a[kMaxCols / 2], s_b[kMaxCols / 2];
    __shared__ float s_f[kMaxCols / 2];
    for (int j = threadIdx.x; j < n; j += kThreads) {
        s_a[j] = src_a[j];
        s_b[j] = src_b ? src_b[j] : -1;
        s_f[j] = fill ? fill[j] : 0.0f;
    }
    __syncthreads();
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    for (int r = 0; r < rows_per_block; ++r) {
        const int64_t b = r0 + r;
        if (b >= bs) break;
        const float* x = in + b * e;
        float* y = out + b * n;
        for (int j = threadIdx.x; j < n; j += kThreads) {
            const int a = s_a[j], c = s_b[j];
            float v = s_f[j];
            if (a >= 0) v = c >= 0 ? x[a] + x[c] : x[a];  // llr_1 + llr_3 (dec.py:629-633)
            y[j] = v;
        }
    }
}

// One wave per codeword: parity = XOR of the generator rows of the 1 bits (crc.py:85-104, the
// k x degree G matrix of :54-73 packed one row per uint32, bit c = parity column c).
__global__ __launch_bounds__(kThreads) void crc_attach_kernel(const float* __restrict__ u, int64_t bs, int k,
                                                              const uint32_t* __restrict__ g_rows, int degree,
                                                              float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (b >= bs) return;
    const float* x = u + b * k;
    float* y = out + b * (int64_t)(k + degree);
    uint32_t acc = 0u;
    for (int m = lane; m < k; m += 64) {
        const float v = x[m];
        y[m] = v;
        if (v != 0.0f) acc ^= g_rows[m];
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, off, 64);
    if (lane < degree) y[k + lane] = (float)((acc >> lane) & 1u);
}

// CRCDecoder.forward (crc.py:119-138): the reference re-encodes the whole received word
// [info, parity] with the generator of its full length and calls it valid iff every parity bit
// of that is 0 (for a cyclic code: the received parity equals the CRC of the info bits).  One
// wave per word, the same row XOR as crc_attach_kernel over all len bits; one byte per word out.
__global__ __launch_bounds__(kThreads) void crc_check_kernel(const float* __restrict__ word, int64_t bs, int len,
                                                             const uint32_t* __restrict__ g_rows,
                                                             uint8_t* __restrict__ valid) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (b >= bs) return;
    const float* x = word + b * len;
    uint32_t acc = 0u;
    for (int m = lane; m < len; m += 64)
        if (x[m] != 0.0f) acc ^= g_rows[m];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, off, 64);
    if (lane == 0) valid[b] = acc == 0u ? 1 : 0;
}

int rows_per_block(int64_t bs) {
    // >= 4 blocks per CU's worth of rows, at most 8 rows per block
    int64_t r = bs / (256 * 8);
    if (r < 1) r = 1;
    if (r > 8) r = 8;
    return (int)r;
}

}  // namespace

extern "C" {

int pl_gather_rows(const float* in, int64_t bs, int32_t n_in, const int32_t* idx, int32_t n_out, float* out,
                   void* stream) {
    if (bs < 0 || n_in < 1 || n_out < 0 || n_out > kMaxCols || (bs > 0 && (!in || !idx || !out))) {
        pl::set_error("pl_gather_rows: bad arguments");
        return PL_EINVAL;
    }
    if (bs == 0 || n_out == 0) return PL_OK;
    const int rpb = rows_per_block(bs);
    const int64_t blocks = (bs + rpb - 1) / rpb;
    if (blocks > 0x7fffffffLL) {
        pl::set_error("pl_gather_rows: batch too large");
        return PL_EINVAL;
    }
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                       in, bs, n_in, idx, n_out, out, rpb);
    return pl::check_hip(hipGetLastError(), "pl_gather_rows launch");
}

int pl_rate_recover(const float* llr, int64_t bs, int32_t e, const int32_t* src_a, const int32_t* src_b,
                    const float* fill, int32_t n, float* out, void* stream) {
    if (bs < 0 || e < 1 || n < 1 || n > kMaxCols / 2 || (bs > 0 && (!llr || !src_a || !out))) {
        pl::set_error("pl_rate_recover: bad arguments");
        return PL_EINVAL;
    }
    if (bs == 0) return PL_OK;
    const int rpb = rows_per_block(bs);
    const int64_t blocks = (bs + rpb - 1) / rpb;
    if (blocks > 0x7fffffffLL) {
        pl::set_error("pl_rate_recover: batch too large");
        return PL_EINVAL;
    }
    hipLaunchKernelGGL(rate_recover_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                       llr, bs, e, src_a, src_b, fill, n, out, rpb);
    return pl::check_hip(hipGetLastError(), "pl_rate_recover launch");
}

int pl_crc_attach(const float* u, int64_t bs, int32_t k, const uint32_t* g_rows, int32_t degree, float* out,
                  void* stream) {
    if (bs < 0 || k < 0 || degree < 1 || degree > 32 || (bs > 0 && (!u || !out || (k > 0 && !g_rows)))) {
        pl::set_error("pl_crc_attach: bad arguments");
        return PL_EINVAL;
    }
    if (bs == 0) return PL_OK;
    const int64_t blocks = (bs + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > 0x7fffffffLL) {
        pl::set_error("pl_crc_attach: batch too large");
        return PL_EINVAL;
    }
    hipLaunchKernelGGL(crc_attach_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                       u, bs, k, g_rows, degree, out);
    return pl::check_hip(hipGetLastError(), "pl_crc_attach launch");
}

int pl_crc_check(const float* word, int64_t bs, int32_t len, const uint32_t* g_rows, int32_t degree,
                 uint8_t* valid, void* stream) {
    if (bs < 0 || len < degree || degree < 1 || degree > 32 || (bs > 0 && (!word || !g_rows || !valid))) {
        pl::set_error("pl_crc_check: bad arguments");
        return PL_EINVAL;
    }
    if (bs == 0) return PL_OK;
    const int64_t blocks = (bs + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > 0x7fffffffLL) {
        pl::set_error("pl_crc_check: batch too large");
        return PL_EINVAL;
    }
    hipLaunchKernelGGL(crc_check_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                       word, bs, len, g_rows, valid);
    return pl::check_hip(hipGetLastError(), "pl_crc_check launch");
}

}  // extern "C"
