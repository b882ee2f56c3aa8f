// channel_kernel.hip -- the Monte-Carlo caller side of the decoder, fused for gfx950:
//
//   awgn_llr_kernel   System_AWGN_model.forward up to the decoder call (x_run_sn_polar/
//                     z_sys_model/awgn_model.py:33-41): random information bits
//                     (BinarySource, my_sn/trans/binary_source.py:18-19), polar encoding
//                     (x_run enc.py:30-43), QPSK Gray mapping (my_sn/trans/mapping.py:136-149),
//                     AWGN of variance no (my_sn/trans/channel/awgn.py:19-29), exact demapping to
//                     logits log P(b=1)/P(b=0) (mapping.py:151-241) -- one launch instead of ~15
//                     torch kernels over [bs, n/2] complex tensors.
//   count_errors_kernel  count_errors + count_block_errors (my_sn/sim.py:7-18) in one pass.
//
// Randomness: Philox4x32-10 (Salmon et al., SC'11; the Random123 reference rounds), keyed by the
// 64-bit seed, counter (row, iteration, domain|block).  The reference draws from torch's CPU
// generator; no GPU stream can reproduce that, so parity here is statistical (the decoder input
// has the reference's distribution), and the bit placement is pinned against a numpy Philox in
// the tests.  Info bit r of a row is bit (r mod 32) of stream word r/32 = component (r/32) mod 4
// of Philox block r/128 (domain 0); the noise of positions 4c .. 4c+3 is Philox block c of domain 1
// (Box-Muller on its four uniforms).
//
// Demapping: for Gray QPSK the reference's logsumexp over the constellation reduces exactly
// (mathematically) to logit_j = -2*sqrt(2)*y_j/no on the real/imaginary component y_j carrying
// code bit j (the terms of the other component cancel); computed in fp32 here, the reference's
// fp32 logsumexp rounds differently at the last ulp -- immaterial next to the noise draw.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../../include/polar_mi355x.h"
#include "plan.h"

namespace {

struct U4 {
    uint32_t x, y, z, w;
};

// Philox4x32-10 (Random123 philox4x32_R(10, ...)): 10 rounds, key bumped between rounds.
__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // the 64-bit products: one v_mad_u64_u32 each (2.2 ns) instead of v_mul_lo + v_mul_hi (4.0 ns,
        // tools/micro/mul_cost.hip)
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}


__device__ __forceinline__ uint32_t span_mask(int h) {
    switch (h) {
        case 1: return 0x55555555u;
        case 2: return 0x33333333u;
        case 4: return 0x0f0f0f0fu;
        case 8: return 0x00ff00ffu;
        default: return 0x0000ffffu;  // 16
    }
}

// Parallel bit deposit: bit i of x goes to the position of the i-th set bit of m (Hacker's
// Delight 7-5, "expand"), five log-steps instead of a loop over the set bits (no divergence).
__device__ __forceinline__ uint32_t expand_bits(uint32_t x, uint32_t m) {
    const uint32_t m0 = m;
    uint32_t mk = ~m << 1, mv[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        uint32_t mp = mk ^ (mk << 1);
        mp ^= mp << 2;
        mp ^= mp << 4;
        mp ^= mp << 8;
        mp ^= mp << 16;
        mv[i] = mp & m;
        m = (m ^ mv[i]) | (mv[i] >> (1 << i));
        mk &= ~mp;
    }
#pragma unroll
    for (int i = 4; i >= 0; --i) x = (x & ~mv[i]) | ((x << (1 << i)) & mv[i]);
    return x & m0;
}

// Philox block b of a row's stream in domain d (0: information bits, 1: noise)
__device__ __forceinline__ U4 stream_block(uint32_t k0, uint32_t k1, int64_t row, uint32_t it, uint32_t d, uint32_t b) {
    return philox(U4{(uint32_t)row, (uint32_t)(row >> 32), it, (d << 31) | b}, k0, k1);
}
__device__ __forceinline__ uint32_t comp(const U4& r, int c) { return c == 0 ? r.x : c == 1 ? r.y : c == 2 ? r.z : r.w; }

// Constants of the logit map: logit = a_s + rs * cos/sin(angle), a_s = +-scale/sqrt(2) by the code
// bit, rs = radius * scale * sqrt(no/2) (the radius' sqrt(2 ln 2) folded into rsc).
struct Logit {
    float a;    // scale / sqrt(2)
    float rsc;  // scale * sqrt(no / 2) * sqrt(2 ln 2)
};

// Four logits from one Philox block and the four code bits in bits 0..3 of `bits`.  Box-Muller on
// the hardware transcendentals (a noise draw, not a decoder value: only its distribution is
// specified):
//   radius  sqrt(-2 ln u) = sqrt(2 ln 2) sqrt(32 - log2 v'), v' = float(v | 1) in [1, 2^32], i.e.
//           u = v' 2^-32 in (0, 1] (tail to 6.66 sigma), v_log_f32 on a normal argument;
//   angle   v_sin / v_cos take revolutions and are periodic: the mantissa bits of v under the
//           exponent of 1.0 give 1 + t, t uniform in [0, 1), and sin(2 pi (1 + t)) = sin(2 pi t).
__device__ __forceinline__ float4 logits4(const U4& rnd, uint32_t bits, const Logit& lc) {
#if PL_AWGN_DIAG == 2
    const float c0 = (float)rnd.x, s0 = (float)rnd.y, c1 = (float)rnd.z, s1 = 1.0f, rs0 = lc.rsc, rs1 = lc.rsc;
#else
    const float rs0 = lc.rsc * __builtin_amdgcn_sqrtf(32.0f - __builtin_amdgcn_logf((float)(rnd.x | 1u)));
    const float rs1 = lc.rsc * __builtin_amdgcn_sqrtf(32.0f - __builtin_amdgcn_logf((float)(rnd.z | 1u)));
    const float t0 = __uint_as_float(0x3F800000u | (rnd.y >> 9)), t1 = __uint_as_float(0x3F800000u | (rnd.w >> 9));
    const float c0 = __builtin_amdgcn_cosf(t0), s0 = __builtin_amdgcn_sinf(t0);
    const float c1 = __builtin_amdgcn_cosf(t1), s1 = __builtin_amdgcn_sinf(t1);
#endif
    // (1 - 2 c) a: the code bit moved to the sign of a
    const uint32_t au = __float_as_uint(lc.a);
    const float a0 = __uint_as_float(au ^ ((bits << 31) & 0x80000000u));
    const float a1 = __uint_as_float(au ^ ((bits << 30) & 0x80000000u));
    const float a2 = __uint_as_float(au ^ ((bits << 29) & 0x80000000u));
    const float a3 = __uint_as_float(au ^ ((bits << 28) & 0x80000000u));
    return float4{__builtin_fmaf(rs0, c0, a0), __builtin_fmaf(rs0, s0, a1), __builtin_fmaf(rs1, c1, a2),
                  __builtin_fmaf(rs1, s1, a3)};
}

// A wave holds cpw = 64 / wpc codewords (wpc = max(1, n/32) lanes per codeword).  Three phases:
//   A  lane w < nq of a group: stream word w (32 information bits, ranks 32w .. 32w+31) -> LDS;
//   B  lane w of a group ("word layout", position 32w + j = bit j): x_w = the information bits
//      deposited at the word's information positions, then the XOR butterfly -> LDS;
//   C  the whole wave over the wave's rows in chunks of CH = min(4, n) positions ("chunk layout",
//      consecutive lanes -> consecutive chunks, so the fp32 rows are written as whole lines):
//      u rows from the stream words, logit rows from the code bits and one Philox block per chunk.
constexpr int kWordsPerWave = 256;
#ifndef PL_AWGN_DIAG
#define PL_AWGN_DIAG 0  // development only (tools/micro/producer_cost.hip): 1 no logit stores,
                        // 2 no noise (Philox + Box-Muller), 3 no Philox for the noise
#endif  // LDS words per wave: stream words (<= 128) + code words (64)
#if !PL_DEV && PL_AWGN_DIAG
#error "PL_AWGN_DIAG gives wrong results: development builds (-DPL_DEV=1) only"
#endif

__global__ __launch_bounds__(256) void awgn_llr_kernel(int64_t bs, int64_t row0, uint32_t k0, uint32_t k1, uint32_t it,
                                                       float no, const uint32_t* __restrict__ frozen_words, int n, int k,
                                                       float* __restrict__ u_out, float* __restrict__ llr_out,
                                                       uint32_t* __restrict__ ubits_out) {
    __shared__ uint32_t lds[4 * kWordsPerWave];
    const int wpc = n >= 32 ? n / 32 : 1, cpw = 64 / wpc, nb = n >= 32 ? 32 : n;
    const int nq = (k + 31) / 32;  // stream words per row
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t b0 = ((int64_t)blockIdx.x * 4 + wv) * cpw;  // first row of this wave
    uint32_t* sw = lds + wv * kWordsPerWave;                   // [cpw][nq] stream words
    uint32_t* cwd = sw + cpw * nq;                             // [cpw][wpc] code words
    const int g = lane / wpc, w = lane % wpc;
    const int64_t row = row0 + b0 + g;

    // A: stream words (rows past bs compute harmless values that are never stored)
    for (int q = w; q < nq; q += wpc) sw[g * nq + q] = comp(stream_block(k0, k1, row, it, 0, q >> 2), q & 3);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // B: information positions of this word (frozen bit 0), their first rank = information
    // positions in the group's earlier words (prefix sum over the group's lanes)
    const uint32_t live = nb == 32 ? 0xFFFFFFFFu : ((1u << nb) - 1u);
    const uint32_t info = ~frozen_words[w] & live;
    int base = 0;
    {
        int c = __popc(info), incl = c;
        for (int d = 1; d < wpc; d <<= 1) {
            const int o = __shfl_up(incl, d, 64);
            if (w >= d) incl += o;
        }
        base = incl - c;
    }
    uint32_t x = 0u;
    if (info) {
        const uint32_t* srow = sw + g * nq;
        const int q0 = base >> 5, sh = base & 31;
        const uint32_t lo = srow[q0];
        const uint32_t hi = q0 + 1 < nq ? srow[q0 + 1] : 0u;
        // the next (up to 32) information bits, deposited at the information positions in order
        x = expand_bits((uint32_t)((((uint64_t)hi << 32) | lo) >> sh), info);
    }
    for (int h = 1; h < nb; h <<= 1) x ^= (x >> h) & span_mask(h);  // x = u G_n (my_sn enc.py:85-96)
    for (int hw = 1; hw < wpc; hw <<= 1) {
        const uint32_t other = (uint32_t)__shfl_xor((int)x, hw, 64);
        if ((w & hw) == 0) x ^= other;
    }
    cwd[g * wpc + w] = x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    const int rows = bs - b0 < cpw ? (int)(bs - b0) : cpw;  // rows of this wave to store
    if (rows <= 0) return;
    // C1: u rows (BinarySource output, float32 0/1)
    if (u_out != nullptr && k > 0) {
        if ((k & 3) == 0 && ((reinterpret_cast<uintptr_t>(u_out) & 15) == 0)) {
            const int kq = k >> 2;
            for (int c = lane; c < rows * kq; c += 64) {
                const int r = c / kq, p = (c - r * kq) * 4;
                const uint32_t v = sw[r * nq + (p >> 5)] >> (p & 31);
                reinterpret_cast<float4*>(u_out + (b0 + r) * k)[p >> 2] =
                    float4{(float)(v & 1u), (float)((v >> 1) & 1u), (float)((v >> 2) & 1u), (float)((v >> 3) & 1u)};
            }
        } else {
            for (int c = lane; c < rows * k; c += 64) {
                const int r = c / k, p = c - r * k;
                u_out[(b0 + r) * k + p] = (float)((sw[r * nq + (p >> 5)] >> (p & 31)) & 1u);
            }
        }
    }
    // C1': the information bits packed, ceil(k/32) words per row (bit m of a row = bit m % 32 of
    // word m / 32: the stream words themselves, bits past k cleared) -- the decode+count kernel's
    // reference (pl_sc_decode_count), 1/32 of the fp32 rows' bytes
    if (ubits_out != nullptr && k > 0) {
        const uint32_t last = (k & 31) ? ((1u << (k & 31)) - 1u) : 0xFFFFFFFFu;
        for (int r = 0; r < rows; ++r)
            for (int q = lane; q < nq; q += 64) ubits_out[(b0 + r) * nq + q] = sw[r * nq + q] & (q == nq - 1 ? last : 0xFFFFFFFFu);
    }
    // C2: logits.  QPSK component of code bit j: (1 - 2 c_j)/sqrt(2) plus sqrt(no) * N(0, 1/2)
    // (awgn.py:24-29, utils.py:11-15); logit = -2 sqrt(2) y / no.  Chunk c of a row = positions
    // [CH c, CH c + CH) draws noise block c (4 uniforms -> 2 Box-Muller pairs).
    const float scale = -2.8284271f / no;
    const Logit lc{scale * 0.70710677f, scale * sqrtf(no) * 0.70710677f * 1.17741002f};  // sqrt(2 ln 2)
    const int CH = n >= 4 ? 4 : n, nch = n / CH, lnch = __builtin_ctz(nch);  // n is a power of two
    const bool vec = CH == 4 && ((reinterpret_cast<uintptr_t>(llr_out) & 15) == 0);
    if (vec && nch >= 64) {
        // rows outer (the row, hence the first Philox products, uniform across the wave), the
        // wave's lanes over the row's chunks: one 1-KiB float4 store per instruction
        for (int r = 0; r < rows; ++r) {
            const int64_t grow = row0 + b0 + r;
            const uint32_t* cw = cwd + r * wpc;
            float4* o = reinterpret_cast<float4*>(llr_out + (b0 + r) * n);
            for (int ch = lane; ch < nch; ch += 64) {
#if PL_AWGN_DIAG == 3
                const U4 rnd = U4{(uint32_t)ch * 0x9E3779B9u, (uint32_t)ch * 0x85EBCA6Bu, (uint32_t)ch * 0xC2B2AE35u,
                                  (uint32_t)ch * 0x27D4EB2Fu};
#else
                const U4 rnd = stream_block(k0, k1, grow, it, 1, (uint32_t)ch);
#endif
                const float4 l = logits4(rnd, cw[ch >> 3] >> ((ch & 7) * 4), lc);
#if PL_AWGN_DIAG == 1
                if (l.x + l.y + l.z + l.w != 1234.5f) continue;
#endif
                o[ch] = l;
            }
        }
        return;
    }
    for (int c = lane; c < rows * nch; c += 64) {
        const int r = c >> lnch, ch = c & (nch - 1), p = ch * CH;
        const U4 rnd = stream_block(k0, k1, row0 + b0 + r, it, 1, (uint32_t)ch);
        const float4 l = logits4(rnd, cwd[r * wpc + (p >> 5)] >> (p & 31), lc);
        float* o = llr_out + (b0 + r) * n + p;
        if (vec) {
            *reinterpret_cast<float4*>(o) = l;
        } else {
            const float lv[4] = {l.x, l.y, l.z, l.w};
            for (int i = 0; i < CH; ++i) o[i] = lv[i];
        }
    }
}

// Bit and block errors of a [rows, k] pair of 0/1 float tensors (exact comparisons, as
// tc.not_equal): a wave takes kRowsPerWave rows (their loads issued together, 16-byte loads when
// rows are 16-byte aligned), the block reduces in LDS, one pair of 64-bit atomics per block.
constexpr int kRowsPerWave = 8;

__global__ __launch_bounds__(256) void count_errors_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                           int64_t rows, int k, unsigned long long* __restrict__ counts) {
    __shared__ unsigned long long part[4][2];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t r0 = ((int64_t)blockIdx.x * 4 + wv) * kRowsPerWave;
    uint32_t bit_err = 0, blk_err = 0;
    const bool vec = (k & 3) == 0 && ((reinterpret_cast<uintptr_t>(a) & 15) == 0) &&
                     ((reinterpret_cast<uintptr_t>(b) & 15) == 0);
    if (vec) {
        const int kq = k >> 2;
        const float4* a4 = reinterpret_cast<const float4*>(a);
        const float4* b4 = reinterpret_cast<const float4*>(b);
#pragma unroll
        for (int r = 0; r < kRowsPerWave; ++r) {
            const int64_t row = r0 + r;
            uint32_t e = 0;
            if (row < rows) {
                for (int c = lane; c < kq; c += 64) {
                    const float4 x = a4[row * kq + c], y = b4[row * kq + c];
                    e += (x.x != y.x) + (x.y != y.y) + (x.z != y.z) + (x.w != y.w);
                }
            }
            bit_err += e;
            blk_err += __builtin_amdgcn_ballot_w64(e != 0) != 0 ? 1u : 0u;
        }
    } else {
        for (int r = 0; r < kRowsPerWave; ++r) {
            const int64_t row = r0 + r;
            uint32_t e = 0;
            if (row < rows)
                for (int i = lane; i < k; i += 64) e += a[row * k + i] != b[row * k + i] ? 1u : 0u;
            bit_err += e;
            blk_err += __builtin_amdgcn_ballot_w64(e != 0) != 0 ? 1u : 0u;
        }
    }
    for (int off = 32; off >= 1; off >>= 1) bit_err += __shfl_xor(bit_err, off, 64);
    if (lane == 0) {
        part[wv][0] = bit_err;
        part[wv][1] = blk_err;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long be = part[0][0] + part[1][0] + part[2][0] + part[3][0];
        const unsigned long long ke = part[0][1] + part[1][1] + part[2][1] + part[3][1];
        if (be) atomicAdd(&counts[0], be);
        if (ke) atomicAdd(&counts[1], ke);
    }
}

// counts[0..1] += sums of the [bit, block] error pairs the decode+count kernel stored per wave:
// kSumBlocks blocks, one pair of atomics each (no contention worth the name on the two counters)
constexpr int kSumBlocks = 64;

__global__ __launch_bounds__(256) void sum_pairs_kernel(const int32_t* __restrict__ part, int64_t pairs,
                                                        unsigned long long* __restrict__ counts) {
    __shared__ unsigned long long red[4][2];
    unsigned long long be = 0, ke = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < pairs; i += (int64_t)gridDim.x * 256) {
        be += (uint32_t)part[2 * i];
        ke += (uint32_t)part[2 * i + 1];
    }
    for (int off = 32; off >= 1; off >>= 1) {
        be += __shfl_xor(be, off, 64);
        ke += __shfl_xor(ke, off, 64);
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) {
        red[wv][0] = be;
        red[wv][1] = ke;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long b = red[0][0] + red[1][0] + red[2][0] + red[3][0];
        const unsigned long long e = red[0][1] + red[1][1] + red[2][1] + red[3][1];
        if (b) atomicAdd(&counts[0], b);
        if (e) atomicAdd(&counts[1], e);
    }
}

}  // namespace

namespace pl {
int launch_sum_pairs(const int32_t* part, int64_t pairs, int64_t* counts, hipStream_t stream) {
    if (pairs <= 0) return PL_OK;
    const int64_t need = (pairs + 255) / 256;
    const unsigned blocks = (unsigned)(need < kSumBlocks ? need : kSumBlocks);
    hipLaunchKernelGGL(sum_pairs_kernel, dim3(blocks), dim3(256), 0, stream, part, pairs,
                       reinterpret_cast<unsigned long long*>(counts));
    return check_hip(hipGetLastError(), "sum_pairs launch");
}
}  // namespace pl

extern "C" {

static int awgn_launch(const pl_plan* p, uint64_t seed, uint64_t iteration, int64_t row0, int64_t bs, float no,
                       float* u_out, uint32_t* ubits_out, float* llr_out, void* stream, const char* what) {
    if (!p || bs < 0 || row0 < 0 || (bs > 0 && !llr_out) || !(no > 0.0f) || (iteration >> 32) != 0) {
        pl::set_error(std::string(what) + ": bad arguments (no must be > 0, iteration < 2^32)");
        return PL_EINVAL;
    }
    if (int r = pl::check_device(p, static_cast<hipStream_t>(stream), what)) return r;
    if (bs == 0) return PL_OK;
    const int wpc = p->n >= 32 ? p->n / 32 : 1;
    const int64_t cpw = 64 / wpc;
    const int64_t blocks = ((bs + cpw - 1) / cpw + 3) / 4;
    if (blocks > 0x7fffffffLL) {
        pl::set_error(std::string(what) + ": batch too large for one launch");
        return PL_EINVAL;
    }
    hipLaunchKernelGGL(awgn_llr_kernel, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream), bs,
                       row0, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)iteration, no, p->d_frozen_words, p->n,
                       p->k, u_out, llr_out, ubits_out);
    return pl::check_hip(hipGetLastError(), what);
}

int pl_awgn_qpsk_llr(const pl_plan* p, uint64_t seed, uint64_t iteration, int64_t row0, int64_t bs, float no,
                     float* u_out, float* llr_out, void* stream) {
    return awgn_launch(p, seed, iteration, row0, bs, no, u_out, nullptr, llr_out, stream, "pl_awgn_qpsk_llr");
}

int pl_awgn_qpsk_llr_bits(const pl_plan* p, uint64_t seed, uint64_t iteration, int64_t row0, int64_t bs, float no,
                          uint32_t* ubits_out, float* llr_out, void* stream) {
    return awgn_launch(p, seed, iteration, row0, bs, no, nullptr, ubits_out, llr_out, stream,
                       "pl_awgn_qpsk_llr_bits");
}

int pl_count_errors(const float* a, const float* b, int64_t rows, int32_t k, int64_t* counts, void* stream) {
    if (rows < 0 || k < 0 || !counts || (rows > 0 && k > 0 && (!a || !b))) {
        pl::set_error("pl_count_errors: bad arguments");
        return PL_EINVAL;
    }
    if (rows == 0 || k == 0) return PL_OK;
    const int64_t blocks = (rows + 4 * kRowsPerWave - 1) / (4 * kRowsPerWave);
    if (blocks > 0x7fffffffLL) {
        pl::set_error("pl_count_errors: too many rows for one launch");
        return PL_EINVAL;
    }
    hipLaunchKernelGGL(count_errors_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       static_cast<hipStream_t>(stream), a, b, rows, k,
                       reinterpret_cast<unsigned long long*>(counts));
    return pl::check_hip(hipGetLastError(), "pl_count_errors launch");
}

}  // extern "C"
