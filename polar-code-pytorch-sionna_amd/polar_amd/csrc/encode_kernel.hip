// encode_kernel.hip -- polar encoder x = u * F2^{(x)m} (mod 2) for gfx950.
//
// Reference: x_run_sn_polar/polar/enc.py:30-43 computes c[:, info_pos] = u; (c @ G) % 2 as a
// dense fp32 [bs,n]x[n,n] GEMM (137 GFLOP at n=1024, bs=65536).  That is bit-identical to the
// XOR butterfly of my_sn/fec/polar/enc.py:85-96, which is what runs here: no MFMA, the work is
// n*log2(n) bit-XORs per codeword.  Each lane owns 32 consecutive positions as one packed word;
// butterflies with span < 32 are in-word shifts/masks, spans >= 32 are lane XOR-shuffles.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/polar_mi355x.h"
#include "plan.h"

namespace {

__device__ __forceinline__ uint32_t span_mask(int h) {
    // positions whose index bit log2(h) is 0 (the "upper" element of each butterfly)
    switch (h) {
        case 1: return 0x55555555u;
        case 2: return 0x33333333u;
        case 4: return 0x0f0f0f0fu;
        case 8: return 0x00ff00ffu;
        default: return 0x0000ffffu;  // 16
    }
}

__global__ __launch_bounds__(256) void encode_kernel(const float* __restrict__ u, int64_t bs, float* __restrict__ cw,
                                                     const int32_t* __restrict__ info_rank, int n, int k) {
    const int wpc = n >= 32 ? n / 32 : 1;  // lanes (words) per codeword
    const int cpw = 64 / wpc;              // codewords per wave
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t row = wave * cpw + lane / wpc;
    const int w = lane % wpc;
    const bool valid = row < bs;
    const int nb = n >= 32 ? 32 : n;  // positions in this word
    uint32_t x = 0u;
    if (valid) {
        const float* ur = u + row * k;
        for (int b = 0; b < nb; ++b) {
            const int r = info_rank[w * 32 + b];
            if (r >= 0 && ur[r] != 0.0f) x |= 1u << b;
        }
    }
    for (int h = 1; h < nb; h <<= 1) x ^= (x >> h) & span_mask(h);
    for (int hw = 1; hw < wpc; hw <<= 1) {
        const uint32_t other = (uint32_t)__shfl_xor((int)x, hw, 64);
        if ((w & hw) == 0) x ^= other;
    }
    if (valid) {
        float* o = cw + row * n + w * 32;
        for (int b = 0; b < nb; ++b) o[b] = ((x >> b) & 1u) ? 1.0f : 0.0f;
    }
}

}  // namespace

namespace pl {
int launch_encode(const pl_plan* p, const float* u, int64_t bs, float* cw, hipStream_t st) {
    if (bs == 0) return PL_OK;
    const int wpc = p->n >= 32 ? p->n / 32 : 1;
    const int64_t cpw = 64 / wpc;
    const int64_t waves = (bs + cpw - 1) / cpw;
    const int64_t blocks = (waves + 3) / 4;
    hipLaunchKernelGGL(encode_kernel, dim3((unsigned)blocks), dim3(256), 0, st, u, bs, cw, p->d_info_rank, p->n, p->k);
    return check_hip(hipGetLastError(), "encode launch");
}
}  // namespace pl
