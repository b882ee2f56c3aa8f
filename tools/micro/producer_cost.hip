// Microbenchmark (development aid): where the fused LLR producer's time goes (awgn_llr_kernel of
// csrc/channel_kernel.hip, included here and built once per PL_AWGN_DIAG variant:
//   0 as shipped, 1 no logit stores, 2 no noise draw, 3 no Philox for the noise)
// at (k=512, n=1024), bs = 65536, the packed-bits output of pl_awgn_qpsk_llr_bits; plus a kernel that
// only writes the same 256 MiB of logits (float4 per lane, 1 KiB per store instruction).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPL_DEV=1 -DPL_AWGN_DIAG=N tools/micro/producer_cost.hip -o ...
#include <cstdio>
#include <string>

#include "../../polar-code-pytorch-sionna_amd/polar_amd/csrc/channel_kernel.hip"

namespace pl {
void set_error(const std::string&) {}
int check_hip(hipError_t e, const char*) { return e == hipSuccess ? 0 : -1; }
int check_device(const pl_plan*, hipStream_t, const char*) { return 0; }
}  // namespace pl

__global__ __launch_bounds__(256) void store_only(float* __restrict__ out, long n4) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256)
        reinterpret_cast<float4*>(out)[i] = float4{(float)i, 1.f, 2.f, 3.f};
}

int main() {
    constexpr int N = 1024, K = 512;
    constexpr long BS = 65536;
    uint32_t fw[N / 32];
    for (int w = 0; w < N / 32; ++w) fw[w] = w < N / 64 ? 0xFFFFFFFFu : 0u;  // first half frozen
    uint32_t* d_fw;
    float* llr;
    uint32_t* bits;
    hipMalloc(&d_fw, sizeof(fw));
    hipMemcpy(d_fw, fw, sizeof(fw), hipMemcpyHostToDevice);
    hipMalloc(&llr, BS * N * 4);
    hipMalloc(&bits, BS * (K / 32) * 4);
    const int blocks = (int)((BS / 2 + 3) / 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto prod = [&](int it) {
        hipLaunchKernelGGL(awgn_llr_kernel, dim3(blocks), dim3(256), 0, 0, BS, 0L, 42u, 0u, (uint32_t)it, 0.5f, d_fw, N,
                           K, nullptr, llr, bits);
    };
    auto store = [&](int) { hipLaunchKernelGGL(store_only, dim3(8192), dim3(256), 0, 0, llr, BS * N / 4); };
    for (int i = 0; i < 200; ++i) prod(i);
    hipDeviceSynchronize();
    for (int round = 0; round < 3; ++round) {
        for (int which = 0; which < 2; ++which) {
            const int reps = 100;
            hipEventRecord(e0, 0);
            for (int i = 0; i < reps; ++i) which == 0 ? prod(i) : store(i);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("diag=%d %-14s %.4f ms per launch\n", PL_AWGN_DIAG, which == 0 ? "producer" : "store_only",
                   ms / reps);
        }
    }
    return 0;
}
