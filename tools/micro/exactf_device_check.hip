// Development aid (GPU box): the device exp_cr / log_cr of csrc/exactf.h (the code the exact-f SC
// kernels run, tables in LDS) on EVERY fp32 bit pattern of their domains, compared bit for bit with
// the host mirror of tools/micro/exactf_rounding.cpp -- which tools/micro/exactf_exhaustive.cpp
// checks against the true values on the same domains (profiles/r05n_exactf_exhaustive.txt).  Equal
// everywhere => the device forms are correctly rounded wherever the mirror is.
//   hipcc --offload-arch=gfx950 -O2 -fopenmp -o tools/micro/exactf_device_check tools/micro/exactf_device_check.hip
#include "../../polar-code-pytorch-sionna_amd/polar_amd/csrc/exactf.h"
#define EXACTF_NO_MAIN
#include "exactf_rounding.cpp"

#include <omp.h>

__global__ __launch_bounds__(256) void k_eval(uint32_t start, uint32_t count, uint32_t* oe, uint32_t* ol) {
    plx::load_tables(threadIdx.x, blockDim.x);  // every thread reaches the barrier inside
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < count) {
        const float x = __uint_as_float(start + i);
        oe[i] = __float_as_uint(plx::exp_cr(x));  // (outside |x| <= 87 the value is not used)
        ol[i] = __float_as_uint(plx::log_cr(x));  // (outside the positive normals: not used)
    }
}

int main() {
    constexpr uint32_t kChunk = 1u << 26;
    uint32_t *de = nullptr, *dl = nullptr;
    if (hipMalloc(&de, kChunk * 4ull) != hipSuccess || hipMalloc(&dl, kChunk * 4ull) != hipSuccess) return 1;
    uint32_t* he = (uint32_t*)malloc(kChunk * 4ull);
    uint32_t* hl = (uint32_t*)malloc(kChunk * 4ull);
    long ne = 0, nl = 0, be = 0, bl = 0;
    uint32_t fe = 0, fl = 0;
    for (uint64_t start = 0; start < (1ull << 32); start += kChunk) {
        hipLaunchKernelGGL(k_eval, dim3(kChunk / 256), dim3(256), 0, 0, (uint32_t)start, kChunk, de, dl);
        if (hipMemcpy(he, de, kChunk * 4ull, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(hl, dl, kChunk * 4ull, hipMemcpyDeviceToHost) != hipSuccess) {
            fprintf(stderr, "device error at chunk 0x%08llx\n", (unsigned long long)start);
            return 2;
        }
#pragma omp parallel for schedule(static) reduction(+ : ne, nl, be, bl)
        for (int64_t i = 0; i < (int64_t)kChunk; ++i) {
            const uint32_t b = (uint32_t)start + (uint32_t)i;
            float x;
            memcpy(&x, &b, 4);
            if ((b & 0x7fffffffu) <= 0x42ae0000u) {  // |x| <= 87
                ++ne;
                const float h = exp_cr(x);
                uint32_t hb;
                memcpy(&hb, &h, 4);
                if (hb != he[i]) {
                    ++be;
#pragma omp critical
                    if (!fe) fe = b;
                }
            }
            if (b >= 0x00800000u && b <= 0x7f7fffffu) {  // positive normals
                ++nl;
                const float h = log_cr(x);
                uint32_t hb;
                memcpy(&hb, &h, 4);
                if (hb != hl[i]) {
                    ++bl;
#pragma omp critical
                    if (!fl) fl = b;
                }
            }
        }
    }
    printf("device exp_cr vs host mirror: %ld fp32 arguments (|x| <= 87), %ld differ (first 0x%08x)\n", ne, be, fe);
    printf("device log_cr vs host mirror: %ld fp32 arguments (positive normals), %ld differ (first 0x%08x)\n", nl, bl, fl);
    free(he);
    free(hl);
    (void)hipFree(de);
    (void)hipFree(dl);
    return (be || bl) ? 3 : 0;
}
