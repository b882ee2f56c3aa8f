// clock_kernel.hip -- shader-clock probe for gfx950 (pl_clock_probe, include/polar_mi355x.h).
//
// One wave runs a dependent chain of `iters` VALU adds and reads both of the chip's counters
// around it: s_memtime counts shader-clock cycles, s_memrealtime the constant 100 MHz reference.
// Their ratio is the clock the CU ran at during the chain (MI355X_MICROARCH.md: DVFS moves it by up
// to ~12 % from box to box and with load).  bench.py launches the probe on the decode stream right
// before and right after its timed region, so a throughput number carries the clock it ran at
// (tools/micro/chain_latency.hip measured the same pair: 2.4017 GHz under a busy loop).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/polar_mi355x.h"
#include "plan.h"

namespace {

__global__ __launch_bounds__(64) void clock_kernel(uint64_t* __restrict__ ticks, int iters) {
    float x = (float)threadIdx.x * 0.001f;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) asm volatile("v_add_f32 %0, %0, %0" : "+v"(x));
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {  // one lane's vector stores
        ticks[0] = t1 - t0;
        ticks[1] = r1 - r0;
        ticks[2] = (uint64_t)__float_as_uint(x);  // keeps the chain observable
    }
}

}  // namespace

extern "C" int pl_clock_probe(uint64_t* ticks, int32_t iters, void* hip_stream) {
    if (ticks == nullptr || iters < 1) {
        pl::set_error("pl_clock_probe: null ticks or iters < 1");
        return PL_EINVAL;
    }
    hipLaunchKernelGGL(clock_kernel, dim3(1), dim3(64), 0, (hipStream_t)hip_stream, ticks, (int)iters);
    return pl::check_hip(hipGetLastError(), "pl_clock_probe launch");
}
