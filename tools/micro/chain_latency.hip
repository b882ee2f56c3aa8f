// Dependent-chain latency of single instruction forms on gfx950, ONE wave on the whole GPU (one
// 64-thread block), and the floor of back-to-back launches of an empty kernel -- the inputs of the
// critical-path bound of tools/isa_chain.py.  Each chain is ITER dependent
// instructions (the form's result feeds its next instance); DPP forms carry the s_nop 1 the ISA
// requires after a VALU write of the DPP source, as the kernels do.  Prints ns per instruction.
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/chain_latency tools/micro/chain_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 4096;
#define KC(NAME, DECL, BODY, USE)                                                  \
    __global__ __launch_bounds__(64) void NAME(float* out, float a, unsigned long long* tm) { \
        DECL;                                                                      \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                \
        for (int it = 0; it < ITER / 8; ++it) {                                    \
            BODY BODY BODY BODY BODY BODY BODY BODY                                \
        }                                                                          \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                \
        out[blockIdx.x * 64 + threadIdx.x] = USE;                                  \
        if (threadIdx.x == 0) *tm = t1 - t0;                                       \
    }
#define DF float x = threadIdx.x * 0.001f; const float av = a
#define DU unsigned x = threadIdx.x; const unsigned av = __float_as_uint(a)
KC(c_add_f32, DF, asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(av));, x)
KC(c_bitop3, DU, asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x6c" : "+v"(x) : "v"(av));, (float)x)
KC(c_min3, DF, asm volatile("v_min3_f32 %0, |%0|, |%1|, %1" : "+v"(x) : "v"(av));, x)
KC(c_med3, DF, asm volatile("v_med3_f32 %0, -|%0|, %1, |%0|" : "+v"(x) : "v"(av));, x)
KC(c_xor, DU, asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(av));, (float)x)
KC(c_alignbit, DU, asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(av));, (float)x)
KC(c_dpp_add, DF, asm volatile("s_nop 1\n v_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(x));, x)
KC(c_dpp_mov, DU, asm volatile("s_nop 1\n v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(x));, (float)x)
KC(c_cmp_cnd, DF, asm volatile("v_cmp_eq_f32 vcc, 0, %0\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(av) : "vcc");, x)
KC(c_fma_f64, double x = threadIdx.x * 0.001; const double av = a, asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x) : "v"(av));, (float)x)
KC(c_pk_add, float2 x = make_float2(threadIdx.x * 0.001f, a),
   asm volatile("v_pk_add_f32 %0, %0, %0" : "+v"(*reinterpret_cast<double*>(&x)));, x.x + x.y)
// LDS round trip: the loaded value is the next address (ds_read_b32 -> ds_read_b32)
__global__ __launch_bounds__(64) void c_lds(float* out, float a, unsigned long long* tm) {
    __shared__ unsigned buf[64];
    buf[threadIdx.x] = (threadIdx.x * 4u) ^ (a > 2.f ? 4u : 0u);
    __syncthreads();
    unsigned x = threadIdx.x * 4u;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; ++it) asm volatile("ds_read_b32 %0, %0\n s_waitcnt lgkmcnt(0)" : "+v"(x));
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = (float)x;
    if (threadIdx.x == 0) *tm = t1 - t0;
}
// ds_bpermute round trip
__global__ __launch_bounds__(64) void c_bperm(float* out, float a, unsigned long long* tm) {
    int x = threadIdx.x * 4;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; ++it) asm volatile("ds_bpermute_b32 %0, %0, %0\n s_waitcnt lgkmcnt(0)" : "+v"(x));
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = (float)x + a;
    if (threadIdx.x == 0) *tm = t1 - t0;
}
__global__ __launch_bounds__(64) void c_empty(float* out, float a, unsigned long long* tm) {
    if (a > 1e30f) out[threadIdx.x] = a + (float)(tm != nullptr);
}
// one dependent global load chain (pointer chasing in a 4 MB ring at word offset kRing of the
// buffer, L2-resident after the first pass; the other kernels write words [0, 65536) only)
constexpr unsigned kRing = 1u << 21, kRingWords = 1u << 20;
__global__ __launch_bounds__(64) void c_gload(float* out, float a, unsigned long long* tm) {
    const unsigned* p = reinterpret_cast<const unsigned*>(out) + kRing;
    unsigned x = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER / 16; ++it) x = __builtin_nontemporal_load(p + (x & (kRingWords - 1))) ^ (unsigned)(a > 1e30f);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[(1 << 20) + threadIdx.x] = (float)x + a;
    if (threadIdx.x == 0) *tm = t1 - t0;
}

// s_memtime and s_memrealtime across one long dependent chain of one wave
__global__ __launch_bounds__(64) void c_clock(float* out, float a, unsigned long long* tm) {
    float x = threadIdx.x * 0.001f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < 64 * ITER; ++it) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(a));
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) {
        tm[0] = t1 - t0;
        tm[1] = r1 - r0;
    }
}

typedef void (*Kern)(float*, float, unsigned long long*);

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);      \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

int main() {
    const struct {
        const char* name;
        Kern k;
        int n;
    } ks[] = {{"v_add_f32", c_add_f32, ITER}, {"v_bitop3_b32", c_bitop3, ITER}, {"v_min3_f32", c_min3, ITER},
              {"v_med3_f32", c_med3, ITER}, {"v_xor_b32", c_xor, ITER}, {"v_alignbit_b32", c_alignbit, ITER},
              {"s_nop1+v_add_f32_dpp", c_dpp_add, ITER}, {"s_nop1+v_mov_b32_dpp", c_dpp_mov, ITER},
              {"v_cmp+v_cndmask", c_cmp_cnd, ITER}, {"v_fma_f64", c_fma_f64, ITER}, {"v_pk_add_f32", c_pk_add, ITER},
              {"ds_read_b32", c_lds, ITER}, {"ds_bpermute_b32", c_bperm, ITER}, {"global_load (L2)", c_gload, ITER / 16}};
    float* buf;
    if (hipMalloc(&buf, (size_t)(1 << 22) * sizeof(float)) != hipSuccess) return 1;
    {  // pointer-chase ring at word kRing: x -> (x * 4093 + 64) mod 2^20 (indices masked in the kernel too)
        unsigned* h = new unsigned[kRingWords];
        for (unsigned i = 0; i < kRingWords; ++i) h[i] = (i * 4093u + 64u) & (kRingWords - 1u);
        CK(hipMemcpy(buf + kRing, h, (size_t)kRingWords * 4, hipMemcpyHostToDevice));
        delete[] h;
    }
    unsigned long long* tmd;
    if (hipMalloc(&tmd, 64) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 200; ++w)  // settle the clock (load on all CUs)
        hipLaunchKernelGGL(c_add_f32, dim3(1024), dim3(64), 0, 0, buf, 1.0001f, tmd);
    (void)hipDeviceSynchronize();
    for (const auto& k : ks) {
        float best = 1e30f;
        unsigned long long cyc = ~0ull;
        for (int r = 0; r < 7; ++r) {
            // keep the clock up: a full-chip launch before each single-wave one
            hipLaunchKernelGGL(c_add_f32, dim3(1024), dim3(64), 0, 0, buf, 1.0001f, tmd + 1);
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, buf, 1.0001f, tmd);
            CK(hipGetLastError());
            (void)hipEventRecord(e1);
            CK(hipEventSynchronize(e1));
            float t = 0;
            (void)hipEventElapsedTime(&t, e0, e1);
            best = t < best ? t : best;
            unsigned long long c = 0;
            CK(hipMemcpy(&c, tmd, 8, hipMemcpyDeviceToHost));
            cyc = c < cyc ? c : cyc;
        }
        printf("%-24s %7.2f s_memtime cycles per dependent instruction (one wave; %.4f ms incl. launch)\n",
               k.name, (double)cyc / k.n, best);
    }
    // launch floor: N back-to-back launches of an empty kernel, 256 one-wave blocks (configs_1's grid)
    for (int blocks : {1, 256, 1024}) {
        const int N = 2000;
        for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(c_empty, dim3(blocks), dim3(64), 0, 0, buf, 1.0f, tmd);
        (void)hipEventRecord(e0);
        for (int i = 0; i < N; ++i) hipLaunchKernelGGL(c_empty, dim3(blocks), dim3(64), 0, 0, buf, 1.0f, tmd);
        CK(hipGetLastError());
        (void)hipEventRecord(e1);
        CK(hipEventSynchronize(e1));
        float t = 0;
        (void)hipEventElapsedTime(&t, e0, e1);
        printf("empty kernel, %4d blocks   %.3f us per back-to-back launch\n", blocks, t * 1e3 / N);
    }
    // the s_memtime clock against s_memrealtime (100 MHz): one long single-wave chain, clock up
    {
        hipLaunchKernelGGL(c_add_f32, dim3(1024), dim3(64), 0, 0, buf, 1.0001f, tmd + 1);
        hipLaunchKernelGGL(c_clock, dim3(1), dim3(64), 0, 0, buf, 1.0001f, tmd);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        unsigned long long c[2] = {0, 0};
        CK(hipMemcpy(c, tmd, 16, hipMemcpyDeviceToHost));
        printf("s_memtime clock: %.4f GHz (%llu cycles in %llu ticks of s_memrealtime at 100 MHz)\n",
               (double)c[0] / ((double)c[1] * 10.0), c[0], c[1]);
    }
    (void)hipFree(buf);
    return 0;
}
