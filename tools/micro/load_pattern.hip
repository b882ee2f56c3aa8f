// Microbenchmark (development aid): HBM read rate of the SC kernel's channel-load shape vs
// alternatives, on a [65536, 1024] fp32 array (256 MiB) + a [65536, 512] fp32 output (128 MiB),
// 256-thread blocks, 4 codewords per wave (as pl_sc_static at n = 1024).
//  A: residue layout, global_load_dword: lane (c, r) reads row c, elements j*16 + r (4 rows x 64 B
//     per instruction, 64 instructions per wave)
//  B: row-contiguous dword: instruction j reads 256 contiguous bytes of one row
//  C: dwordx4: lane reads 16 B; an instruction covers 4 rows x 256 B
//  D: dwordx4: an instruction covers 1 KiB of one row
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int N = 1024, K = 512;
constexpr long BS = 65536;

template <int MODE, int MINW, int NT = 0>
__global__ __launch_bounds__(256, MINW) void k(const float* __restrict__ llr, float* __restrict__ out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long cw0 = ((long)blockIdx.x * 4 + wave) * 4;
    float acc = 0.f;
    if constexpr (MODE == 0) {
        const float* ch = llr + (cw0 + (lane >> 4)) * N + (lane & 15);
        float v[64];
#pragma unroll
        for (int j = 0; j < 64; ++j) v[j] = (NT & 2) ? __builtin_nontemporal_load(ch + j * 16) : ch[j * 16];
#pragma unroll
        for (int j = 0; j < 64; ++j) acc += v[j];
    } else if constexpr (MODE == 1) {
        float v[64];
#pragma unroll
        for (int j = 0; j < 64; ++j) v[j] = llr[(cw0 + (j >> 4)) * N + (j & 15) * 64 + lane];
#pragma unroll
        for (int j = 0; j < 64; ++j) acc += v[j];
    } else if constexpr (MODE == 2) {
        const float4* ch = reinterpret_cast<const float4*>(llr + (cw0 + (lane >> 4)) * N) + (lane & 15);
        float4 v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = ch[j * 16];
#pragma unroll
        for (int j = 0; j < 16; ++j) acc += v[j].x + v[j].y + v[j].z + v[j].w;
    } else {
        float4 v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = reinterpret_cast<const float4*>(llr + (cw0 + (j >> 2)) * N)[(j & 3) * 64 + lane];
#pragma unroll
        for (int j = 0; j < 16; ++j) acc += v[j].x + v[j].y + v[j].z + v[j].w;
    }
    // output: 4 rows x 2 KiB, float4 per lane (as the SC kernel's emit)
    float4 o = {acc, acc, acc, acc};
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int it = 0; it < 2; ++it) {
            typedef float v4f __attribute__((ext_vector_type(4)));
            v4f* p = reinterpret_cast<v4f*>(out + (cw0 + g) * K) + lane + 64 * it;
            const v4f ov = {o.x, o.y, o.z, o.w};
            if constexpr (NT & 1) __builtin_nontemporal_store(ov, p);
            else *p = ov;
        }
}

template <class F>
float run(F kern, float* const* in, float* const* out, int nbuf) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int blocks = BS / 16;
    for (int r = 0; r < 20; ++r) kern<<<blocks, 256>>>(in[r % nbuf], out[r % nbuf]);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 96; ++r) kern<<<blocks, 256>>>(in[r % nbuf], out[r % nbuf]);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 96;
}

int main() {
    // 3 input and output buffers: rotating through them (1.15 GB) defeats the 256 MB Infinity
    // Cache; the same buffer every launch lets the input stay partly resident there
    float *in[3], *out[3];
    for (int b = 0; b < 3; ++b) {
        (void)hipMalloc(&in[b], BS * N * 4);
        (void)hipMalloc(&out[b], BS * K * 4);
        (void)hipMemset(in[b], 0, BS * N * 4);
    }
    const double bytes = BS * (N + K) * 4.0;
    struct { const char* n; void (*k)(const float*, float*); } ks[] = {
        {"A residue dword (3 w/SIMD)", k<0, 3>}, {"A residue dword (2 w/SIMD)", k<0, 2>},
        {"A + nt stores", k<0, 3, 1>}, {"A + nt loads", k<0, 3, 2>}, {"A + nt loads and stores", k<0, 3, 3>},
        {"B row-contig dword", k<1, 3>}, {"C dwordx4 4 rows", k<2, 3>}, {"D dwordx4 1 row", k<3, 3>}};
    for (auto& x : ks) {
        const float same = run(x.k, in, out, 1), rot = run(x.k, in, out, 3);
        printf("%-30s same buffers %.4f ms %.2f TB/s | rotating 3 buffers %.4f ms %.2f TB/s\n", x.n, same,
               bytes / same / 1e9, rot, bytes / rot / 1e9);
    }
    return 0;
}
