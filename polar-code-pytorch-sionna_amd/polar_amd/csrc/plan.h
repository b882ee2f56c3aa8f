// plan.h -- internal (non-ABI) plan layout shared by the HIP translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

struct pl_plan {
    int32_t n = 0, log_n = 0, k = 0, list_size = 1, f_mode = 0;
    float llr_max = 30.0f;
    uint32_t flags = 0;
    int32_t device = -1;                 // HIP device the plan's tables and module live on
    // Device-resident, immutable after pl_plan_create:
    uint32_t* d_frozen_words = nullptr;  // ceil(n/32) words, bit (i&31) of word i>>5 = frozen[i]
    uint32_t* d_rate0_words = nullptr;   // n-1 node flags: bit OFF(s)+(p>>s), OFF(s)=n-(n>>(s-1))
    uint32_t* d_type_words = nullptr;    // 4 x type_stride words: rate-0 / rate-1 / repetition / SPC
    int32_t type_stride = 64;            //   node flags, same bit indexing as d_rate0_words
    int32_t* d_info_pos = nullptr;       // k ascending information positions
    int32_t* d_info_rank = nullptr;      // n entries: rank among info positions, -1 if frozen
    // Code-specialised SC kernel (jit.cpp / sc_static.h); null module = generic kernel.
    int32_t* d_info_loc = nullptr;       // k (padded to 4): (lane-in-group << 8) | slot of info bit m
    hipModule_t sc_module = nullptr;
    hipFunction_t sc_fn_f32 = nullptr, sc_fn_u8 = nullptr;
    hipFunction_t sc_fn_cnt = nullptr;   // decode + error count (pl_sc_decode_count); null if absent
    hipFunction_t sc_fn_sim = nullptr;   // producer + decode + count (pl_sc_sim_count); null if absent
    std::string kernel_path;             // code object the module came from
    int32_t crc_deg = 0;                 // SCL CRC-aided pick: degree (0 = none) and generator
    uint32_t crc_g = 0;                  //   mask without the leading term
    int32_t sc_log_g = 0;                // specialised kernel: log2(lanes per codeword) it was built for
    int32_t sc_waves = 4;                // waves per work-group of the specialised kernel (pl_sc_waves)
    int32_t sc_persistent = 0;           // kernel walks batches with a grid stride (grid capped)
    int32_t resident_blocks = 0;         // 256-thread blocks resident at 2 waves/SIMD on the device
};

namespace pl {
void set_error(const std::string& msg);
int check_hip(hipError_t e, const char* what);

// Launchers (return PL_* codes); defined in sc_kernel.hip / scl_kernel.hip / encode_kernel.hip
int launch_sc(const pl_plan* plan, const float* llr, int64_t bs, void* out, int out_kind,
              hipStream_t stream);
size_t scl_workspace_size(const pl_plan* plan, int64_t bs);
int launch_scl(const pl_plan* plan, const float* llr, int64_t bs, void* out, int out_kind,
               double* out_pm, void* ws, size_t ws_bytes, hipStream_t stream);
// SCL "register subtree" kernel (scl_tree_kernel.hip); launch_scl dispatches to it when eligible
bool scl_tree_eligible(const pl_plan* plan);
// Whether some SCL kernel decodes this plan (sets the error string when not); scl_kernel.hip
bool scl_supported(const pl_plan* plan);
int launch_scl_tree(const pl_plan* plan, const float* llr, int64_t bs, void* out, int out_kind, double* out_pm,
                    void* ws, size_t ws_bytes, hipStream_t stream);
// device scratch the subtree kernel uses (the exact-f leftmost-chain cache), 0 if none
size_t scl_tree_workspace_size(const pl_plan* plan, int64_t bs);
// PL_OK when the stream (NULL: the current device) is on the plan's device, else PL_EINVAL; capi.cpp
int check_device(const pl_plan* plan, hipStream_t stream, const char* what);
int launch_encode(const pl_plan* plan, const float* u, int64_t bs, float* cw, hipStream_t stream);

// Code-specialised SC kernels (jit.cpp)
int attach_static(pl_plan* plan, const uint8_t* frozen_mask, bool allow_compile);
void detach_static(pl_plan* plan);
int launch_sc_static(const pl_plan* plan, const float* llr, int64_t bs, void* out, int out_kind,
                     hipStream_t stream);
// decode + count (specialised kernel's pl_sc_static_cnt): per-wave [bit, block] error pairs into
// part (int32[2 * waves]), waves = sc_count_waves(plan, bs)
int64_t sc_count_waves(const pl_plan* plan, int64_t bs);
int launch_sc_static_count(const pl_plan* plan, const float* llr, int64_t bs, const uint32_t* ref, int32_t* part,
                           hipStream_t stream);
int launch_sc_static_sim(const pl_plan* plan, uint64_t seed, uint64_t iteration, int64_t row0, int64_t bs, float no,
                         int32_t* part, float* llr_dump, float* u_dump, hipStream_t stream);
// counts[0..1] += the sums of the [bit, block] pairs of part (channel_kernel.hip)
int launch_sum_pairs(const int32_t* part, int64_t pairs, int64_t* counts, hipStream_t stream);
}  // namespace pl
