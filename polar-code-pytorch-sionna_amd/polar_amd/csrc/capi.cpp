// capi.cpp -- extern "C" boundary of libpolar_mi355x.so (declared in include/polar_mi355x.h).
//
// Plan construction mirrors the reference decoder constructors:
//   SC_Dec.__init__  x_run_sn_polar/polar/polar_sc.py:10-32  (k = n - |frozen|, sorted info_pos)
//   SCL_Dec.__init__ x_run_sn_polar/polar/polar_scl.py:13-42 (n, list_size powers of two)
// and precomputes, once, everything the kernels query: the frozen bitmask, the rate-0 node
// bitmask (all-frozen subtrees, skipped exactly), info_pos and the inverse rank table.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/polar_mi355x.h"
#include "plan.h"

namespace {
thread_local std::string g_last_error;
}

namespace pl {
void set_error(const std::string& msg) { g_last_error = msg; }
int check_hip(hipError_t e, const char* what) {
    if (e == hipSuccess) return PL_OK;
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return PL_EHIP;
}
// A plan's tables (hipMalloc) and specialised kernel module (hipModuleLoadData) belong to the
// device that was current at pl_plan_create; launching it on another device's stream would hand
// that device foreign pointers and a foreign module.
int check_device(const pl_plan* p, hipStream_t st, const char* what) {
    int dev = -1;
    const hipError_t e = st ? hipStreamGetDevice(st, &dev) : hipGetDevice(&dev);
    if (e != hipSuccess) return check_hip(e, what);
    if (dev != p->device) {
        set_error(std::string(what) + ": the plan was created on device " + std::to_string(p->device) +
                  " but the stream is on device " + std::to_string(dev) + " (plans are device-bound)");
        return PL_EINVAL;
    }
    return PL_OK;
}
}  // namespace pl

namespace {

int ilog2_exact(int n) {
    int s = 0;
    while ((1 << s) < n) ++s;
    return ((1 << s) == n) ? s : -1;
}

template <typename T>
int upload(T** dst, const std::vector<T>& src) {
    if (src.empty()) return PL_OK;
    int r = pl::check_hip(hipMalloc(reinterpret_cast<void**>(dst), src.size() * sizeof(T)), "hipMalloc(plan)");
    if (r) return r;
    return pl::check_hip(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy(plan)");
}

void free_plan(pl_plan* p) {
    if (!p) return;
    // release on the plan's own device (the module and the tables live there)
    int cur = -1;
    const bool switch_dev = hipGetDevice(&cur) == hipSuccess && p->device >= 0 && cur != p->device &&
                            hipSetDevice(p->device) == hipSuccess;
    pl::detach_static(p);
    (void)hipFree(p->d_info_loc);
    (void)hipFree(p->d_frozen_words);
    (void)hipFree(p->d_rate0_words);
    (void)hipFree(p->d_type_words);
    (void)hipFree(p->d_info_pos);
    (void)hipFree(p->d_info_rank);
    if (switch_dev) (void)hipSetDevice(cur);
    delete p;
}

}  // namespace

extern "C" {

const char* pl_last_error_string(void) { return g_last_error.c_str(); }
const char* pl_version(void) { return "polar_mi355x 0.2.0 (gfx950)"; }

int pl_plan_create(pl_plan** out, int32_t n, const uint8_t* frozen_mask, int32_t list_size, int32_t f_mode,
                   float llr_max, uint32_t flags) {
    if (!out || !frozen_mask) {
        pl::set_error("pl_plan_create: null pointer");
        return PL_EINVAL;
    }
    *out = nullptr;
    const int log_n = ilog2_exact(n);
    if (log_n < 1 || log_n > 11) {
        pl::set_error("pl_plan_create: n must be a power of two in [2, 2048]");
        return PL_EINVAL;
    }
    if (list_size < 1 || list_size > 32 || (list_size & (list_size - 1))) {
        pl::set_error("pl_plan_create: list_size must be a power of two in [1, 32]");
        return PL_EINVAL;
    }
    if (f_mode != PL_F_MINSUM && f_mode != PL_F_EXACT) {
        pl::set_error("pl_plan_create: unknown f_mode");
        return PL_EINVAL;
    }
    if (!(llr_max > 0.0f) || (list_size > 1 && !(llr_max <= 700.0f))) {
        // list decoders: the metric penalty log(1 + exp(z)) is evaluated for |z| <= 700
        // (softplus.h); beyond that the reference's float64 exp overflows anyway
        pl::set_error("pl_plan_create: llr_max must be positive (and <= 700 for list decoding)");
        return PL_EINVAL;
    }
    pl_plan* p = new pl_plan();
    p->n = n;
    p->log_n = log_n;
    p->list_size = list_size;
    p->f_mode = f_mode;
    p->llr_max = llr_max;
    p->flags = flags;
    if (list_size > 1 && !pl::scl_supported(p)) {  // reject at construction, not at the first decode
        delete p;
        return PL_ENOTSUP;
    }
    if (int r = pl::check_hip(hipGetDevice(&p->device), "pl_plan_create: hipGetDevice")) {
        delete p;
        return r;
    }

    const int nwords = (n + 31) / 32;
    std::vector<uint32_t> fw(nwords, 0u);
    std::vector<int32_t> info, rank(n, -1);
    for (int i = 0; i < n; ++i) {
        if (frozen_mask[i]) {
            fw[i >> 5] |= 1u << (i & 31);
        } else {
            rank[i] = (int32_t)info.size();
            info.push_back(i);
        }
    }
    p->k = (int32_t)info.size();
    // Node classification (exact SC shortcuts, see sc_kernel.hip): stage s in 1..log_n, node q
    // (positions [q*2^s, (q+1)*2^s)) -> bit OFF(s) + q with OFF(s) = n - (n >> (s-1)).
    //   rate-0: all frozen   rate-1: none frozen   repetition: all frozen but the last
    //   SPC: only the first frozen
    const int nflag = n - 1;
    const int fwords = (nflag + 31) / 32;
    p->type_stride = fwords > 64 ? fwords : 64;
    std::vector<uint32_t> r0(fwords + 1, 0u), types(4 * (size_t)p->type_stride, 0u);
    for (int s = 1; s <= log_n; ++s) {
        const int off = n - (n >> (s - 1));
        for (int q = 0; q < (n >> s); ++q) {
            const int a = q << s, m = 1 << s;
            int nfz = 0;
            for (int i = a; i < a + m; ++i) nfz += frozen_mask[i] != 0;
            const bool is_r0 = nfz == m, is_r1 = nfz == 0;
            const bool is_rep = nfz == m - 1 && !frozen_mask[a + m - 1];
            const bool is_spc = nfz == 1 && frozen_mask[a];
            const int bit = off + q;
            const uint32_t mbit = 1u << (bit & 31);
            if (is_r0) r0[bit >> 5] |= mbit;
            if (is_r0) types[0 * p->type_stride + (bit >> 5)] |= mbit;
            if (is_r1) types[1 * p->type_stride + (bit >> 5)] |= mbit;
            if (is_rep) types[2 * p->type_stride + (bit >> 5)] |= mbit;
            if (is_spc) types[3 * p->type_stride + (bit >> 5)] |= mbit;
        }
    }
    int r = upload(&p->d_frozen_words, fw);
    if (!r) r = upload(&p->d_rate0_words, r0);
    if (!r) r = upload(&p->d_type_words, types);
    if (!r) r = upload(&p->d_info_rank, rank);
    if (!r && !info.empty()) r = upload(&p->d_info_pos, info);
    if (r) {
        free_plan(p);
        return r;
    }
    // SC plans get a kernel specialised to this frozen set (jit.cpp) when its code object is in a
    // kernel cache, unless the caller or PL_SC_SPECIALIZE=0 asks for the generic one.  Compiling a
    // missing one in this process (hiprtc) is opt-in (PL_PLAN_JIT): in a process that has loaded
    // another ROCm's amd_comgr (torch's bundled runtime) hiprtc is not reliable (DESIGN.md
    // section 1), so by default a cache miss leaves the plan on the generic kernel.  Failure to
    // specialise is not an error: the generic kernel is exact too; pl_plan_kernel() reports which
    // one the plan uses.
    const char* env = getenv("PL_SC_SPECIALIZE");
    const bool want = list_size == 1 && !(flags & PL_PLAN_GENERIC) && !(env && env[0] == '0');
    if (want) {
        const std::string saved = g_last_error;
        const bool jit = (flags & PL_PLAN_JIT) && !(flags & PL_PLAN_CACHE_ONLY);
        const int rs = pl::attach_static(p, frozen_mask, jit);
        if (rs != PL_OK) {
            if (getenv("PL_VERBOSE")) fprintf(stderr, "polar_mi355x: generic SC kernel (%s)\n", g_last_error.c_str());
            pl::detach_static(p);
            (void)hipGetLastError();
        }
        g_last_error = saved;
    }
    *out = p;
    return PL_OK;
}

int pl_plan_destroy(pl_plan* plan) {
    free_plan(plan);
    return PL_OK;
}

int pl_plan_set_crc(pl_plan* p, int32_t degree, uint32_t poly_mask) {
    if (!p || degree < 0 || degree > 31 || (degree > 0 && p->k < degree) ||
        (degree > 0 && (poly_mask >> degree) != 0u)) {
        pl::set_error("pl_plan_set_crc: bad arguments (0 <= degree <= min(31, k), mask below x^degree)");
        return PL_EINVAL;
    }
    p->crc_deg = degree;
    p->crc_g = degree > 0 ? poly_mask : 0u;
    return PL_OK;
}

int pl_plan_device(const pl_plan* p, int32_t* device) {
    if (!p || !device) {
        pl::set_error("pl_plan_device: null argument");
        return PL_EINVAL;
    }
    *device = p->device;
    return PL_OK;
}

int pl_plan_info(const pl_plan* p, int32_t* n, int32_t* k, int32_t* list_size) {
    if (!p) {
        pl::set_error("pl_plan_info: null plan");
        return PL_EINVAL;
    }
    if (n) *n = p->n;
    if (k) *k = p->k;
    if (list_size) *list_size = p->list_size;
    return PL_OK;
}

int pl_sc_decode(const pl_plan* p, const float* llr, int64_t bs, void* out, int32_t out_kind, void* stream) {
    if (!p || bs < 0 || (bs > 0 && (!llr || (!out && p->k > 0)))) {
        pl::set_error("pl_sc_decode: bad arguments");
        return PL_EINVAL;
    }
    if (out_kind != PL_OUT_F32 && out_kind != PL_OUT_U8) {
        pl::set_error("pl_sc_decode: unknown out_kind");
        return PL_EINVAL;
    }
    if (int r = pl::check_device(p, static_cast<hipStream_t>(stream), "pl_sc_decode")) return r;
    if (p->sc_module) return pl::launch_sc_static(p, llr, bs, out, out_kind, static_cast<hipStream_t>(stream));
    return pl::launch_sc(p, llr, bs, out, out_kind, static_cast<hipStream_t>(stream));
}

size_t pl_sc_count_workspace_size(const pl_plan* p, int64_t bs) {
    if (!p || bs <= 0 || !p->sc_module) return 0;
    return (size_t)pl::sc_count_waves(p, bs) * 2 * sizeof(int32_t);
}

int pl_sc_decode_count(const pl_plan* p, const float* llr, int64_t bs, const uint32_t* ref_bits, int64_t* counts,
                       void* ws, size_t ws_bytes, void* stream) {
    if (!p || bs < 0 || !counts || (bs > 0 && p->k > 0 && (!llr || !ref_bits))) {
        pl::set_error("pl_sc_decode_count: bad arguments");
        return PL_EINVAL;
    }
    if (p->list_size != 1) {
        pl::set_error("pl_sc_decode_count: needs an SC plan (list_size 1)");
        return PL_EINVAL;
    }
    if (!p->sc_module || !p->sc_fn_cnt) {
        pl::set_error("pl_sc_decode_count: the plan runs the generic SC kernel (no fused count); "
                      "decode with pl_sc_decode and count with pl_count_errors");
        return PL_ENOTSUP;
    }
    if (int r = pl::check_device(p, static_cast<hipStream_t>(stream), "pl_sc_decode_count")) return r;
    if (bs == 0 || p->k == 0) return PL_OK;
    if (ws_bytes < pl_sc_count_workspace_size(p, bs) || !ws) {
        pl::set_error("pl_sc_decode_count: workspace too small (pl_sc_count_workspace_size)");
        return PL_EINVAL;
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    int32_t* part = static_cast<int32_t*>(ws);
    if (int r = pl::launch_sc_static_count(p, llr, bs, ref_bits, part, st)) return r;
    return pl::launch_sum_pairs(part, pl::sc_count_waves(p, bs), counts, st);
}

int pl_sc_sim_count(const pl_plan* p, uint64_t seed, uint64_t iteration, int64_t row0, int64_t bs, float no,
                    int64_t* counts, void* ws, size_t ws_bytes, float* llr_dump, float* u_dump, void* stream) {
    if (!p || bs < 0 || row0 < 0 || !counts || !(no > 0.0f) || (iteration >> 32) != 0) {
        pl::set_error("pl_sc_sim_count: bad arguments (no must be > 0, iteration < 2^32)");
        return PL_EINVAL;
    }
    if (p->list_size != 1) {
        pl::set_error("pl_sc_sim_count: needs an SC plan (list_size 1)");
        return PL_EINVAL;
    }
    if (!p->sc_module || !p->sc_fn_sim) {
        pl::set_error("pl_sc_sim_count: the plan's kernel has no fused Monte-Carlo entry (generic kernel, or not "
                      "64 channel slots per lane); use pl_awgn_qpsk_llr_bits + pl_sc_decode_count");
        return PL_ENOTSUP;
    }
    if (int r = pl::check_device(p, static_cast<hipStream_t>(stream), "pl_sc_sim_count")) return r;
    if (bs == 0) return PL_OK;
    if (ws_bytes < pl_sc_count_workspace_size(p, bs) || !ws) {
        pl::set_error("pl_sc_sim_count: workspace too small (pl_sc_count_workspace_size)");
        return PL_EINVAL;
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    int32_t* part = static_cast<int32_t*>(ws);
    if (int r = pl::launch_sc_static_sim(p, seed, iteration, row0, bs, no, part, llr_dump, u_dump, st)) return r;
    return pl::launch_sum_pairs(part, pl::sc_count_waves(p, bs), counts, st);
}

size_t pl_scl_workspace_size(const pl_plan* p, int64_t bs) { return p ? pl::scl_workspace_size(p, bs) : 0; }

int pl_scl_decode(const pl_plan* p, const float* llr, int64_t bs, void* out, int32_t out_kind, double* out_pm,
                  void* ws, size_t ws_bytes, void* stream) {
    if (!p || bs < 0 || (bs > 0 && (!llr || (!out && p->k > 0)))) {
        pl::set_error("pl_scl_decode: bad arguments");
        return PL_EINVAL;
    }
    if (out_kind != PL_OUT_F32 && out_kind != PL_OUT_U8) {
        pl::set_error("pl_scl_decode: unknown out_kind");
        return PL_EINVAL;
    }
    if ((ws != nullptr || ws_bytes != 0) && ws_bytes < pl::scl_workspace_size(p, bs)) {
        pl::set_error("pl_scl_decode: workspace too small");
        return PL_EINVAL;
    }
    if (int r = pl::check_device(p, static_cast<hipStream_t>(stream), "pl_scl_decode")) return r;
    return pl::launch_scl(p, llr, bs, out, out_kind, out_pm, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

int pl_polar_encode(const pl_plan* p, const float* u, int64_t bs, float* cw, void* stream) {
    if (!p || bs < 0 || (bs > 0 && (!cw || (!u && p->k > 0)))) {
        pl::set_error("pl_polar_encode: bad arguments");
        return PL_EINVAL;
    }
    if (int r = pl::check_device(p, static_cast<hipStream_t>(stream), "pl_polar_encode")) return r;
    return pl::launch_encode(p, u, bs, cw, static_cast<hipStream_t>(stream));
}

}  // extern "C"
