// jit.cpp -- code-specialised SC kernels: source generation, hiprtc compilation, a
// content-addressed code-object cache, module loading and launch.
//
// A plan for an SC code (list_size 1) gets its own kernel: sc_static.h instantiated with the
// code's node-type table (R0/R1/REP/SPC/GEN for every node of the decoding tree), so every
// node-type decision of the reference recursion (x_run_sn_polar/polar/polar_sc.py:54-98) is
// resolved at compile time.  Code objects are cached by a hash of the generated source and
// the compile options; build.py pre-compiles the codes the reference harness uses, so plans
// for them load without compiling.  If hiprtc is unavailable or fails, the plan keeps the
// generic kernel (sc_kernel.hip), which is equally exact.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <stdint.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "../../../include/polar_mi355x.h"
#include "plan.h"

namespace {

const char kStaticSrc[] =
#include "sc_static_src.inc"
    ;

const char* kOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off"};
constexpr int kNumOpts = sizeof(kOpts) / sizeof(kOpts[0]);

// Out-of-process build of a specialised kernel (polar_amd/_lib.py compile_code_object reads both
// lines from the head of the generated source): the hipcc flags, and the compiler this library
// was built with.  Both are part of the source, hence of the cache name, so a code object built
// with other flags or by another compiler release is never picked up under this name; the Python
// side refuses to compile when `hipcc --version` does not report the same compiler.
const char kGencoFlags[] = "--offload-arch=gfx950 --genco --no-gpu-bundle-output -O3 -std=c++17 -ffp-contract=off";

enum : int { R0 = 0, R1 = 1, REP = 2, SPC = 3, GEN = 4 };

uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
    for (unsigned char c : s) {
        h ^= c;
        h *= 1099511628211ull;
    }
    return h;
}

int log2_exact(int n) {
    int s = 0;
    while ((1 << s) < n) ++s;
    return (1 << s) == n ? s : -1;
}

std::string lib_dir() {
    Dl_info info;
    if (dladdr(reinterpret_cast<const void*>(&fnv1a), &info) && info.dli_fname) {
        std::string p(info.dli_fname);
        const size_t cut = p.find_last_of('/');
        if (cut != std::string::npos) return p.substr(0, cut);
    }
    return ".";
}

bool mkdirs(const std::string& d) {
    if (d.empty()) return false;
    struct stat st;
    if (stat(d.c_str(), &st) == 0) return S_ISDIR(st.st_mode);
    const size_t cut = d.find_last_of('/');
    if (cut != std::string::npos && cut > 0) mkdirs(d.substr(0, cut));
    return mkdir(d.c_str(), 0755) == 0 || errno == EEXIST;
}

// Cache directories, in lookup order: $PL_KERNEL_CACHE, <dir of this library>/kcache (pre-built
// by build.py, travels with the package), $HOME/.cache/polar_mi355x.
std::vector<std::string> cache_dirs() {
    std::vector<std::string> d;
    if (const char* e = getenv("PL_KERNEL_CACHE")) {
        if (*e) d.push_back(e);
    }
    d.push_back(lib_dir() + "/kcache");
    if (const char* h = getenv("HOME")) d.push_back(std::string(h) + "/.cache/polar_mi355x");
    return d;
}

bool read_file(const std::string& path, std::vector<char>& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return !out.empty();
}

bool write_file_atomic(const std::string& dir, const std::string& name, const std::vector<char>& data) {
    if (!mkdirs(dir) || access(dir.c_str(), W_OK) != 0) return false;
    const std::string tmp = dir + "/." + name + "." + std::to_string(getpid()) + ".tmp";
    {
        std::ofstream f(tmp, std::ios::binary);
        if (!f) return false;
        f.write(data.data(), (std::streamsize)data.size());
        if (!f) return false;
    }
    return rename(tmp.c_str(), (dir + "/" + name).c_str()) == 0;
}

}  // namespace

namespace pl {

// Node types in heap order: node of size 2^s at position p -> index (n >> s) + (p >> s).
std::vector<uint8_t> node_types(int n, const uint8_t* frozen) {
    const int log_n = log2_exact(n);
    std::vector<uint8_t> nt(2 * (size_t)n, R0);
    for (int s = 0; s <= log_n; ++s) {
        const int S = 1 << s;
        for (int p = 0; p < n; p += S) {
            int nfz = 0;
            for (int i = p; i < p + S; ++i) nfz += frozen[i] != 0;
            int t;
            if (nfz == S) t = R0;
            else if (nfz == 0) t = R1;
            else if (S >= 2 && nfz == S - 1 && !frozen[p + S - 1]) t = REP;
            else if (S >= 2 && nfz == 1 && frozen[p]) t = SPC;
            else t = GEN;
            nt[(size_t)(n >> s) + (size_t)(p >> s)] = (uint8_t)t;
        }
    }
    return nt;
}

// Min-sum codes of n = 256, 512, 1024 run n/64 lanes per codeword (instead of n/128) at 3
// waves/SIMD, with the v_bitop3 sign merge in f, and decode their lane-level SPC nodes (size <= G)
// by the plain recursion rather than the DPP parity/minimum shortcut.  Same-process A/B on MI355X
// (tools/static_probe.py, bs = 65536): (512,1024) 0.1009 vs 0.1177 ms, (256,512) 0.0419 vs
// 0.0489 ms, (128,256) 0.0230 vs 0.0411 ms; n = 128 is faster at one lane per codeword, and
// n = 2048 already uses the widest group (16 lanes).
bool tuned_wide(int log_n, int f_mode) { return f_mode == PL_F_MINSUM && log_n >= 8 && log_n <= 10; }

// log2(lanes per codeword).  Development builds only (PL_DEV, tools/): PL_SC_LOG_G overrides it
// (A/B of layouts; part of the source, hence of the cache key).
int static_log_g(int log_n, int f_mode) {
#if PL_DEV
    if (const char* e = getenv("PL_SC_LOG_G")) {
        const int v = atoi(e);
        if (v >= 0 && v <= 4 && v <= log_n) return v;
    }
#endif
    if (tuned_wide(log_n, f_mode)) return log_n - 6;
    return log_n > 7 ? log_n - 7 : 0;
}

// Lane of the codeword group holding residue r (mirror-butterfly layout of sc_static.h).
int mirror_lane(int G, int r) {
    if (G == 1) return 0;
    return r < G / 2 ? mirror_lane(G / 2, r) : G - 1 - mirror_lane(G / 2, r - G / 2);
}

std::string static_source(int n, const uint8_t* frozen, int f_mode_in) {
    // PL_F_WIDE_RANGE (exact f only): the code object of plans with llr_max > 43
    const bool wide = (f_mode_in & PL_F_WIDE_RANGE) != 0;
    const int f_mode = f_mode_in & ~PL_F_WIDE_RANGE;
    const int log_n = log2_exact(n), lg = static_log_g(log_n, f_mode);
    std::vector<uint8_t> nt = node_types(n, frozen);
    if (tuned_wide(log_n, f_mode)) {
        // lane-level SPC nodes (size <= G) by the plain recursion (A/B at n = 1024: 0.1009 vs
        // 0.1088 ms; the in-lane SPC nodes keep the shortcut)
        for (int s = 1; s <= lg; ++s)
            for (int p = 0; p < n; p += 1 << s) {
                uint8_t& t = nt[(size_t)(n >> s) + (size_t)(p >> s)];
                if (t == SPC) t = GEN;
            }
    }
    std::ostringstream o;
    o << "// pl-genco-flags: " << kGencoFlags << "\n// pl-compiler: " << __clang_version__ << "\n";
    if (tuned_wide(log_n, f_mode)) o << "#define PL_SC_MINW 3\n#define PL_SC_F_BITOP3 1\n";
    // Exact-f codes with 128 channel slots per lane (n >= 128) at 3 waves per SIMD (the f's fp64
    // chains wait on latency at 2 waves; same-process A/B at (512,1024), bs = 65536,
    // profiles/r04d_sc_exact_ab.txt: 1.153 ms at 3 waves, 1.148 at 4, 1.295 at 2).  The 128 channel
    // registers did not fit under that cap: 129 VGPRs were spilled to scratch (194 scratch
    // instructions per wave, ~0.5 GB of scratch traffic per launch).  Round 5: the stage-(n/2)
    // buffer in VGPRs and the channel read once per half (PL_SC_ROOT_MODE 1, whose second read the
    // caches serve -- a second load latency, cheap against this kernel's ~1 ms): 8 spills,
    // 13 scratch instructions per wave; same-process A/B (profiles/r05c_sc_exact_ab_*.txt)
    // 0.9155 vs 0.9469 ms at (512,1024), 0.1801 vs 0.1979 ms at (128,256).
    if (f_mode == PL_F_EXACT && log_n >= 7) o << "#define PL_SC_MINW 3\n#define PL_SC_ROOT_MODE 1\n";
    // Exact f: one code object per llr_max range (exactf.h PL_EXF_RANGE), so no f tests llr_max
    // and the lane-level f is inlined in the fast one (same-process A/B at (512,1024), bs = 65536,
    // profiles/r05f_sc_exact_ab_1024.txt: 0.9181 ms with the test in every f, 0.8618 without,
    // 0.8126 inlined; (128,256) 0.1802 / 0.1723 / 0.1705 ms).  Not inlined at n = 2048, whose
    // inlined kernel takes ~3 minutes to compile (the critical path of the code-object pre-build).
    if (f_mode == PL_F_EXACT)
        o << (wide ? "#define PL_EXF_RANGE 2\n"
                   : (log_n <= 10 ? "#define PL_EXF_RANGE 1\n#define PL_SC_FLANE_INLINE 1\n" : "#define PL_EXF_RANGE 1\n"));
    const int G = 1 << lg, NS = n >> lg;
    if (NS == 64) o << "#define PL_SC_SIM 1\n";  // the fused Monte-Carlo entry (sc_static.h OUT_SIM)
    std::string body = kStaticSrc;
#if PL_DEV
    // Development builds only (PL_DEV, tools/): PL_SC_DEFINES="NAME=VALUE ..." overrides the
    // kernel's tuning and diagnostic macros, PL_SC_SOURCE=<file> replaces the embedded sc_static.h
    // (A/B of kernel versions).  Both are part of the source, hence of the cache key; the source
    // is marked PL_DEV so that sc_static.h accepts its diagnostic (wrong-result) macros.  A
    // release library reads neither variable.
    o << "#define PL_DEV 1\n";
    if (const char* defs = getenv("PL_SC_DEFINES")) {
        std::istringstream in(defs);
        std::string tok;
        while (in >> tok) {
            const size_t eq = tok.find('=');
            o << "#define " << tok.substr(0, eq) << " " << (eq == std::string::npos ? "1" : tok.substr(eq + 1)) << "\n";
        }
    }
    if (const char* alt = getenv("PL_SC_SOURCE")) {
        std::vector<char> text;
        if (*alt && read_file(alt, text)) body.assign(text.begin(), text.end());
    }
#endif
    int k = 0;
    for (int i = 0; i < n; ++i) k += frozen[i] == 0;
    o << body << "\nstruct PlCode {\n  static constexpr int N = " << n << ", K = " << k << ", LOG_N = " << log_n
      << ", LOG_G = " << lg << ", G = " << (1 << lg) << ", NS = " << (n >> lg) << ", FM = " << f_mode
      << ";\n  static constexpr unsigned char NT[" << nt.size() << "] = {";
    for (size_t i = 0; i < nt.size(); ++i) o << (i ? "," : "") << (int)nt[i];
    o << "};\n";
    if (NS == 64) {
        // INFO_LANE[r]: bit j = position r + G j is an information position
        o << "  static constexpr unsigned long long INFO_LANE[" << G << "] = {";
        for (int r = 0; r < G; ++r) {
            unsigned long long m = 0;
            for (int j = 0; j < 64; ++j)
                if (!frozen[r + G * j]) m |= 1ull << j;
            o << (r ? "," : "") << m << "ull";
        }
        o << "};\n";
    }
    o << "};\nPL_SC_STATIC_KERNELS(PlCode)\n";
    return o.str();
}

// Cache file names.  hipcc --genco objects ("sc_"): the source names flags and compiler (above).
// In-process hiprtc objects ("scr_"): the source plus the hiprtc options and version -- a
// different compiler build, so never shared with the hipcc name.
std::string cache_name(const std::string& src) {
    char buf[32];
    snprintf(buf, sizeof buf, "sc_%016llx.co", (unsigned long long)fnv1a(src));
    return buf;
}

std::string cache_name_hiprtc(const std::string& src) {
    std::string key = src;
    for (int i = 0; i < kNumOpts; ++i) key += std::string("\n//opt ") + kOpts[i];
    int major = 0, minor = 0;
    if (hiprtcVersion(&major, &minor) == HIPRTC_SUCCESS) key += "\n//hiprtc " + std::to_string(major) + "." + std::to_string(minor);
    char buf[32];
    snprintf(buf, sizeof buf, "scr_%016llx.co", (unsigned long long)fnv1a(key));
    return buf;
}

// Compile (or find in a cache) the code object of one code.  No GPU needed.
int specialize(int n, const uint8_t* frozen, int f_mode, const char* forced_dir, bool allow_compile,
               std::vector<char>& image, std::string& path) {
    const std::string src = static_source(n, frozen, f_mode);
    const std::string name = cache_name_hiprtc(src);
    std::vector<std::string> dirs;
    if (forced_dir && *forced_dir) dirs.push_back(forced_dir);
    else dirs = cache_dirs();
    for (const std::string& nm : {cache_name(src), name}) {  // hipcc-built first
        for (const auto& d : dirs) {
            if (read_file(d + "/" + nm, image)) {
                path = d + "/" + nm;
                return PL_OK;
            }
        }
    }
    if (!allow_compile) {
        set_error("specialised SC kernel not in cache: " + name);
        return PL_ENOTSUP;
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "pl_sc_static.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        set_error("hiprtcCreateProgram failed");
        return PL_ENOTSUP;
    }
    const hiprtcResult rc = hiprtcCompileProgram(prog, kNumOpts, kOpts);
    if (rc != HIPRTC_SUCCESS) {
        size_t ls = 0;
        hiprtcGetProgramLogSize(prog, &ls);
        std::string log(ls, '\0');
        if (ls) hiprtcGetProgramLog(prog, &log[0]);
        hiprtcDestroyProgram(&prog);
        set_error("hiprtc compile of the specialised SC kernel failed: " + log.substr(0, 2000));
        return PL_ENOTSUP;
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    image.assign(cs, 0);
    hiprtcGetCode(prog, image.data());
    hiprtcDestroyProgram(&prog);
    path.clear();
    for (const auto& d : dirs) {
        if (write_file_atomic(d, name, image)) {
            path = d + "/" + name;
            break;
        }
    }
    return PL_OK;
}

// Per-plan setup: info_loc table + module (called from pl_plan_create for SC plans).
int attach_static(pl_plan* p, const uint8_t* frozen, bool allow_compile) {
    std::vector<char> image;
    std::string path;
    const int fm = p->f_mode == PL_F_EXACT && p->llr_max > 43.0f ? (PL_F_EXACT | PL_F_WIDE_RANGE) : p->f_mode;
    int r = specialize(p->n, frozen, fm, nullptr, allow_compile, image, path);
    if (r) return r;
    hipModule_t mod;
    r = check_hip(hipModuleLoadData(&mod, image.data()), "hipModuleLoadData(specialised SC kernel)");
    if (r) return r;
    hipFunction_t f32, u8;
    r = check_hip(hipModuleGetFunction(&f32, mod, "pl_sc_static_f32"), "hipModuleGetFunction");
    if (!r) r = check_hip(hipModuleGetFunction(&u8, mod, "pl_sc_static_u8"), "hipModuleGetFunction");
    hipFunction_t cnt = nullptr;  // optional (absent from diagnostic builds): decode + error count
    if (!r && hipModuleGetFunction(&cnt, mod, "pl_sc_static_cnt") != hipSuccess) {
        cnt = nullptr;
        (void)hipGetLastError();
    }
    hipFunction_t sim = nullptr;  // optional (codes with 64 slots per lane): producer + decode + count
    if (!r && hipModuleGetFunction(&sim, mod, "pl_sc_static_sim") != hipSuccess) {
        sim = nullptr;
        (void)hipGetLastError();
    }
    // info_loc[m]: where the u bit of information position m sits in a wave's LDS u words
    // (sc_static.h emit): (byte offset of its word in codeword 0's area) << 5 | bit in the word
    const int lg = static_log_g(p->log_n, p->f_mode);
    const int G = 1 << lg, WPL = (p->n / G + 31) / 32;
    std::vector<int32_t> loc;
    for (int i = 0; i < p->n; ++i)
        if (!frozen[i]) loc.push_back((((mirror_lane(G, i % G) * WPL + (i / G) / 32) * 4) << 5) | ((i / G) & 31));
    while (loc.size() % 4) loc.push_back(0);  // int4 reads of the table
    if (!r && !loc.empty()) {
        r = check_hip(hipMalloc(reinterpret_cast<void**>(&p->d_info_loc), loc.size() * sizeof(int32_t)),
                      "hipMalloc(info_loc)");
        if (!r)
            r = check_hip(hipMemcpy(p->d_info_loc, loc.data(), loc.size() * sizeof(int32_t), hipMemcpyHostToDevice),
                          "hipMemcpy(info_loc)");
    }
    if (r) {
        (void)hipModuleUnload(mod);
        return r;
    }
    // persistent kernels get a grid of the resident capacity (2 blocks of 4 waves per CU)
    hipDeviceptr_t gp = nullptr;
    size_t gsz = 0;
    int persistent = 0;
    if (hipModuleGetGlobal(&gp, &gsz, mod, "pl_sc_persistent") == hipSuccess && gsz == sizeof(int))
        (void)hipMemcpyDtoH(&persistent, gp, sizeof(int));
    (void)hipGetLastError();
    int bpc = 2;  // resident blocks per CU of a persistent kernel (pl_sc_blocks_per_cu, default 2)
    if (persistent && hipModuleGetGlobal(&gp, &gsz, mod, "pl_sc_blocks_per_cu") == hipSuccess && gsz == sizeof(int))
        (void)hipMemcpyDtoH(&bpc, gp, sizeof(int));
    (void)hipGetLastError();
    if (bpc < 1) bpc = 1;
    int waves = 4;  // waves per work-group (pl_sc_waves; objects built before it existed: 4)
    if (hipModuleGetGlobal(&gp, &gsz, mod, "pl_sc_waves") == hipSuccess && gsz == sizeof(int))
        (void)hipMemcpyDtoH(&waves, gp, sizeof(int));
    (void)hipGetLastError();
    if (waves != 1 && waves != 2 && waves != 4) {
        (void)hipModuleUnload(mod);
        set_error("specialised SC kernel: unsupported waves per work-group");
        return PL_EINVAL;
    }
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    p->sc_log_g = lg;
    p->sc_waves = waves;
    p->sc_persistent = persistent;
    p->resident_blocks = bpc * cus;
    p->sc_module = mod;
    p->sc_fn_f32 = f32;
    p->sc_fn_u8 = u8;
    p->sc_fn_cnt = cnt;
    p->sc_fn_sim = sim;
    p->kernel_path = path;
    return PL_OK;
}

void detach_static(pl_plan* p) {
    if (p->sc_module) (void)hipModuleUnload(p->sc_module);
    p->sc_module = nullptr;
    p->sc_fn_f32 = p->sc_fn_u8 = p->sc_fn_cnt = p->sc_fn_sim = nullptr;
}

int64_t sc_count_waves(const pl_plan* p, int64_t bs) {
    const int64_t per_block = p->sc_waves * (64 / (1 << p->sc_log_g));
    return ((bs + per_block - 1) / per_block) * p->sc_waves;
}

int launch_sc_static_count(const pl_plan* p, const float* llr, int64_t bs, const uint32_t* ref, int32_t* part,
                           hipStream_t st) {
    if (bs == 0 || p->k == 0) return PL_OK;
    if (p->sc_persistent) {
        set_error("SC decode+count: the plan's kernel is a persistent diagnostic build");
        return PL_ENOTSUP;
    }
    const int64_t blocks = sc_count_waves(p, bs) / p->sc_waves;
    if (blocks > 0x7fffffffLL) {
        set_error("SC decode+count: batch too large for one launch");
        return PL_EINVAL;
    }
    const float lmax = p->llr_max;
    int k = p->k;
    const int32_t* loc = p->d_info_loc;
    void* args[] = {(void*)&llr, (void*)&bs, (void*)&part, (void*)&loc, (void*)&k, (void*)&lmax, (void*)&ref};
    return check_hip(hipModuleLaunchKernel(p->sc_fn_cnt, (unsigned)blocks, 1, 1, 64 * p->sc_waves, 1, 1, 0, st, args, nullptr),
                     "SC decode+count launch (specialised)");
}

int launch_sc_static_sim(const pl_plan* p, uint64_t seed, uint64_t iteration, int64_t row0, int64_t bs, float no,
                         int32_t* part, float* llr_dump, float* u_dump, hipStream_t st) {
    if (bs == 0) return PL_OK;
    const int64_t blocks = sc_count_waves(p, bs) / p->sc_waves;
    if (blocks > 0x7fffffffLL) {
        set_error("SC Monte-Carlo iteration: batch too large for one launch");
        return PL_EINVAL;
    }
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32), it = (uint32_t)iteration;
    const float lmax = p->llr_max;
    int k = p->k;
    const int32_t* loc = p->d_info_loc;
    void* args[] = {(void*)&bs,  (void*)&row0, (void*)&k0, (void*)&k1,   (void*)&it,       (void*)&no,
                    (void*)&part, (void*)&loc, (void*)&k,  (void*)&lmax, (void*)&llr_dump, (void*)&u_dump};
    return check_hip(hipModuleLaunchKernel(p->sc_fn_sim, (unsigned)blocks, 1, 1, 64 * p->sc_waves, 1, 1, 0, st, args, nullptr),
                     "SC Monte-Carlo iteration launch (specialised)");
}

int launch_sc_static(const pl_plan* p, const float* llr, int64_t bs, void* out, int out_kind, hipStream_t st) {
    if (bs == 0 || p->k == 0) return PL_OK;
    const int G = 1 << p->sc_log_g;           // the layout the plan's kernel was built for
    const int64_t per_block = p->sc_waves * (64 / G);  // pls::kWaves codeword groups of 64/G
    int64_t blocks = (bs + per_block - 1) / per_block;
    if (p->sc_persistent && p->resident_blocks > 0 && blocks > p->resident_blocks) blocks = p->resident_blocks;
    if (blocks > 0x7fffffffLL) {
        set_error("SC decode: batch too large for one launch");
        return PL_EINVAL;
    }
    const float lmax = p->llr_max;
    int k = p->k;
    const int32_t* loc = p->d_info_loc;
    void* args[] = {(void*)&llr, (void*)&bs, (void*)&out, (void*)&loc, (void*)&k, (void*)&lmax};
    hipFunction_t fn = out_kind == PL_OUT_F32 ? p->sc_fn_f32 : p->sc_fn_u8;
    return check_hip(hipModuleLaunchKernel(fn, (unsigned)blocks, 1, 1, 64 * p->sc_waves, 1, 1, 0, st, args, nullptr),
                     "SC decode launch (specialised)");
}

}  // namespace pl

extern "C" {

int pl_sc_specialize(int32_t n, const uint8_t* frozen_mask, int32_t f_mode, const char* cache_dir, char* path_out,
                     size_t path_len) {
    if (!frozen_mask || log2_exact(n) < 1 || log2_exact(n) > 11 || (f_mode != PL_F_MINSUM && f_mode != PL_F_EXACT && f_mode != (PL_F_EXACT | PL_F_WIDE_RANGE))) {
        pl::set_error("pl_sc_specialize: bad arguments");
        return PL_EINVAL;
    }
    std::vector<char> image;
    std::string path;
    const int r = pl::specialize(n, frozen_mask, f_mode, cache_dir, true, image, path);
    if (r) return r;
    if (path_out && path_len) {
        strncpy(path_out, path.c_str(), path_len - 1);
        path_out[path_len - 1] = 0;
    }
    return PL_OK;
}

int pl_sc_source(int32_t n, const uint8_t* frozen_mask, int32_t f_mode, char* src_out, size_t src_len,
                 size_t* src_size, char* name_out, size_t name_len) {
    if (!frozen_mask || log2_exact(n) < 1 || log2_exact(n) > 11 || (f_mode != PL_F_MINSUM && f_mode != PL_F_EXACT && f_mode != (PL_F_EXACT | PL_F_WIDE_RANGE))) {
        pl::set_error("pl_sc_source: bad arguments");
        return PL_EINVAL;
    }
    const std::string src = pl::static_source(n, frozen_mask, f_mode);
    const std::string name = pl::cache_name(src);
    if (src_size) *src_size = src.size() + 1;
    if (src_out && src_len) {
        if (src_len < src.size() + 1) {
            pl::set_error("pl_sc_source: source buffer too small");
            return PL_EINVAL;
        }
        memcpy(src_out, src.c_str(), src.size() + 1);
    }
    if (name_out && name_len) {
        strncpy(name_out, name.c_str(), name_len - 1);
        name_out[name_len - 1] = 0;
    }
    return PL_OK;
}

int pl_plan_kernel(const pl_plan* p, int32_t* kind, char* path_out, size_t path_len) {
    if (!p) {
        pl::set_error("pl_plan_kernel: null plan");
        return PL_EINVAL;
    }
    if (kind) {
        if (p->list_size > 1) *kind = pl::scl_tree_eligible(p) ? PL_KERNEL_SCL_SUBTREE : PL_KERNEL_GENERIC;
        else *kind = p->sc_module ? PL_KERNEL_SPECIALIZED : PL_KERNEL_GENERIC;
    }
    if (path_out && path_len) {
        strncpy(path_out, p->kernel_path.c_str(), path_len - 1);
        path_out[path_len - 1] = 0;
    }
    return PL_OK;
}

}  // extern "C"
