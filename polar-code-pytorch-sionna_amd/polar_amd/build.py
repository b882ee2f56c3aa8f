"""Build libpolar_mi355x.so (the HIP kernels + C ABI) in-tree for gfx950, and pre-build the
code-specialised SC kernels of the reference's codes into polar_amd/kcache/.

    python -m polar_amd.build            # from polar-code-pytorch-sionna_amd/

hipcc (and hiprtc) cross-compile for gfx950 without a GPU, so this runs in the build container;
the library and the kernel cache travel to the GPU box with the repository snapshot.
"""
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_obj")
LIB = os.path.join(HERE, "libpolar_mi355x.so")
KCACHE = os.path.join(HERE, "kcache")
SOURCES = ["sc_kernel.hip", "scl_kernel.hip", "encode_kernel.hip", "ratematch_kernel.hip", "channel_kernel.hip",
           "clock_kernel.hip", "capi.cpp", "jit.cpp"]
# scl_tree_kernel.hip is compiled once per list size (its instantiations, in parallel) and once
# for the launcher: (object name, source, defines)
UNITS = [(s + ".o", s, []) for s in SOURCES] + \
    [(f"scl_tree_L{L}.o", "scl_tree_kernel.hip", [f"-DPL_SCL_TREE_L={L}"]) for L in (2, 4, 8, 16, 32)] + \
    [("scl_tree_dispatch.o", "scl_tree_kernel.hip", ["-DPL_SCL_TREE_DISPATCH"])]
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _hipcc():
    for cand in (os.environ.get("HIPCC"), os.path.join(ROCM, "bin", "hipcc"), shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found; the MI355X decoder library cannot be built")


def _needs(obj, src, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in [src] + deps)


def _fnv_files(paths, extra=b""):
    h = 0xcbf29ce484222325
    for path in paths:
        for b in os.path.basename(path).encode() + b"\0" + open(path, "rb").read():
            h = ((h ^ b) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    for b in extra:
        h = ((h ^ b) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


HEADER = os.path.join(HERE, "..", "..", "include", "polar_mi355x.h")


def source_hash():
    """FNV-1a 64 over the library's sources (csrc/*, the C header) in name order: pl_version()
    reports it, so a prebuilt library that travels without its sources can be matched to them."""
    files = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp", ".h")))
    return _fnv_files([os.path.join(CSRC, f) for f in files] + [HEADER])


# the sources the subtree SCL kernel is compiled from (profiles/valu.json records of its SQ passes
# stay valid while these are unchanged, whatever else in csrc/ changes)
SCL_TREE_SOURCES = ("scl_tree_kernel.hip", "softplus.h", "plan.h")


# the compile flags of the object files (build() below): part of what a kernel record describes
COMPILE_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-ffp-contract=off"]


def kernel_source_hash(files):
    """FNV-1a 64 over the named csrc/ files and the C header, in the given order, and the compile
    flags and -D defines the library's units of those sources are built with (a
    flags-only change must make the records of the kernel stale too)."""
    defs = sorted(" ".join(d) for _, src, d in UNITS if src in files)
    extra = (" ".join([ARCH] + COMPILE_FLAGS) + "|" + "|".join(defs)).encode()
    return _fnv_files([os.path.join(CSRC, f) for f in files] + [HEADER], extra)


def _write_src_hash(obj_dir):
    """obj_dir/src_hash.h: the source hash as PL_SRC_HASH (rewritten only when it changes, so
    capi.cpp rebuilds exactly when a source does)."""
    path = os.path.join(obj_dir, "src_hash.h")
    text = f'#define PL_SRC_HASH "{source_hash()}"\n'
    if not os.path.exists(path) or open(path).read() != text:
        with open(path, "w") as f:
            f.write(text)
    return path


def _embed_static_source():
    """sc_static.h as a C++ raw string literal (the hiprtc source of the specialised kernels)."""
    src = open(os.path.join(CSRC, "sc_static.h")).read()
    inc_line = '#include "exactf.h"  // build.py inlines it into the embedded source\n'
    assert inc_line in src
    src = src.replace(inc_line, open(os.path.join(CSRC, "exactf.h")).read().replace("#pragma once\n", ""))
    assert ")PLSRC\"" not in src
    inc = os.path.join(OBJ, "sc_static_src.inc")
    text = 'R"PLSRC(' + src + ')PLSRC"\n'
    if not os.path.exists(inc) or open(inc).read() != text:
        with open(inc, "w") as f:
            f.write(text)
    return inc


# Development library (tools/ only): -DPL_DEV=1 compiles in the A/B hooks -- environment variables
# that replace kernel sources or switch on diagnostic (wrong-result) macros -- which the release
# library above does not contain (tests/test_abi.py checks).  polar_amd._lib.use_dev_library()
# makes a process load it instead of the release library.
OBJ_DEV = os.path.join(HERE, "_obj_dev")
LIB_DEV = os.path.join(HERE, "libpolar_mi355x_dev.so")


def build(force=False, verbose=False, dev=False):
    hipcc = _hipcc()
    obj_dir, lib_path = (OBJ_DEV, LIB_DEV) if dev else (OBJ, LIB)
    dev_flags = ["-DPL_DEV=1"] if dev else []
    os.makedirs(obj_dir, exist_ok=True)
    inc = _embed_static_source()
    hash_h = _write_src_hash(obj_dir)
    deps = [os.path.join(CSRC, "plan.h"), os.path.join(CSRC, "softplus.h"), os.path.join(CSRC, "exactf.h"),
            os.path.join(HERE, "..", "..", "include", "polar_mi355x.h")]
    jobs = []
    for oname, s, defs in UNITS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(obj_dir, oname)
        extra = [inc] if s == "jit.cpp" else [hash_h] if s == "capi.cpp" else []
        if force or _needs(obj, src, deps + extra):
            lang = ["-x", "hip"] if s.endswith(".cpp") else []
            cmd = [hipcc, f"--offload-arch={ARCH}", *COMPILE_FLAGS, f"-I{obj_dir}", f"-I{OBJ}", *dev_flags, *defs, *lang,
                   "-c", src, "-o", obj]
            jobs.append(cmd)

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
        if verbose and (r.stdout or r.stderr):
            print(r.stdout + r.stderr)
    with ThreadPoolExecutor(max_workers=min(8, len(jobs) or 1)) as ex:
        list(ex.map(run, jobs))
    objs = [os.path.join(obj_dir, u[0]) for u in UNITS]
    if force or jobs or not os.path.exists(lib_path) or \
            any(os.path.getmtime(o) > os.path.getmtime(lib_path) for o in objs):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, f"-L{ROCM}/lib",
               f"-Wl,-rpath,{ROCM}/lib", "-lhiprtc", "-o", lib_path]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
    return lib_path


def prebuild_codes(codes, workers=None, prune=True):
    """Compile the specialised SC kernels of `codes` = [(frozen_mask uint8[n], f_mode)] into
    KCACHE with hipcc --genco, one child process per code (content-addressed names from
    pl_sc_source: unchanged codes are found and skipped).  Not hiprtc: in a process that has
    imported torch, hiprtc runs against torch's bundled amd_comgr (see _lib.py)."""
    from . import _lib
    os.makedirs(KCACHE, exist_ok=True)
    jobs, keep = [], set()
    for m, fm in codes:
        src, name = _lib.sc_source(len(m), m, int(fm))
        keep.add(name)
        if not os.path.exists(os.path.join(KCACHE, name)):
            jobs.append((len(m), src, name))
    jobs.sort(key=lambda j: -j[0])  # longest compiles first
    workers = workers or min(8, os.cpu_count() or 1)

    def one(job):
        n, src, name = job
        return _lib.compile_code_object(src, KCACHE, name), f"n={n} {name}"
    with ThreadPoolExecutor(max_workers=workers) as ex:
        res = list(ex.map(one, jobs))
    errs = [what for ok, what in res if not ok]
    if errs:
        raise RuntimeError("specialised SC kernel pre-build (hipcc --genco) failed:\n" + "\n".join(errs))
    if prune:  # drop code objects of older kernel versions (they would only travel as dead weight)
        for f in os.listdir(KCACHE):
            if f.endswith(".co") and f not in keep:
                os.remove(os.path.join(KCACHE, f))


def test_random_codes():
    """The arbitrary frozen sets tests/test_sc_gpu.py::test_sc_random_vs_oracle decodes with the
    specialised kernel (every n = 2 ... 2048, same seeds), so the GPU tests never compile."""
    import numpy as np
    out = []
    for log_n in range(1, 12):
        for rate in (0.25, 0.5, 0.75):
            n = 1 << log_n
            rng = np.random.default_rng(log_n * 10 + int(rate * 4))
            k = max(1, int(n * rate))
            fp = np.sort(rng.permutation(n)[: n - k])
            m = np.zeros(n, dtype=np.uint8)
            m[fp] = 1
            out.append((m, 0))
    return out


ROOT_HALF_PAIRS = [("R0", "GEN"), ("GEN", "R0"), ("R0", "R1"), ("R1", "R0"), ("REP", "SPC"), ("SPC", "REP"),
                   ("GEN", "R1"), ("R1", "GEN"), ("REP", "GEN"), ("GEN", "SPC")]


def root_half_codes():
    """n = 1024 frozen masks whose two root halves are each rate-0, rate-1, repetition, SPC or the
    reference (512,1024) code's half (tests/test_sc_gpu.py::test_sc_root_half_types): every branch
    of the specialised kernel's virtual root, including the LDS channel half (sc_static.h Ch)."""
    import numpy as np
    data = os.path.join(HERE, "data", "frozen_sets.npz")
    with np.load(data) as d:
        ref = np.zeros(1024, dtype=np.uint8)
        ref[d["k512_n1024"].astype(np.int64)] = 1
    h = 512
    kinds = {"R0": np.ones(h, np.uint8), "R1": np.zeros(h, np.uint8),
             "REP": np.r_[np.ones(h - 1, np.uint8), 0], "SPC": np.r_[1, np.zeros(h - 1, np.uint8)]}
    out = []
    for a, b in ROOT_HALF_PAIRS:
        left = ref[:h] if a == "GEN" else kinds[a]
        right = ref[h:] if b == "GEN" else kinds[b]
        out.append((a + "_" + b, np.concatenate([left, right]).astype(np.uint8)))
    return out


# 5G NR (k, E) configurations the package's tests decode (tests/test_polar5g_gpu.py); their
# mother codes are decoded by the exact-f SC kernel (Polar5GDecoder dec_type="SC")
POLAR5G_TEST_CODES = [(12, 20), (12, 160), (16, 64), (19, 100), (20, 40), (24, 300), (32, 64), (40, 100), (48, 64),
                      (64, 128), (64, 200), (100, 180), (120, 1000), (140, 576), (200, 400), (250, 300),
                      (300, 1088), (500, 1024), (512, 700), (1013, 1088), (30, 1088), (64, 1024)]


def polar5g_codes():
    """Exact-f SC codes of the 5G mother codes in POLAR5G_TEST_CODES (uplink)."""
    import numpy as np
    from .polar5g import _rate_match_tables
    out = []
    for k, e in POLAR5G_TEST_CODES:
        _, n_polar, frozen, _, _ = _rate_match_tables(k, e, "uplink")
        m = np.zeros(n_polar, dtype=np.uint8)
        m[np.asarray(frozen, dtype=np.int64)] = 1
        out.append((m, 1))
    return out


def reference_codes():
    """The codes the reference harness and this package's tests/bench use: every pinned
    reference frozen set with n <= 2048 (min-sum), the golden shapes in exact-f mode, and the
    5G mother codes the tests decode (exact f)."""
    import numpy as np
    data = os.path.join(HERE, "data", "frozen_sets.npz")
    out = []
    with np.load(data) as d:
        for key in d.files:
            k, n = (int(v[1:]) for v in key.split("_"))
            if n > 2048:
                continue
            m = np.zeros(n, dtype=np.uint8)
            m[d[key].astype(np.int64)] = 1
            out.append((m, 0))
            if (k, n) in ((2, 4), (4, 8), (8, 16), (16, 32), (16, 64), (32, 64), (48, 64), (128, 256),
                          (256, 512), (512, 1024), (1024, 2048)):
                out.append((m, 1))
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):  # the CRC6 warning of 12 <= k <= 19
        out += polar5g_codes()
    out += test_random_codes()
    out += [(m, 0) for _, m in root_half_codes()]
    # tests/test_sc_gpu.py::test_sc_edge_cases: n = 64 with every position frozen (k = 0) and none (k = n)
    out += [(np.ones(64, dtype=np.uint8), 0), (np.zeros(64, dtype=np.uint8), 0)]
    # tests/test_sc_gpu.py::test_sc_exact_large_llr_max_*: every n = 2, 4 code with k >= 1, exact f,
    # llr_max 60 and 80 (the full-range code object, PL_F_WIDE_RANGE) and the default 30
    for n in (2, 4):
        for code in range(1, 1 << n):
            m = np.array([((code >> i) & 1) ^ 1 for i in range(n)], dtype=np.uint8)
            out += [(m, 1), (m, 1 | 0x100)]
    uniq = {}
    for m, fm in out:
        uniq[(bytes(bytearray(m)), fm)] = (m, fm)
    return list(uniq.values())


if __name__ == "__main__":
    if "--dev" in sys.argv:  # the development library only (tools/)
        print(build(force="--force" in sys.argv, verbose=True, dev=True))
        sys.exit(0)
    print(build(force="--force" in sys.argv, verbose=True))
    if "--no-kernels" not in sys.argv:
        prebuild_codes(reference_codes())
        print("kcache:", len(os.listdir(KCACHE)), "code objects")
