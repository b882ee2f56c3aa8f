"""Build libpolar_mi355x.so (the HIP kernels + C ABI) in-tree for gfx950.

    python -m polar_amd.build            # from polar-code-pytorch-sionna_amd/

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build container; the
resulting .so travels to the GPU box with the repository snapshot.
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
SOURCES = ["sc_kernel.hip", "scl_kernel.hip", "encode_kernel.hip", "capi.cpp"]
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found; the MI355X decoder library cannot be built")


def _needs(obj, src, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in [src] + deps)


def build(force=False, verbose=False):
    hipcc = _hipcc()
    os.makedirs(OBJ, exist_ok=True)
    deps = [os.path.join(CSRC, "plan.h"),
            os.path.join(HERE, "..", "..", "include", "polar_mi355x.h")]
    jobs = []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OBJ, s + ".o")
        if force or _needs(obj, src, deps):
            lang = ["-x", "hip"] if s.endswith(".cpp") else []
            cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
                   "-ffp-contract=off", *lang, "-c", src, "-o", obj]
            jobs.append(cmd)
    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
        if verbose and (r.stdout or r.stderr):
            print(r.stdout + r.stderr)
    with ThreadPoolExecutor(max_workers=min(8, len(jobs) or 1)) as ex:
        list(ex.map(run, jobs))
    objs = [os.path.join(OBJ, s + ".o") for s in SOURCES]
    if force or jobs or not os.path.exists(LIB):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
