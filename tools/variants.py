"""Development aid: build SC-kernel variants (-D flags) and time them in ONE process on the GPU.

  python tools/variants.py build NAME:"-DFOO=1" ...     (build container; hipcc)
  python tools/variants.py time [--k 512 --n 1024 --bs 65536]   (GPU box)
Variant libraries go to polar-code-pytorch-sionna_amd/polar_amd/_variants/ (git-ignored).
"""
import ctypes, json, os, subprocess, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "polar-code-pytorch-sionna_amd")
VAR = os.path.join(PKG, "polar_amd", "_variants")
sys.path.insert(0, PKG)


def build(specs):
    from polar_amd import build as b
    os.makedirs(VAR, exist_ok=True)
    hipcc = b._hipcc()
    objs = [os.path.join(b.OBJ, s + ".o") for s in b.SOURCES if s != "sc_kernel.hip"]
    b.build()
    def one(spec):
        name, flags = spec.split(":", 1)
        o = os.path.join(VAR, f"sc_{name}.o")
        cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", *flags.split(),
               "-c", os.path.join(b.CSRC, "sc_kernel.hip"), "-o", o]
        subprocess.check_call(cmd)
        subprocess.check_call([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", o, *objs, "-o",
                               os.path.join(VAR, f"lib_{name}.so")])
        return name
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(8) as ex:
        print(list(ex.map(one, specs)))


def time_all(k=512, n=1024, bs=65536, reps=20, rounds=3, only=None):
    import torch
    import polar_amd
    from polar_amd import _lib, channel
    libs = sorted(f for f in os.listdir(VAR) if f.startswith("lib_") and f.endswith(".so"))
    if only:
        libs = [f for f in libs if f == f"lib_{only}.so"]
    fp = polar_amd.reference_frozen_pos(k, n)
    mask = polar_amd.frozen_mask(fp, n)
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(42)
    model = channel.System_AWGN_model(n, k, channel.GpuEncoder(fp, n), None, device=dev, generator=gen)
    inputs = {}
    for db in (2.0, 4.0):
        bits, _, llr = model.llrs(bs, torch.tensor(db))
        inputs[f"awgn{db}"] = (bits, llr.contiguous())
    inputs["randn"] = (None, (torch.randn(bs, n, device=dev, generator=gen) * 2 + 1).contiguous())
    handles = {}
    for f in libs:
        L = _lib._declare(ctypes.CDLL(os.path.join(VAR, f)))
        h = ctypes.c_void_p()
        assert L.pl_plan_create(ctypes.byref(h), n, mask.ctypes.data_as(ctypes.c_void_p), 1, 0, 30.0, 0) == 0
        handles[f] = (L, h)
    out = torch.empty((bs, k), device=dev)
    ref = {}
    res = {f: {nm: [] for nm in inputs} for f in libs}
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for r in range(rounds):
        for f, (L, h) in handles.items():
            for nm, (bits, x) in inputs.items():
                call = lambda: L.pl_sc_decode(h, ctypes.c_void_p(x.data_ptr()), bs, ctypes.c_void_p(out.data_ptr()), 0, st)
                call(); call()
                torch.cuda.synchronize()
                if r == 0:
                    key = nm
                    if key not in ref:
                        ref[key] = out.clone()
                    elif not torch.equal(ref[key], out):
                        print(f"MISMATCH {f} {nm}")
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    call()
                e1.record()
                torch.cuda.synchronize()
                res[f][nm].append(e0.elapsed_time(e1) / reps)
    for f in libs:
        print(f, {nm: f"{min(v):.4f}ms {bs / min(v) / 1e3:.1f}Mcw/s" for nm, v in res[f].items()}, flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        import argparse
        ap = argparse.ArgumentParser()
        ap.add_argument("--k", type=int, default=512)
        ap.add_argument("--n", type=int, default=1024)
        ap.add_argument("--bs", type=int, default=65536)
        ap.add_argument("--only", default=None)
        ap.add_argument("--reps", type=int, default=20)
        ap.add_argument("--rounds", type=int, default=3)
        a = ap.parse_args(sys.argv[2:])
        time_all(a.k, a.n, a.bs, a.reps, a.rounds, a.only)
