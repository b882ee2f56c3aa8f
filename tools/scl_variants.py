"""Development aid: build SCL subtree-kernel variants (-D flags, L = 8 only) and time them in ONE
process on the GPU against the default library.

  python tools/scl_variants.py build NAME:"-DPL_SCL_R=4" ...     (build container; hipcc)
  python tools/scl_variants.py time [--n 1024 --k 512 --bs 8192]   (GPU box)
Variant libraries go to polar-code-pytorch-sionna_amd/polar_amd/_variants/ (git-ignored).
Environment knobs read at launch (PL_SCL_VIRTUAL=<max virtual stages>) apply to every library.
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "polar-code-pytorch-sionna_amd")
VAR = os.path.join(PKG, "polar_amd", "_variants")
sys.path.insert(0, PKG)


def build(specs):
    from polar_amd import build as b
    b.build(dev=True)  # variants and the baseline: development builds (PL_SCL_VIRTUAL, diagnostic macros)
    os.makedirs(VAR, exist_ok=True)
    hipcc = b._hipcc()
    objs = [os.path.join(b.OBJ_DEV, u[0]) for u in b.UNITS if u[1] != "scl_tree_kernel.hip"]

    def one(spec):
        name, flags = spec.split(":", 1)
        base = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-DPL_DEV=1", *flags.split()]
        # SCL_VARIANT_SRC: another copy of the kernel source (in csrc/, for its includes), e.g. the
        # committed version (git show HEAD:... > csrc/_head_scl_tree_kernel.hip) against the working tree
        src = os.path.join(b.CSRC, os.environ.get("SCL_VARIANT_SRC", "scl_tree_kernel.hip"))
        o1, o2 = os.path.join(VAR, f"sclt_{name}_L8.o"), os.path.join(VAR, f"sclt_{name}_disp.o")
        subprocess.check_call(base + ["-DPL_SCL_TREE_L=8", "-c", src, "-o", o1])
        subprocess.check_call(base + ["-DPL_SCL_TREE_DISPATCH", "-DPL_SCL_VARIANT_ONLY_L8", "-c", src, "-o", o2])
        subprocess.check_call([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", o1, o2, *objs,
                               f"-L{b.ROCM}/lib", f"-Wl,-rpath,{b.ROCM}/lib", "-lhiprtc",
                               "-o", os.path.join(VAR, f"libscl_{name}.so")])
        return name
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(4) as ex:
        print(list(ex.map(one, specs)))


def time_all(n=1024, k=512, bs=8192, reps=5, rounds=2):
    import numpy as np
    import torch
    import polar_amd
    from polar_amd import _lib
    from polar_amd import build as b
    libs = [("default", b.LIB_DEV)] + [(f[7:-3], os.path.join(VAR, f)) for f in sorted(os.listdir(VAR))
                                           if f.startswith("libscl_") and f.endswith(".so")]
    fp = polar_amd.reference_frozen_pos(k, n).numpy()
    mask = np.ascontiguousarray(polar_amd.frozen_mask(fp, n), dtype=np.uint8)
    g = torch.Generator(device="cuda").manual_seed(5)
    llr = torch.randn((bs, n), device="cuda", generator=g) * 2.5 + 1.0
    if os.environ.get("SCL_INPUT") == "awgn":  # the bench's input: AWGN LLRs at Eb/N0 = 2 dB
        from polar_amd import channel
        model = channel.System_AWGN_model(n, k, channel.GpuEncoder(torch.as_tensor(fp), n), None, device="cuda",
                                          generator=g)
        with torch.no_grad():
            _, _, llr = model.llrs(bs, torch.tensor(2.0))
        llr = llr.contiguous()
    ref = None
    handles = []
    for name, path in libs:
        L = _lib._declare(ctypes.CDLL(path))
        h = ctypes.c_void_p()
        flags = int(os.environ.get("SCL_FLAGS", "0"))  # e.g. 4 = PL_PLAN_FAST_SCL
        fmode = int(os.environ.get("SCL_FMODE", "0"))
        assert L.pl_plan_create(ctypes.byref(h), n, mask.ctypes.data_as(ctypes.c_void_p), 8, fmode, 30.0, flags) == 0
        handles.append((name, L, h, True))
        if os.environ.get("SCL_WS_AB") == "1":  # the same library without its workspace (exact-f chain cache off)
            handles.append((name + "-nows", L, h, False))
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    # settle the clock before the first timed round (DVFS: a cold MI355X runs its first ~0.1 s of
    # work slower, which otherwise lands on whichever library round 0 times first)
    warm = torch.empty((bs, k), device="cuda")
    wpm = torch.empty((bs, 16), device="cuda", dtype=torch.float64)
    _, L0, h0, _ = handles[0]
    wsb0 = int(L0.pl_scl_workspace_size(h0, bs))
    ws0 = torch.empty((max(wsb0, 1),), dtype=torch.uint8, device="cuda")
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for _ in range(20):
            L0.pl_scl_decode(h0, ctypes.c_void_p(llr.data_ptr()), bs, ctypes.c_void_p(warm.data_ptr()), 0,
                             ctypes.c_void_p(wpm.data_ptr()), ctypes.c_void_p(ws0.data_ptr() if wsb0 else 0), wsb0, stream)
        torch.cuda.synchronize()
    for rnd in range(rounds):
        for name, L, h, use_ws in handles:
            out = torch.empty((bs, k), device="cuda")
            pm = torch.empty((bs, 16), device="cuda", dtype=torch.float64)
            wsb = int(L.pl_scl_workspace_size(h, bs)) if use_ws else 0
            ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device="cuda")
            call = lambda: L.pl_scl_decode(h, ctypes.c_void_p(llr.data_ptr()), bs, ctypes.c_void_p(out.data_ptr()),  # noqa
                                           0, ctypes.c_void_p(pm.data_ptr()),
                                           ctypes.c_void_p(ws.data_ptr() if wsb else 0), wsb, stream)
            assert call() == 0, L.pl_last_error_string()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                call()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / reps
            if ref is None:
                ref = (out.clone(), pm.clone())
            same = torch.equal(out, ref[0]) and torch.equal(pm, ref[1])
            rows = int((out != ref[0]).any(1).sum())  # rows whose bits differ from the first library's
            print(f"round {rnd} {name:16s} {ms:8.3f} ms  {bs / ms / 1e3:7.4f} Mcw/s  identical={same} rows_differing={rows}",
                  flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        import argparse
        ap = argparse.ArgumentParser()
        ap.add_argument("cmd")
        ap.add_argument("--n", type=int, default=1024)
        ap.add_argument("--k", type=int, default=512)
        ap.add_argument("--bs", type=int, default=8192)
        a = ap.parse_args()
        time_all(a.n, a.k, a.bs, reps=int(os.environ.get("SCL_REPS", "5")),
                 rounds=int(os.environ.get("SCL_ROUNDS", "2")))
