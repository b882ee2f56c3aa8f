"""Development aid: per-phase time of the SCL subtree kernel (PL_SCL_PROF, s_memtime per wave).

  python tools/scl_prof.py build                     (container: the variant library libscl_prof.so)
  python tools/scl_prof.py run [--fmode 0|1] [--fast] [--bs 8192]     (GPU box)

Prints, per phase of the decoder loop (scl_tree_kernel.hip, PL_SCL_PROF), the mean cycles per wave,
the share of the sum, and the decode time of the same launch without instrumentation (default
library) for scale.
"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "polar-code-pytorch-sionna_amd")
VAR = os.path.join(PKG, "polar_amd", "_variants")
sys.path.insert(0, PKG)
PHASES = ["virtual f passes", "stored passes", "subtree rest", "repoint+ps", "combines", "virt g / pruned",
          "set-up", "final", "subtree f/g", "subtree pen", "subtree rank", "subtree moves"]
NS = len(PHASES)


def run(fmode, fast, bs, n=1024, k=512, L=8, reps=3, variants=("prof",)):
    import numpy as np
    import torch
    import polar_amd
    from polar_amd import _lib
    from polar_amd import build as b
    fp = polar_amd.reference_frozen_pos(k, n).numpy()
    mask = np.ascontiguousarray(polar_amd.frozen_mask(fp, n), dtype=np.uint8)
    g = torch.Generator(device="cuda").manual_seed(5)
    llr = torch.randn((bs, n), device="cuda", generator=g) * 2.5 + 1.0
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    waves = (bs + (32 // L) - 1) // (32 // L)
    res = {}
    for name, path in [("default", b.LIB_DEV)] + [(v, os.path.join(VAR, f"libscl_{v}.so")) for v in variants]:
        lib = _lib._declare(ctypes.CDLL(path))
        h = ctypes.c_void_p()
        assert lib.pl_plan_create(ctypes.byref(h), n, mask.ctypes.data_as(ctypes.c_void_p), L, fmode, 30.0,
                                  4 if fast else 0) == 0
        out = torch.empty((bs, k), device="cuda")
        pm = torch.zeros((bs * 2 * L + waves * NS,), device="cuda", dtype=torch.float64)
        wsb = int(lib.pl_scl_workspace_size(h, bs))
        ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device="cuda")

        def call():
            return lib.pl_scl_decode(h, ctypes.c_void_p(llr.data_ptr()), bs, ctypes.c_void_p(out.data_ptr()), 0,
                                     ctypes.c_void_p(pm.data_ptr()), ctypes.c_void_p(ws.data_ptr() if wsb else 0),
                                     wsb, stream)
        assert call() == 0, lib.pl_last_error_string()
        for _ in range(10):  # settle the clock
            call()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            call()
        e.record()
        torch.cuda.synchronize()
        res[name] = (s.elapsed_time(e) / reps, out.clone(), pm[bs * 2 * L:].view(torch.int64).cpu().numpy())
        lib.pl_plan_destroy(h)
    for v in variants:
        print(f"fmode={fmode} fast={fast} bs={bs}: default {res['default'][0]:.4f} ms, {v} "
              f"{res[v][0]:.4f} ms, decisions identical: {bool(torch.equal(res['default'][1], res[v][1]))}")
        cyc = res[v][2].reshape(waves, NS).astype(np.float64)
        tot = cyc.sum(axis=1).mean()
        for i, ph in enumerate(PHASES):
            m = cyc[:, i].mean()
            print(f"  {ph:16s} {m:12.0f} cycles/wave  {100 * m / tot:5.1f} %")
        print(f"  {'sum':16s} {tot:12.0f} cycles/wave  (max over waves {cyc.sum(axis=1).max():.0f})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run"])
    ap.add_argument("--fmode", type=int, default=0)
    ap.add_argument("--fast", action="store_true")
    ap.add_argument("--bs", type=int, default=8192)
    ap.add_argument("--variants", default="prof", help="comma-separated variant libraries built with PL_SCL_PROF=1")
    ap.add_argument("--flags", nargs="*", default=[], help="build: NAME:-D... variant specs (PL_SCL_PROF=1 added)")
    a = ap.parse_args()
    if a.mode == "build":
        specs = ["prof:-DPL_SCL_PROF=1"] + [f"{sp} -DPL_SCL_PROF=1" for sp in a.flags]
        subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "scl_variants.py"), "build", *specs])
    else:
        run(a.fmode, a.fast, a.bs, variants=tuple(a.variants.split(",")))


if __name__ == "__main__":
    main()
