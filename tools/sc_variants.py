"""Development aid: A/B the specialised SC kernel under different tuning macros, through the
product path (jit.cpp + hiprtc), in one process on the GPU.

  python tools/sc_variants.py build NAME="DEF=V DEF=V" ...   (container: hiprtc into _variants/kcache)
     a spec may start with "@file.h " to compile another version of sc_static.h (PL_SC_SOURCE)
  python tools/sc_variants.py run NAME ... [--k 512 --n 1024 --rounds 5]   (GPU box)
Specs are remembered in _variants/specs.json.
"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "polar-code-pytorch-sionna_amd")
VAR = os.path.join(PKG, "polar_amd", "_variants")
KC = os.path.join(VAR, "kcache")
SPECS = os.path.join(VAR, "specs.json")
sys.path.insert(0, PKG)
from polar_amd import _lib as _pl_lib  # noqa: E402

_pl_lib.use_dev_library()  # the A/B hooks (PL_SC_DEFINES, PL_SC_SOURCE, PL_SC_LOG_G) exist only in the dev build


def _env(spec):
    src = ""
    if spec.startswith("@"):
        src, _, spec = spec[1:].partition(" ")
    os.environ["PL_SC_DEFINES"] = spec
    if src:
        os.environ["PL_SC_SOURCE"] = src if os.path.isabs(src) else os.path.join(VAR, src)
    else:
        os.environ.pop("PL_SC_SOURCE", None)


def _mask(k, n):
    import polar_amd
    return polar_amd.frozen_mask(polar_amd.reference_frozen_pos(k, n), n)


def build(args, k=512, n=1024):
    from polar_amd import build as _b
    _b.build(dev=True)
    os.makedirs(KC, exist_ok=True)
    specs = json.load(open(SPECS)) if os.path.exists(SPECS) else {}
    from concurrent.futures import ProcessPoolExecutor
    for a in args:
        name, defs = a.split("=", 1) if "=" in a.split()[0] else (a, "")
        specs[name] = defs
    json.dump(specs, open(SPECS, "w"), indent=1)
    jobs = [(specs[a.split("=", 1)[0]], k, n) for a in args]
    with ProcessPoolExecutor(8) as ex:
        for r in ex.map(_one, jobs):
            print(r)


def _one(job):
    import ctypes
    defs, k, n = job
    _env(defs)
    from polar_amd import _lib
    _lib.use_dev_library()
    m = _mask(k, n)
    buf = ctypes.create_string_buffer(4096)
    rc = _lib.lib().pl_sc_specialize(n, m.ctypes.data_as(ctypes.c_void_p), 0, KC.encode(), buf, 4096)
    return (defs, rc, buf.value.decode() if rc == 0 else _lib.lib().pl_last_error_string().decode()[:3000])


def run(names, k=512, n=1024, rounds=5, reps=20, bs=65536):
    import numpy as np
    import torch
    import polar_amd
    from polar_amd import _lib, channel, ops
    specs = json.load(open(SPECS))
    os.environ["PL_KERNEL_CACHE"] = KC
    fp = polar_amd.reference_frozen_pos(k, n)
    mask = polar_amd.frozen_mask(fp, n)
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(42)
    model = channel.System_AWGN_model(n, k, channel.GpuEncoder(fp, n), None, device=dev, generator=gen)
    _, _, llr = model.llrs(bs, torch.tensor(2.0))
    llr = llr.contiguous()
    x2 = (torch.randn(bs, n, device=dev, generator=gen) * 2).contiguous()
    x3 = torch.round(x2 * 2) / 2
    gplan = _lib.Plan(n, mask, 1, 0, flags=_lib.PL_PLAN_GENERIC)
    plans = {}
    for nm in names:
        _env(specs[nm])
        p = _lib.Plan(n, mask, 1, 0, flags=_lib.PL_PLAN_CACHE_ONLY)
        assert p.kernel()[0] == "specialized", (nm, p.kernel())
        plans[nm] = p
    _env("")
    out = torch.empty((bs, k), device=dev)
    for nm, p in plans.items():
        bad = 0
        for x in (llr, x2, x3):
            bad += int((ops.sc_decode(p, x) != ops.sc_decode(gplan, x)).any(1).sum())
        print(f"{nm}: exact={bad == 0} ({bad} rows differ)  [{specs[nm]}]", flush=True)
    times = {nm: [] for nm in plans}
    for r in range(rounds):
        for nm, p in plans.items():
            for _ in range(3):
                ops.sc_decode(p, llr, out=out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                ops.sc_decode(p, llr, out=out)
            e1.record()
            torch.cuda.synchronize()
            times[nm].append(e0.elapsed_time(e1) / reps)
    for nm, t in times.items():
        t = np.array(t)
        print(f"{nm:12s} min {t.min():.4f} ms  med {np.median(t):.4f} ms  ({bs / t.min() / 1e3:.1f} Mcw/s best)", flush=True)


if __name__ == "__main__":
    import argparse
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        ap = argparse.ArgumentParser()
        ap.add_argument("names", nargs="+")
        ap.add_argument("--k", type=int, default=512)
        ap.add_argument("--n", type=int, default=1024)
        ap.add_argument("--rounds", type=int, default=5)
        a = ap.parse_args(sys.argv[2:])
        run(a.names, a.k, a.n, a.rounds)
