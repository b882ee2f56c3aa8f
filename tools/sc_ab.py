"""Development aid: same-process A/B of specialised SC kernel variants through the product path
(pl_sc_source -> hipcc --genco -> plan from the code-object cache), exactly what Plan() runs.

  python tools/sc_ab.py build NAME="DEF=V ..." NAME2="@alt_sc_static.h DEF=V" ... [--k 512 --n 1024]
        (container: hipcc --genco into polar_amd/_variants/kcache; specs kept in _variants/ab.json)
  python tools/sc_ab.py run NAME ... [--k 512 --n 1024 --rounds 5 --bs 65536]      (GPU box)

A variant is a set of macro overrides (PL_SC_DEFINES) and optionally another sc_static.h body
(PL_SC_SOURCE, "@file"); "base" is the unmodified source.  `run` checks every variant bit-exact
against the base kernel on AWGN, random and tie/zero-heavy LLRs, then times all of them
interleaved for several rounds (kernel time by HIP events).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "polar-code-pytorch-sionna_amd")
VAR = os.path.join(PKG, "polar_amd", "_variants")
KC = os.path.join(VAR, "kcache")
SPECS = os.path.join(VAR, "ab.json")
sys.path.insert(0, PKG)
from polar_amd import _lib as _pl_lib  # noqa: E402

_pl_lib.use_dev_library()  # the A/B hooks (PL_SC_DEFINES, PL_SC_SOURCE, PL_SC_LOG_G) exist only in the dev build


def _env(spec):
    src = ""
    if spec.startswith("@"):
        src, _, spec = spec[1:].partition(" ")
    # "LOG_G=k" in a spec selects the lanes per codeword (jit.cpp PL_SC_LOG_G), not a macro
    toks = spec.split()
    lg = [t for t in toks if t.startswith("LOG_G=")]
    spec = " ".join(t for t in toks if not t.startswith("LOG_G="))
    if lg:
        os.environ["PL_SC_LOG_G"] = lg[0].split("=")[1]
    else:
        os.environ.pop("PL_SC_LOG_G", None)
    if spec:
        os.environ["PL_SC_DEFINES"] = spec
    else:
        os.environ.pop("PL_SC_DEFINES", None)
    if src:
        os.environ["PL_SC_SOURCE"] = src if os.path.isabs(src) else os.path.join(VAR, src)
    else:
        os.environ.pop("PL_SC_SOURCE", None)


def _mask(k, n):
    import polar_amd
    return polar_amd.frozen_mask(polar_amd.reference_frozen_pos(k, n), n)


def _load_specs():
    return json.load(open(SPECS)) if os.path.exists(SPECS) else {"base": ""}


def build(names, k, n, fm):
    from concurrent.futures import ThreadPoolExecutor

    from polar_amd import build as _b
    _b.build(dev=True)

    from polar_amd import _lib
    os.makedirs(KC, exist_ok=True)
    specs = _load_specs()
    for a in names:
        name, _, defs = a.partition("=")
        if "=" in a:
            specs[name] = defs
    json.dump(specs, open(SPECS, "w"), indent=1)
    m = _mask(k, n)
    jobs = []
    for a in names:
        name = a.partition("=")[0]
        _env(specs[name])
        src, cname = _lib.sc_source(n, m, fm)
        jobs.append((name, src, cname))
    _env("")

    def one(job):
        name, src, cname = job
        ok = os.path.exists(os.path.join(KC, cname)) or _lib.compile_code_object(src, KC, cname)
        return name, cname, ok
    with ThreadPoolExecutor(8) as ex:
        for r in ex.map(one, jobs):
            print(*r, flush=True)


def run(names, k, n, fm, rounds, bs, only=False, rotate=1):
    import torch

    import polar_amd
    from polar_amd import _lib, channel, ops
    specs = _load_specs()
    os.environ["PL_KERNEL_CACHE"] = KC
    m = _mask(k, n)
    fp = polar_amd.reference_frozen_pos(k, n)
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(42)
    model = channel.System_AWGN_model(n, k, channel.GpuEncoder(fp, n), None, device=dev, generator=gen)
    _, _, llr = model.llrs(bs, torch.tensor(2.0))
    llr = llr.contiguous()
    x2 = (torch.randn(bs, n, device=dev, generator=gen) * 2).contiguous()
    x3 = torch.round(x2 * 2) / 2
    x4 = (x2 * 40).contiguous()
    plans = {}
    for name in (names if only else ["base"] + [v for v in names if v != "base"]):
        _env(specs[name])
        p = _lib.Plan(n, m, 1, fm, flags=_lib.PL_PLAN_CACHE_ONLY)
        kind, path = p.kernel()
        if kind != "specialized":
            print(f"{name}: not built ({kind})", flush=True)
            continue
        plans[name] = p
    _env("")
    out = torch.empty((bs, k), device=dev)
    gplan = _lib.Plan(n, m, 1, fm, flags=_lib.PL_PLAN_GENERIC)  # independent kernel as the reference
    for name, p in ({} if only else plans).items():
        bad = 0
        for x in (llr, x2, x3, x4):
            want = ops.sc_decode(gplan, x)
            got = ops.sc_decode(p, x)
            bad += int((got != want).any(dim=1).sum())
        print(f"{name}: {'exact' if bad == 0 else f'{bad} MISMATCHING ROWS'} vs the generic kernel", flush=True)

    # rotate > 1: cycle through that many input/output buffer pairs, so the Infinity Cache
    # (256 MB) cannot hold an input across launches
    ins = [llr] + [llr.clone() for _ in range(rotate - 1)]
    outs = [out] + [torch.empty_like(out) for _ in range(rotate - 1)]

    def tm(p, reps=20 if only else 200):
        for r in range(20):
            ops.sc_decode(p, ins[r % rotate], out=outs[r % rotate])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for r in range(reps):
            ops.sc_decode(p, ins[r % rotate], out=outs[r % rotate])
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps
    # settle the clock
    first = next(iter(plans.values()))
    for _ in range(20 if only else 2000):
        ops.sc_decode(first, llr, out=out)
    res = {nm: [] for nm in plans}
    for r in range(rounds):
        for nm, p in plans.items():
            res[nm].append(tm(p))
    for nm, ts in res.items():
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        rel = f"({med / sorted(res['base'])[len(ts) // 2]:.3f}x base)" if "base" in res else ""
        print(f"{nm:24s} median {med:.4f} ms  min {ts[0]:.4f}  {bs / med / 1e3:.1f} Mcw/s  {rel}", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("names", nargs="+")
    ap.add_argument("--k", type=int, default=512)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--fm", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--bs", type=int, default=65536)
    ap.add_argument("--only", action="store_true", help="run: time the named variants only (no base, no check)")
    ap.add_argument("--rotate", type=int, default=1, help="run: cycle through this many input/output buffers")
    a = ap.parse_args()
    if a.cmd == "build":
        build(a.names, a.k, a.n, a.fm)
    else:
        run(a.names, a.k, a.n, a.fm, a.rounds, a.bs, a.only, a.rotate)
