"""Development aid: build the code-specialised SC kernel for one (k, n) as a standalone .so and,
on the GPU box, check it bit-exact against the library kernel and time both.

  python tools/static_probe.py build K N [NAME] [extra hipcc flags...]   (container)
  python tools/static_probe.py run K N [NAME...]                           (GPU box)
"""
import ctypes, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "polar-code-pytorch-sionna_amd")
CSRC = os.path.join(PKG, "polar_amd", "csrc")
OUT = os.path.join(PKG, "polar_amd", "_variants")
sys.path.insert(0, PKG)
R0, R1, REP, SPC, GEN = range(5)

def ntable(mask):
    n = len(mask); logn = n.bit_length() - 1
    nt = [0] * (2 * n)
    for s in range(logn + 1):
        S = 1 << s
        for p in range(0, n, S):
            f = mask[p:p + S]
            if f.all(): t = R0
            elif not f.any(): t = R1
            elif S >= 2 and f[:-1].all(): t = REP
            elif S >= 2 and f[0] and not f[1:].any(): t = SPC
            else: t = GEN
            nt[(n >> s) + (p >> s)] = t
    # PROBE_NT_MAP="3:4,1:4:16": demote node types (e.g. SPC/rate-1 -> generic recursion) for A/B,
    # optionally only for nodes of at most / at least the given size ("3:4:16" / "3:4:-32")
    for spec in filter(None, os.environ.get("PROBE_NT_MAP", "").split(",")):
        f = [int(v) for v in spec.split(":")]
        a, b = f[0], f[1]
        lim = f[2] if len(f) > 2 else 0
        for s in range(logn + 1):
            S = 1 << s
            if lim > 0 and S > lim: continue
            if lim < 0 and S < -lim: continue
            for p in range(0, n, S):
                i = (n >> s) + (p >> s)
                if nt[i] == a: nt[i] = b
    return nt

def lg_of(n, name=None):
    """log2(lanes per codeword): the library's rule (n/128), or PROBE_LG / a name ending in _lgK."""
    if name and "_lg" in name:
        return int(name.rsplit("_lg", 1)[1])
    if os.environ.get("PROBE_LG"):
        return int(os.environ["PROBE_LG"])
    logn = n.bit_length() - 1
    return logn - 7 if logn > 7 else 0

def lam(G):
    if G == 1: return [0]
    h = lam(G // 2)
    return h + [G - 1 - x for x in h]

def info_loc(mask, name=None):
    n = len(mask); G = 1 << lg_of(n, name); L = lam(G)
    pos = np.nonzero(mask == 0)[0]
    WPL = (n // G + 31) // 32  # sc_static.h emit encoding (jit.cpp attach_static)
    return np.array([(((L[p % G] * WPL + (p // G) // 32) * 4) << 5) | ((p // G) & 31) for p in pos], dtype=np.int32)

def code_src(mask, fm=0, name=None):
    n = len(mask); logn = n.bit_length() - 1; lg = lg_of(n, name)
    nt = ntable(mask)
    return (f"struct PlCode {{ static constexpr int N = {n}, LOG_N = {logn}, LOG_G = {lg}, G = {1<<lg}, NS = {n>>lg}, FM = {fm};\n"
            f"  static constexpr unsigned char NT[{2*n}] = {{{','.join(map(str, nt))}}}; }};\n")

import numpy as np

def build(k, n, name, flags):
    import polar_amd
    fp = polar_amd.reference_frozen_pos(k, n).numpy()
    mask = polar_amd.frozen_mask(fp, n)
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(OUT, f"st_{name}.hip")
    open(src, "w").write('#include "sc_static.h"\n' + code_src(mask, int(os.environ.get("PROBE_FM", "0")), name) + "PL_SC_STATIC_KERNELS(PlCode)\n" + r'''
extern "C" int st_launch(const float* llr, long bs, void* out, const int* info_loc, int k, float lmax, void* st, long pf) {
    const long per = (long)pls::kWaves * (64 / PlCode::G);
    long blocks = (bs + per - 1) / per;
    if (pf > 0 && pf < blocks) blocks = pf;  // persistent variants: pf = grid size in blocks
    hipLaunchKernelGGL(pl_sc_static_f32, dim3((unsigned)blocks), dim3(64 * pls::kWaves), 0,
                       (hipStream_t)st, llr, (int64_t)bs, out, info_loc, k, lmax);
    return (int)hipGetLastError();
}
''')
    so = os.path.join(OUT, f"st_{name}.so")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-ffp-contract=off", f"-I{CSRC}", *flags, src, "-o", so])
    print("built", so)

def run(k, n, names):
    import torch, polar_amd
    from polar_amd import _lib, channel, ops
    fp = polar_amd.reference_frozen_pos(k, n)
    mask = polar_amd.frozen_mask(fp, n)
    dev = torch.device("cuda")
    bs = 65536 if n >= 512 else 65536
    gen = torch.Generator(device=dev).manual_seed(42)
    model = channel.System_AWGN_model(n, k, channel.GpuEncoder(fp, n), None, device=dev, generator=gen)
    bits, _, llr = model.llrs(bs, torch.tensor(2.0))
    llr = llr.contiguous()
    x2 = (torch.randn(bs, n, device=dev, generator=gen) * 2).contiguous()
    x3 = torch.round(x2 * 2) / 2  # ties and exact zeros
    plan = _lib.Plan(n, mask, 1, int(os.environ.get("PROBE_FM", "0")))
    iloc = torch.from_numpy(info_loc(mask)).to(dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    def tm(fn, reps=20):
        for _ in range(3): fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps): fn()
        e1.record(); torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps
    ref_out = torch.empty((bs, k), device=dev)
    t_ref = tm(lambda: ops.sc_decode(plan, llr, out=ref_out))
    print(f"library kernel ({k},{n}) bs={bs}: {t_ref:.4f} ms  {bs / t_ref / 1e3:.1f} Mcw/s", flush=True)
    for name in names:
        iloc = torch.from_numpy(info_loc(mask, name)).to(dev)
        L = ctypes.CDLL(os.path.join(OUT, f"st_{name}.so"))
        L.st_launch.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_long]
        pfs = [int(v) for v in os.environ.get("PROBE_PF", "0").split(",")]
        if "stamp" in name:
            nw = (bs // (64 // (1 << lg_of(n))))
            big = torch.zeros(bs * k + nw * 16 + 64, device=dev)
            L.st_launch(llr.data_ptr(), bs, big.data_ptr(), iloc.data_ptr(), k, 30.0, st, 0)
            L.st_launch(llr.data_ptr(), bs, big.data_ptr(), iloc.data_ptr(), k, 30.0, st, 0)
            torch.cuda.synchronize()
            d = big[bs * k: bs * k + nw * 16].view(torch.int64).view(nw, 8).cpu().numpy()
            t0 = d[:, 0].min()
            ld, tree, bar, outp = d[:, 1] - d[:, 0], d[:, 2] - d[:, 1], d[:, 3] - d[:, 2], d[:, 4] - d[:, 3]
            tot = d[:, 4] - d[:, 0]
            for nm, v in (("load", ld), ("tree", tree), ("barrier", bar), ("output", outp), ("total", tot)):
                print(f"  stamp {nm}: mean {v.mean():.0f} p10 {np.percentile(v, 10):.0f} p50 {np.median(v):.0f} p90 {np.percentile(v, 90):.0f}")
            print(f"  span {d[:, 4].max() - t0}  start spread p50 {np.median(d[:, 0] - t0):.0f} p90 {np.percentile(d[:, 0] - t0, 90):.0f}")
            np.save(os.path.join(ROOT, "gpurun_out", f"stamps_{name}.npy"), d)
            hw = d[:, 5]
            print("  hw_id sample:", [hex(int(v)) for v in hw[:8]], [hex(int(v)) for v in hw[1024:1032]])
            continue
        out = torch.empty((bs, k), device=dev)
        ok = True
        for x in (llr, x2, x3):
            want = ops.sc_decode(plan, x)
            out.fill_(7)
            assert L.st_launch(x.data_ptr(), bs, out.data_ptr(), iloc.data_ptr(), k, 30.0, st, pfs[-1]) == 0
            torch.cuda.synchronize()
            nbad = int((out != want).any(dim=1).sum())
            ok &= nbad == 0
            if nbad: print(f"  {name}: {nbad} mismatching rows", flush=True)
        for pf in pfs:
            t = tm(lambda: L.st_launch(llr.data_ptr(), bs, out.data_ptr(), iloc.data_ptr(), k, 30.0, st, pf))
            print(f"static[{name}] pf={pf} ({k},{n}): {t:.4f} ms  {bs / t / 1e3:.1f} Mcw/s  exact={ok}", flush=True)

    t_ref = tm(lambda: ops.sc_decode(plan, llr, out=ref_out))
    print(f"library kernel again ({k},{n}) bs={bs}: {t_ref:.4f} ms  {bs / t_ref / 1e3:.1f} Mcw/s", flush=True)
    fn = _lib.lib().pl_sc_decode
    args = (plan.handle, ctypes.c_void_p(llr.data_ptr()), bs, ctypes.c_void_p(ref_out.data_ptr()), 0, st)
    t_dir = tm(lambda: fn(*args))
    print(f"library kernel, direct ctypes call ({k},{n}): {t_dir:.4f} ms  {bs / t_dir / 1e3:.1f} Mcw/s", flush=True)
    import time as _t
    small = llr[:64].contiguous(); so = torch.empty((64, k), device=dev)
    for f_, nm in ((lambda: ops.sc_decode(plan, small, out=so), "ops.sc_decode"),
                   (lambda: fn(plan.handle, ctypes.c_void_p(small.data_ptr()), 64, ctypes.c_void_p(so.data_ptr()), 0, st),
                    "direct")):
        for _ in range(100): f_()
        torch.cuda.synchronize(); t0 = _t.perf_counter()
        for _ in range(2000): f_()
        t1 = _t.perf_counter(); torch.cuda.synchronize()
        print(f"host cost per call ({nm}, bs=64): {(t1 - t0) / 2000 * 1e6:.1f} us", flush=True)

if __name__ == "__main__":
    if sys.argv[1] == "build":
        k, n = int(sys.argv[2]), int(sys.argv[3])
        name = sys.argv[4] if len(sys.argv) > 4 else f"k{k}n{n}"
        build(k, n, name, sys.argv[5:])
    else:
        run(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4:])
