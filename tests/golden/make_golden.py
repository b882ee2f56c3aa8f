"""Generate the golden fixtures under tests/golden/ from the reference decoders.

TEST INFRASTRUCTURE ONLY.  This script imports the reference (jaco267/polar-code-pytorch-sionna,
read-only at /root/reference) and therefore runs only in the build container; the GPU box never
sees the reference.  Its outputs (small .npz files of inputs and expected outputs) are committed
and are what the oracle and the HIP kernels are pinned against.

Reference call sites used (file:line under /root/reference):
  * frozen sets   x_run_sn_polar/polar/froze.py:4-16      get_Kern_frozen_bits (torch argsort ties)
  * SC min-sum    x_run_sn_polar/polar/polar_sc.py:113-133 SC_Dec.forward
  * SCL (x_run)   x_run_sn_polar/polar/polar_scl.py:210-234 SCL_Dec.forward (+ msg_pm after :204)
  * SC exact      my_sn/fec/polar/dec.py:130-157           SC_Dec.forward (exact boxplus f)
  * SCL (my_sn)   my_sn/fec/polar/dec.py:476-537           SCL_Dec.forward (fast-SCL, exact f)
  * harness       x_run_sn_polar/z_sys_model/awgn_model.py:33-44, my_sn/sim.py:19-140,
                  x_run_sn_polar/main.py:24-59 (seed 42 per code), config 1 = (32,64), bs=100
The harness encoder (x_run_sn_polar/polar/enc.py:30-43) cannot be imported here (it pulls in
importlib_resources, absent), so an arithmetic twin (c[:,info_pos]=u; (c@G)%2) is used; it consumes
no RNG, so the RNG call order is untouched.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import hashlib
import importlib.util
import os
import sys
import time

import numpy as np
import torch as tc

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
PKG_DATA = os.path.join(os.path.dirname(os.path.dirname(OUT)),
                        "polar-code-pytorch-sionna_amd", "polar_amd", "data")
sys.dont_write_bytecode = True
sys.path += [os.path.join(REF, "x_run_sn_polar"), REF]

from polar.froze import get_Kern_frozen_bits  # noqa: E402
from polar.polar_sc import SC_Dec as XSC  # noqa: E402
from polar.polar_scl import SCL_Dec as XSCL  # noqa: E402
from z_sys_model.awgn_model import System_AWGN_model  # noqa: E402
from my_sn.sim import sim_ber  # noqa: E402

_spec = importlib.util.spec_from_file_location("ref_mysn_dec", os.path.join(REF, "my_sn/fec/polar/dec.py"))
mysn = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mysn)

F2 = tc.tensor([[1, 0], [1, 1]], dtype=tc.float32)


def h16(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def frozen(k, n):
    G, _, fp = get_Kern_frozen_bits(n, n - k, F2)
    return G, fp


class DenseEncoder(tc.nn.Module):
    """Arithmetic twin of x_run_sn_polar/polar/enc.py:30-43 (c[:,info]=u; (c@G)%2, fp32)."""

    def __init__(self, frozen_pos, n, G):
        super().__init__()
        self.n = n
        self.info_pos = np.setdiff1d(np.arange(n), np.asarray(frozen_pos))
        self.G = G

    def forward(self, u):
        c = tc.zeros([u.shape[0], self.n], dtype=tc.float32)
        c[..., tc.from_numpy(self.info_pos)] = u
        return (c @ self.G % 2).to(tc.float32)


class Capture(tc.nn.Module):
    """Decoder wrapper that records the LLR logits it is handed."""

    def __init__(self, inner):
        super().__init__()
        self.inner = inner
        self.seen = []

    def forward(self, llr):
        self.seen.append(llr.clone())
        return self.inner(llr)


def awgn_llrs(k, n, bs, ebno_db, seed):
    G, fp = frozen(k, n)
    cap = Capture(XSC(fp, n))
    model = System_AWGN_model(n, k, DenseEncoder(fp, n, G), cap)
    tc.manual_seed(seed)
    model(bs, tc.tensor(ebno_db, dtype=tc.float32))
    return cap.seen[0].numpy().astype(np.float32)


def llr_sets(k, n, bs, small_bs):
    g = tc.Generator().manual_seed(1234)
    rand = (tc.randn(bs, n, generator=g) * 2).numpy()
    g = tc.Generator().manual_seed(99)
    z = (tc.randn(small_bs, n, generator=g) * 2)
    mask = tc.rand(small_bs, n, generator=g) < 0.3
    z[mask] = 0.0
    neg = tc.rand(small_bs, n, generator=g) < 0.5
    z[mask & neg] = -0.0
    ties = tc.round(tc.randn(small_bs, n, generator=g) * 2)
    sat = tc.randn(small_bs, n, generator=g) * 40
    sets = {
        "rand": rand.astype(np.float32),
        "zeros": z.numpy().astype(np.float32),
        "ties": ties.numpy().astype(np.float32),
        "sat": sat.numpy().astype(np.float32),
    }
    for db in (0.0, 2.0, 4.0):
        sets[f"awgn{int(db)}"] = awgn_llrs(k, n, small_bs, db, seed=7 + int(db))
    return sets


def sc_fixture(k, n, bs, small_bs):
    _, fp = frozen(k, n)
    dec = XSC(fp, n)
    ex = mysn.SC_Dec(fp, n)
    out = {"frozen_pos": fp.numpy().astype(np.int16), "k": k, "n": n}
    for name, llr in llr_sets(k, n, bs, small_bs).items():
        x = tc.from_numpy(llr)
        b = dec(x).numpy().astype(np.uint8)
        e = ex(x).numpy().astype(np.uint8)
        out[f"llr_{name}"] = llr
        out[f"bits_{name}"] = b
        out[f"exact_{name}"] = e
        print(f"  SC ({k},{n}) {name:6s} bs={llr.shape[0]:4d} bits {h16(b)} ones={int(b.sum())} "
              f"exact-vs-minsum rows differ={int((e != b).any(1).sum())}")
    np.savez_compressed(os.path.join(OUT, f"sc_{k}_{n}.npz"), **out)


class _StableArgsortNumpy:
    """numpy proxy whose argsort is stable.  The reference sorts path metrics with np.argsort
    (polar_scl.py:88, dec.py:322), whose tie order is host-dependent (AVX-512 sort here).  Running
    the reference once more with this proxy gives the deterministic-tie-order golden the
    decoders are held to on inputs that produce exact path-metric ties."""

    def __getattr__(self, name):
        return getattr(np, name)

    @staticmethod
    def argsort(a, axis=-1):
        return np.argsort(a, axis=axis, kind="stable")


def _run_scl(tag, fp, n, L, x, stable):
    mod = sys.modules[XSCL.__module__] if tag == "x_run" else mysn
    saved = mod.np
    if stable:
        mod.np = _StableArgsortNumpy()
    try:
        dec = XSCL(fp, n, list_size=L) if tag == "x_run" else mysn.SCL_Dec(fp, n, list_size=L)
        b = dec(x).numpy().astype(np.uint8)
        return b, np.asarray(dec.msg_pm, dtype=np.float64)
    finally:
        mod.np = saved


def scl_fixture(k, n, L, rows, set_names, tag="x_run"):
    _, fp = frozen(k, n)
    sets = llr_sets(k, n, rows, rows)
    out = {"frozen_pos": fp.numpy().astype(np.int16), "k": k, "n": n, "L": L}
    for name in set_names:
        llr = sets[name][:rows]
        x = tc.from_numpy(llr)
        t0 = time.time()
        b, pm = _run_scl(tag, fp, n, L, x, stable=False)
        bs_, pms = _run_scl(tag, fp, n, L, x, stable=True)
        out[f"llr_{name}"] = llr
        out[f"bits_{name}"] = b
        out[f"pm_{name}"] = pm
        out[f"bits_stable_{name}"] = bs_
        out[f"pm_stable_{name}"] = pms
        print(f"  SCL[{tag}] L={L} ({k},{n}) {name:6s} rows={rows} bits {h16(b)} "
              f"pm0={pm[0, 0]!r} rows changed by stable tie order: {int((b != bs_).any(1).sum())} "
              f"({time.time() - t0:.1f}s)")
    fn = f"scl_L{L}_{k}_{n}.npz" if tag == "x_run" else f"mysn_scl_L{L}_{k}_{n}.npz"
    np.savez_compressed(os.path.join(OUT, fn), **out)


def harness_fixture():
    """Config 1 end to end: main.py:42-59 with (k,n)=(32,64), bs=100, mc_iter=1, SNR 0:0.5:4.5."""
    k, n, bs = 32, 64, 100
    ebno = np.arange(0, 5, 0.5)
    G, fp = frozen(k, n)
    out = {"ebno_db": ebno, "k": k, "n": n, "bs": bs}
    for name, dec in (("sc", XSC(fp, n)), ("scl8", XSCL(fp, n, list_size=8))):
        cap = Capture(dec)
        model = System_AWGN_model(n, k, DenseEncoder(fp, n, G), cap)
        np.random.seed(42)
        tc.manual_seed(42)
        ber, bler = sim_ber(model, ebno, bs, max_mc_iter=1, target_block_errs=1000, verbose=False)
        out[f"{name}_ber"] = ber.numpy()
        out[f"{name}_bler"] = bler.numpy()
        out[f"{name}_llr"] = np.stack([s.numpy() for s in cap.seen]).astype(np.float32)
        print(f"  harness {name}: bler={np.round(bler.numpy(), 4).tolist()}")
    np.savez_compressed(os.path.join(OUT, "harness_c1.npz"), **out)


def main():
    tc.set_num_threads(8)
    # frozen sets: every power-of-two n up to 4096 at rates 1/4, 1/2, 3/4 (+ the config shapes)
    fs = {}
    for m in range(1, 13):
        n = 1 << m
        for k in sorted({n // 4, n // 2, (3 * n) // 4, n - 1, 1}):
            if 0 < k < n:
                fs[f"k{k}_n{n}"] = frozen(k, n)[1].numpy().astype(np.int16)
    for key, ref in (("k32_n64", "d18446833e4c61a5"), ("k128_n256", "654dbde04f5616e2"),
                     ("k512_n1024", "3cc861afe3878fc7")):
        got = h16(fs[key].astype(np.int64))
        print(f"frozen {key}: {got} (survey {ref}) {'OK' if got == ref else 'MISMATCH'}")
    np.savez_compressed(os.path.join(OUT, "frozen_sets.npz"), **fs)
    os.makedirs(PKG_DATA, exist_ok=True)
    np.savez_compressed(os.path.join(PKG_DATA, "frozen_sets.npz"), **fs)

    for (k, n, bs, sbs) in ((2, 4, 64, 64), (4, 8, 128, 64), (8, 16, 128, 64), (16, 32, 128, 64),
                            (32, 64, 256, 64), (16, 64, 64, 64), (48, 64, 64, 64),
                            (128, 256, 256, 64), (256, 512, 64, 32), (512, 1024, 256, 32),
                            (1024, 2048, 32, 16)):
        sc_fixture(k, n, bs, sbs)
    for L in (1, 2, 4, 8, 16):
        scl_fixture(32, 64, L, 64, ("rand", "zeros", "ties", "sat", "awgn0", "awgn2"))
    scl_fixture(8, 16, 8, 64, ("rand", "zeros", "ties", "sat"))
    scl_fixture(128, 256, 8, 64, ("rand", "ties", "sat", "awgn2"))
    scl_fixture(128, 256, 4, 32, ("rand", "awgn2"))
    scl_fixture(512, 1024, 8, 16, ("rand", "sat", "awgn2"))
    scl_fixture(32, 64, 8, 32, ("rand", "awgn2"), tag="my_sn")
    scl_fixture(128, 256, 8, 16, ("rand", "awgn2"), tag="my_sn")
    harness_fixture()


if __name__ == "__main__":
    main()
