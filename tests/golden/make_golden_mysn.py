"""Golden fixtures for the my_sn decoder extras: CRC and my_sn SCL_Dec.

TEST INFRASTRUCTURE ONLY; runs in the build container (imports the reference read-only from
/root/reference) and writes small .npz files next to this script.

Reference call sites (file:line under /root/reference):
  * CRCEncoder.forward   my_sn/fec/crc.py:85-104 (G-matrix CRC of the 5G polynomials :38-52)
  * CRCDecoder.forward   my_sn/fec/crc.py:119-138
  * SCL_Dec.forward      my_sn/fec/polar/dec.py:476-537 with use_fast_scl=False (plain SCL, exact f)
                         and with crc_degree="CRC11" (CRC-aided pick :507-518)

The reference's CRCEncoder cannot be constructed as shipped: build() reads self.device, which is
never set (crc.py:81; only a module-level `device` exists, crc.py:5).  This script sets the
missing class attribute at run time (CRCEncoder.device = "cpu") before constructing it; nothing
else is changed.  The polar encoding of the CRC test codewords uses the plain XOR butterfly (no
reference code involved).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_mysn.py
"""
import importlib.util
import os
import sys

import numpy as np
import torch as tc

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path += [os.path.join(REF, "x_run_sn_polar"), REF]

import my_sn.fec.crc as refcrc  # noqa: E402

refcrc.CRCEncoder.device = "cpu"  # crc.py:81 reads self.device, which is never assigned

_spec = importlib.util.spec_from_file_location("ref_mysn_dec", os.path.join(REF, "my_sn/fec/polar/dec.py"))
mysn = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mysn)

CRCS = ("CRC24A", "CRC24B", "CRC24C", "CRC16", "CRC11", "CRC6")


def polar_encode(u, info_pos, n):
    x = np.zeros((u.shape[0], n), dtype=np.uint8)
    x[:, info_pos] = u.astype(np.uint8)
    h = 1
    while h < n:
        for a in range(0, n, 2 * h):
            x[:, a:a + h] ^= x[:, a + h:a + 2 * h]
        h *= 2
    return x


def crc_fixture():
    rng = np.random.default_rng(11)
    out = {}
    for name in CRCS:
        for k in (7, 40, 100):
            u = rng.integers(0, 2, (16, k)).astype(np.float32)
            enc = refcrc.CRCEncoder(name, k)
            c = enc(tc.from_numpy(u)).numpy().astype(np.float32)
            bad = c.copy()
            flip = rng.integers(0, k + enc.crc_length, 16)
            bad[np.arange(0, 16, 2), flip[::2]] = 1 - bad[np.arange(0, 16, 2), flip[::2]]
            dec = refcrc.CRCDecoder(refcrc.CRCEncoder(name, k + enc.crc_length))
            _, valid = dec(bad)
            out[f"{name}_k{k}_u"] = u
            out[f"{name}_k{k}_enc"] = c
            out[f"{name}_k{k}_word"] = bad
            out[f"{name}_k{k}_valid"] = np.asarray(valid).reshape(-1).astype(np.uint8)
            print(f"  {name} k={k}: crc len {enc.crc_length}, valid {int(np.asarray(valid).sum())}/16")
    np.savez_compressed(os.path.join(OUT, "crc.npz"), **out)


class _Stable:
    def __getattr__(self, name):
        return getattr(np, name)

    @staticmethod
    def argsort(a, axis=-1):
        return np.argsort(a, axis=axis, kind="stable")


def run_mysn(fp, n, L, x, stable, **kw):
    saved = mysn.np
    if stable:
        mysn.np = _Stable()
    try:
        dec = mysn.SCL_Dec(fp, n, list_size=L, **kw)
        b = dec(tc.from_numpy(x)).numpy().astype(np.uint8)
        return b, np.asarray(dec.msg_pm, dtype=np.float64)
    finally:
        mysn.np = saved


def scl_fixture(tag, k, n, L, sets, **kw):
    fs = np.load(os.path.join(OUT, "frozen_sets.npz"))
    fp = fs[f"k{k}_n{n}"].astype(np.int64)
    out = {"frozen_pos": fp.astype(np.int16), "k": k, "n": n, "L": L}
    for name, x in sets.items():
        b, pm = run_mysn(fp, n, L, x, False, **kw)
        bs_, pms = run_mysn(fp, n, L, x, True, **kw)
        out[f"llr_{name}"] = x
        out[f"bits_{name}"] = b
        out[f"pm_{name}"] = pm
        out[f"bits_stable_{name}"] = bs_
        out[f"pm_stable_{name}"] = pms
        print(f"  my_sn SCL {tag} L={L} ({k},{n}) {name}: rows={len(x)} tie-order rows changed "
              f"{int((b != bs_).any(1).sum())}")
    np.savez_compressed(os.path.join(OUT, f"mysn_scl_{tag}_L{L}_{k}_{n}.npz"), **out)


def main():
    tc.set_num_threads(8)
    crc_fixture()
    rng = np.random.default_rng(5)
    g = tc.Generator().manual_seed(1234)
    rand64 = (tc.randn(24, 64, generator=g) * 2).numpy().astype(np.float32)
    awgn = lambda bits, sd: ((2.0 * bits - 1.0) * 2.0 + rng.standard_normal(bits.shape) * sd).astype(np.float32)
    fs = np.load(os.path.join(OUT, "frozen_sets.npz"))
    # plain SCL (no pruning), exact f
    fp = fs["k32_n64"].astype(np.int64)
    info = np.setdiff1d(np.arange(64), fp)
    cw = polar_encode(rng.integers(0, 2, (24, 32)), info, 64)
    scl_fixture("nofast", 32, 64, 4, {"rand": rand64, "awgn": awgn(cw, 1.2)}, use_fast_scl=False)
    # CRC-aided: information words carry a CRC11 (21 data + 11 parity bits)
    enc = refcrc.CRCEncoder("CRC11", 21)
    u = enc(tc.from_numpy(rng.integers(0, 2, (32, 21)).astype(np.float32))).numpy()
    cw = polar_encode(u, info, 64)
    scl_fixture("crc11", 32, 64, 8, {"rand": rand64, "awgn": awgn(cw, 1.3), "awgn_hi": awgn(cw, 1.6)},
                crc_degree="CRC11")
    fp = fs["k128_n256"].astype(np.int64)
    info = np.setdiff1d(np.arange(256), fp)
    enc = refcrc.CRCEncoder("CRC24C", 104)
    u = enc(tc.from_numpy(rng.integers(0, 2, (12, 104)).astype(np.float32))).numpy()
    cw = polar_encode(u, info, 256)
    scl_fixture("crc24c", 128, 256, 8, {"awgn": awgn(cw, 1.4)}, crc_degree="CRC24C")


if __name__ == "__main__":
    main()
