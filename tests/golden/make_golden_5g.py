"""Golden fixtures for the 5G rate-matching wrapper: Polar5GEncoder and
Polar5GDecoder of my_sn/fec/polar (enc.py:115-392, dec.py:539-666) and the 5G reliability
sequence (utils.py:6-71, codes/polar_5G.csv = 3GPP TS 38.212 Table 5.3.1.2-1).

TEST INFRASTRUCTURE ONLY; runs in the build container (imports the reference read-only from
/root/reference) and writes tests/golden/polar5g.npz plus the package data file
polar_amd/data/polar5g_ranking.npy (the reliability table, a 3GPP standard table).

Run-time shims, set by this script only (nothing in the reference is modified):
  * `importlib_resources` is not installed: a module object exposing the standard library's
    importlib.resources.files / as_file is placed in sys.modules (utils.py:4 imports it).
  * The reference's CRCEncoder cannot be constructed as shipped: build() reads self.device,
    which is never set (crc.py:81).  The class attribute CRCEncoder.device = "cpu" is set.
  * PolarEncoder.forward (enc.py:97-114) asserts H @ c == 0 with a parity-check matrix; kept.
Downlink: Polar5GEncoder.forward raises for channel_type="downlink" (enc.py:375-377), so
downlink cases record the rate-matching tables only.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_5g.py
"""
import importlib.resources
import os
import sys
import types

import numpy as np
import torch as tc

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
PKG_DATA = os.path.join(OUT, "..", "..", "polar-code-pytorch-sionna_amd", "polar_amd", "data")
sys.dont_write_bytecode = True
sys.path += [REF]

_shim = types.ModuleType("importlib_resources")
_shim.files = importlib.resources.files
_shim.as_file = importlib.resources.as_file
sys.modules["importlib_resources"] = _shim

import my_sn.fec.crc as refcrc  # noqa: E402

refcrc.CRCEncoder.device = "cpu"  # crc.py:81 reads self.device, which is never assigned

from my_sn.fec.polar import Polar5GDecoder, Polar5GEncoder  # noqa: E402
from my_sn.fec.polar.utils import generate_5g_ranking  # noqa: E402

# (k, n): uplink CRC6 (12 <= k <= 19) and CRC11; puncturing (K/E <= 7/16, E < N), shortening
# (E < N, K/E > 7/16), repetition (E >= N), and E = N
UPLINK = [(12, 20), (12, 160), (16, 64), (19, 100), (20, 40), (24, 300), (32, 64), (40, 100), (48, 64),
          (64, 128), (64, 200), (100, 180), (120, 1000), (140, 576), (200, 400), (250, 300),
          (300, 1088), (500, 1024), (512, 700), (1013, 1088), (30, 1088), (64, 1024)]
DOWNLINK = [(20, 64), (40, 100), (100, 300), (140, 576), (1, 25), (20, 50)]


def ebno_logits(c, ebno_db, rate, rng):
    """BPSK-equivalent AWGN logits log P(b=1)/P(b=0) (QPSK per-bit LLRs, mapping.py sign)."""
    no = 1.0 / (10 ** (ebno_db / 10) * rate * 2)
    s = 1.0 - 2.0 * c  # bit 0 -> +1
    y = s + rng.standard_normal(c.shape) * np.sqrt(no)
    return (-4.0 * y / (2 * no) * 0.5).astype(np.float32)


def main():
    out = {}
    ch = np.genfromtxt(os.path.join(REF, "my_sn/fec/polar/codes/polar_5G.csv"), delimiter=";").astype(np.int16)
    os.makedirs(PKG_DATA, exist_ok=True)
    np.save(os.path.join(PKG_DATA, "polar5g_ranking.npy"), ch)
    for n in (32, 64, 128, 256, 512, 1024):
        for k in (1, n // 4, n // 2, n - 1):
            fz, info = generate_5g_ranking(k, n)
            out[f"rank_{k}_{n}_frozen"] = fz.astype(np.int16)
        r, _ = generate_5g_ranking(0, n, sort=False)
        out[f"rank_0_{n}_unsorted"] = r.astype(np.int16)
    rng = np.random.default_rng(2024)
    tc.manual_seed(5)
    for k, n in UPLINK:
        enc = Polar5GEncoder(k, n, channel_type="uplink")
        tag = f"ul_{k}_{n}"
        out[tag + "_frozen"] = np.asarray(enc._frozen_pos).astype(np.int16)
        out[tag + "_idx_rm"] = np.asarray(enc._ind_rate_matching).astype(np.int16)
        out[tag + "_meta"] = np.array([enc.k_polar, enc.n_polar, enc.enc_crc.crc_length], dtype=np.int32)
        u = rng.integers(0, 2, (24, k)).astype(np.float32)
        c = enc(tc.from_numpy(u)).numpy().astype(np.float32)
        out[tag + "_u"] = u
        out[tag + "_c"] = c
        llr = ebno_logits(c, 1.5 if k * 2 < n else 3.0, k / n, rng)
        out[tag + "_llr"] = llr
        sc = Polar5GDecoder(enc, dec_type="SC")
        inner = sc._polar_dec
        seen = []

        class _Capture(tc.nn.Module):  # records the mother-code LLRs (dec.py:621-654 output)
            def forward(self, x):
                seen.append(x.detach().clone().numpy())
                return inner(x)
        sc._polar_dec = _Capture()
        out[tag + "_sc"] = sc(tc.from_numpy(llr)).numpy().astype(np.uint8)
        out[tag + "_llr_mother"] = seen[0].astype(np.float32)
        if n <= 300 and k <= 140:
            scl = Polar5GDecoder(enc, dec_type="SCL", list_size=8)
            out[tag + "_scl"] = scl(tc.from_numpy(llr)).numpy().astype(np.uint8)
        print(f"  uplink k={k} n={n}: n_polar={enc.n_polar} k_polar={enc.k_polar} crc={enc.enc_crc.crc_length}")
    for k, n in DOWNLINK:
        enc = Polar5GEncoder(k, n, channel_type="downlink")
        tag = f"dl_{k}_{n}"
        out[tag + "_frozen"] = np.asarray(enc._frozen_pos).astype(np.int16)
        out[tag + "_idx_rm"] = np.asarray(enc._ind_rate_matching).astype(np.int16)
        out[tag + "_iil"] = np.asarray(enc._ind_input_int).astype(np.int16)
        out[tag + "_meta"] = np.array([enc.k_polar, enc.n_polar, enc.enc_crc.crc_length], dtype=np.int32)
        print(f"  downlink k={k} n={n}: n_polar={enc.n_polar} k_polar={enc.k_polar}")
    # interleavers on their own
    e = Polar5GEncoder(64, 128)
    for m in (20, 64, 100, 160, 1088):
        out[f"chint_{m}"] = e.channel_interleaver(np.arange(m)).astype(np.int16)
    for m in (32, 64, 256, 1024):
        out[f"subint_{m}"] = e.subblock_interleaving(np.arange(m)).astype(np.int16)
    out["input_int_164"] = e.input_interleaver(np.arange(164)).astype(np.int16)
    out["input_int_64"] = e.input_interleaver(np.arange(64)).astype(np.int16)
    np.savez_compressed(os.path.join(OUT, "polar5g.npz"), **out)
    print("wrote", os.path.join(OUT, "polar5g.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
