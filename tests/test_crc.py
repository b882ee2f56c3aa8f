"""my_sn CRC and frozen-set helpers, host side (CPU only): polar_amd.crc.CRCEncoder / CRCDecoder
construction and properties (my_sn/fec/crc.py:6-138), their generator against the reference's
CRC (tests/golden/crc.npz, made by tests/golden/make_golden_mysn.py), int_mod_2
(my_sn/fec/utils.py:2-13) and generate_rm_code (my_sn/fec/polar/utils.py:73-101) against the
reference's output for every 0 <= r <= m <= 10 (tests/golden/rm_codes.npz, made by
tests/golden/make_golden_rm.py).  The kernels are checked in tests/test_crc_gpu.py.
"""
import os

import numpy as np
import pytest
import torch

import polar_amd
from polar_amd import polar5g

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CRCS = ("CRC24A", "CRC24B", "CRC24C", "CRC16", "CRC11", "CRC6")


def test_crc_encoder_properties():
    lengths = {"CRC24A": 24, "CRC24B": 24, "CRC24C": 24, "CRC16": 16, "CRC11": 11, "CRC6": 6}
    for name in CRCS:
        e = polar_amd.CRCEncoder(name, 40)
        assert (e.crc_degree, e.crc_length, e.k, e.n) == (name, lengths[name], 40, 40 + lengths[name])
        pol = e.crc_pol
        assert len(pol) == e.crc_length + 1 and pol[0] == 1 and pol[-1] == 1
        assert e.g_rows.shape == (40,) and e.g_rows.dtype == np.uint32
    # crc.py:_select_crc_pol, CRC11 = x^11 + x^10 + x^9 + x^5 + 1, MSB first
    assert list(polar_amd.CRCEncoder("CRC11", 8).crc_pol) == [1, 1, 1, 0, 0, 0, 1, 0, 0, 0, 0, 1]
    with pytest.raises(AssertionError):
        polar_amd.CRCEncoder(11, 8)
    with pytest.raises(ValueError):
        polar_amd.CRCEncoder("CRC7", 8)
    with pytest.raises(AssertionError):
        polar_amd.CRCDecoder(object())


def test_crc_generator_vs_reference():
    """Parity = XOR of the encoder's generator rows over the 1 bits == the reference's CRCEncoder."""
    d = np.load(os.path.join(GOLDEN, "crc.npz"))
    n = 0
    for key in d.files:
        if not key.endswith("_u"):
            continue
        name, kk = key.split("_")[:2]
        e = polar_amd.CRCEncoder(name, int(kk[1:]))
        u = d[key].astype(bool)
        acc = np.bitwise_xor.reduce(np.where(u, e.g_rows[None, :], 0).astype(np.uint32), axis=1)
        par = ((acc[:, None] >> np.arange(e.crc_length)[None, :]) & 1).astype(np.float32)
        assert np.array_equal(np.concatenate([d[key], par], 1), d[f"{name}_{kk}_enc"]), key
        n += 1
    assert n == 18


def test_rebuild_changes_k():
    e = polar_amd.CRCEncoder("CRC16", 12)
    e.build([3, 7, 30])
    assert (e.k, e.n, e.g_rows.shape) == (30, 46, (30,))


def test_int_mod_2():
    x = torch.tensor([[0.0, 1.0, 2.0, 3.0, 7.0, 10.0]])
    y = polar_amd.int_mod_2(x)
    assert y.dtype == torch.float32 and y.tolist() == [[0, 1, 0, 1, 1, 0]]
    xi = torch.arange(-4, 5, dtype=torch.int64)
    assert polar_amd.int_mod_2(xi).tolist() == [0, 1, 0, 1, 0, 1, 0, 1, 0]  # two's complement AND


def test_generate_rm_code_vs_reference():
    d = np.load(os.path.join(GOLDEN, "rm_codes.npz"))
    for m in range(11):
        for r in range(m + 1):
            frozen, info, n, k, d_min = polar5g.generate_rm_code(r, m)
            t = f"r{r}_m{m}_"
            assert np.array_equal(frozen, d[t + "frozen"]) and np.array_equal(info, d[t + "info"]), t
            assert [n, k, d_min] == list(d[t + "meta"]), t
    with pytest.raises(AssertionError):
        polar5g.generate_rm_code(4, 3)


def test_generate_rm_code_feeds_decoders():
    """An RM frozen set is an ordinary frozen set for the decoders (host-side construction only)."""
    frozen, _, n, k, _ = polar5g.generate_rm_code(2, 6)
    from polar_amd import mysn
    dec = mysn.SCL_Dec(frozen, n, list_size=4)
    assert (dec.n, dec.k) == (n, k) == (64, 22)
