"""my_sn CRC drop-ins on the GPU (polar_amd.crc: pl_crc_attach / pl_crc_check) against the
reference's CRCEncoder / CRCDecoder outputs (tests/golden/crc.npz, made by
tests/golden/make_golden_mysn.py from my_sn/fec/crc.py) and, at larger sizes, against the C
oracle's shift-register CRC (oracle/polar_oracle.c orc_crc_encode / orc_crc_check).  Bit-exact.
"""
import os

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CRCS = ("CRC24A", "CRC24B", "CRC24C", "CRC16", "CRC11", "CRC6")


@pytest.fixture(scope="module")
def d():
    assert torch.cuda.is_available()
    return np.load(os.path.join(GOLDEN, "crc.npz"))


def _keys(d):
    return [(k.split("_")[0], int(k.split("_")[1][1:])) for k in d.files if k.endswith("_u")]


def test_encoder_vs_reference(d):
    from polar_amd import CRCEncoder
    for name, k in _keys(d):
        enc = CRCEncoder(name, k)
        u = torch.from_numpy(d[f"{name}_k{k}_u"])
        want = d[f"{name}_k{k}_enc"]
        got = enc(u.cuda())
        assert got.device.type == "cuda" and got.dtype == torch.float32
        assert np.array_equal(got.cpu().numpy(), want), (name, k)
        assert np.array_equal(enc(u).numpy(), want), (name, k)  # CPU tensors round-trip
        # rank 3 (crc.py: any rank >= 2, CRC over the last dimension)
        got3 = enc(u.reshape(4, 4, k).cuda())
        assert got3.shape == (4, 4, k + enc.crc_length)
        assert np.array_equal(got3.reshape(16, -1).cpu().numpy(), want), (name, k)


def test_decoder_vs_reference(d):
    from polar_amd import CRCDecoder, CRCEncoder
    for name, k in _keys(d):
        word = d[f"{name}_k{k}_word"]
        want = d[f"{name}_k{k}_valid"].astype(bool)
        L = CRCEncoder(name, k).crc_length
        # the fixture's decoder was built on CRCEncoder(name, k + L); the encoder's k does not matter
        for enc_k in (k + L, k):
            x, valid = CRCDecoder(CRCEncoder(name, enc_k))(word)
            assert isinstance(x, np.ndarray) and isinstance(valid, np.ndarray)  # numpy in, numpy out
            assert valid.dtype == bool and valid.shape == (16, 1)
            assert np.array_equal(x, word[:, :-L])
            assert np.array_equal(valid[:, 0], want), (name, k, enc_k)
        enc = CRCEncoder(name, k)
        x_t, v_t = CRCDecoder(enc)(torch.from_numpy(word).cuda())
        assert x_t.device.type == "cuda" and v_t.device.type == "cuda"
        assert np.array_equal(v_t[:, 0].cpu().numpy(), want)
        assert enc.k == k  # not rebuilt by the decoder


def test_round_trip_vs_oracle_large():
    from polar_amd import CRCDecoder, CRCEncoder
    rng = np.random.default_rng(5)
    for name in CRCS:
        for k in (1, 33, 64, 500, 1013):
            u = rng.integers(0, 2, (3000, k)).astype(np.float32)
            enc = CRCEncoder(name, k)
            c = enc(torch.from_numpy(u).cuda())
            want = oracle.crc_encode(u, name)
            assert np.array_equal(c.cpu().numpy(), want), (name, k)
            bad = want.copy()
            flips = rng.integers(0, k + enc.crc_length, 3000)
            rows = np.arange(0, 3000, 3)
            bad[rows, flips[rows]] = 1 - bad[rows, flips[rows]]
            _, valid = CRCDecoder(enc)(torch.from_numpy(bad).cuda())
            exp = oracle.crc_check(bad, name)
            assert np.array_equal(valid[:, 0].cpu().numpy(), exp), (name, k)
            assert not exp[rows].any() and exp[np.setdiff1d(np.arange(3000), rows)].all()  # single flips caught


def test_edge_cases():
    from polar_amd import CRCDecoder, CRCEncoder
    enc = CRCEncoder("CRC11", 20)
    assert enc(torch.empty((0, 20), device="cuda")).shape == (0, 31)
    assert torch.all(enc(torch.zeros((5, 20), device="cuda")) == 0)
    # rebuild on a new last dimension (crc.py:93-95, without its breakpoint)
    out = enc(torch.ones((2, 40), device="cuda"))
    assert (enc.k, enc.n, tuple(out.shape)) == (40, 51, (2, 51))
    assert np.array_equal(out.cpu().numpy(), oracle.crc_encode(np.ones((2, 40), np.float32), "CRC11"))
    dec = CRCDecoder(enc)
    x, v = dec(np.zeros((0, 31), np.float32))
    assert x.shape == (0, 20) and v.shape == (0, 1)
    x, v = dec(np.zeros((2, 11), np.float32))  # word of parity bits only
    assert x.shape == (2, 0) and v.all()
    with pytest.raises(AssertionError):
        dec(np.zeros((2, 10), np.float32))
    with pytest.raises(AssertionError):
        dec(np.zeros(31, np.float32))
    # output dtype
    assert CRCEncoder("CRC6", 12, dtype=torch.float64)(torch.ones((1, 12), device="cuda")).dtype == torch.float64


def test_polar5g_uses_crc_encoder():
    import contextlib
    import io

    from polar_amd import CRCEncoder, polar5g
    with contextlib.redirect_stdout(io.StringIO()):
        enc = polar5g.Polar5GEncoder(64, 128)
    assert isinstance(enc.enc_crc, CRCEncoder) and enc.enc_crc.crc_degree == "CRC11"
    u = torch.randint(0, 2, (100, 64), device="cuda").float()
    assert torch.equal(enc.enc_crc(u), enc.crc_attach(u))
