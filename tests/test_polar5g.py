"""5G NR wrapper, host side, CPU only: the rate-matching tables built by
polar_amd.polar5g against the reference's (tests/golden/make_golden_5g.py ran my_sn/fec/polar
Polar5GEncoder / Polar5GDecoder / generate_5g_ranking), and the data path restated in numpy with
the C oracle's encoder (test infrastructure) against the reference's codewords and mother-code
LLRs, bit for bit.  The GPU kernels are checked against the same fixtures in
tests/test_polar5g_gpu.py.
"""
import contextlib
import io
import os

import numpy as np
import pytest

import oracle
from polar_amd import polar5g

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def g():
    return np.load(os.path.join(GOLDEN, "polar5g.npz"))


def _cases(g, prefix):
    return sorted({tuple(int(v) for v in k.split("_")[1:3]) for k in g.files if k.startswith(prefix + "_")})


def _tables(k, n, ch):
    with contextlib.redirect_stdout(io.StringIO()):
        return polar5g._rate_match_tables(k, n, ch)


def test_ranking(g):
    for key in g.files:
        if not key.startswith("rank_"):
            continue
        _, k, n, kind = key.split("_")
        k, n = int(k), int(n)
        if kind == "unsorted":
            got, _ = polar5g.generate_5g_ranking(0, n, sort=False)
        else:
            got, _ = polar5g.generate_5g_ranking(k, n)
        assert np.array_equal(got, g[key].astype(np.int64)), key
    with pytest.raises(AssertionError):
        polar5g.generate_5g_ranking(4, 16)


def test_interleavers(g):
    for key in g.files:
        if key.startswith("chint_"):
            m = int(key.split("_")[1])
            assert np.array_equal(polar5g.channel_interleaver(np.arange(m)), g[key]), key
        if key.startswith("subint_"):
            m = int(key.split("_")[1])
            assert np.array_equal(polar5g.subblock_interleaving(np.arange(m)), g[key]), key
    assert np.array_equal(polar5g.input_interleaver(np.arange(164)), g["input_int_164"])
    assert np.array_equal(polar5g.input_interleaver(np.arange(64)), g["input_int_64"])


@pytest.mark.parametrize("ch", ["ul", "dl"])
def test_rate_match_tables(g, ch):
    cases = _cases(g, ch)
    assert len(cases) >= (20 if ch == "ul" else 5)
    for k, n in cases:
        tag = f"{ch}_{k}_{n}"
        crc, n_polar, frozen, idx_rm, iil = _tables(k, n, "uplink" if ch == "ul" else "downlink")
        k_polar = n_polar - len(frozen)
        assert [k_polar, n_polar, polar5g.mysn.crc_params(crc)[0]] == list(g[tag + "_meta"]), tag
        assert np.array_equal(frozen, g[tag + "_frozen"].astype(np.int64)), tag
        assert np.array_equal(idx_rm, g[tag + "_idx_rm"].astype(np.int64)), tag
        if ch == "dl":
            assert np.array_equal(iil, g[tag + "_iil"].astype(np.int64)), tag


def test_rate_match_asserts():
    with pytest.raises(ValueError):
        _tables(8, 100, "uplink")  # k < 12 uplink (enc.py:281-283)
    with pytest.raises(AssertionError):
        _tables(200, 300, "downlink")  # k > 140 downlink
    with pytest.raises(AssertionError):
        _tables(20, 2000, "uplink")  # n > 1088


def test_crc_generator_rows_vs_reference_crc():
    """parity = XOR of generator rows of the 1 bits == CRCEncoder output (tests/golden/crc.npz)."""
    d = np.load(os.path.join(GOLDEN, "crc.npz"))
    for key in d.files:
        if not key.endswith("_u"):
            continue
        name, kk = key.split("_")[:2]
        k = int(kk[1:])
        rows = polar5g.crc_generator_rows(name, k)
        u = d[key].astype(np.uint8)
        deg = polar5g.mysn.crc_params(name)[0]
        acc = np.bitwise_xor.reduce(np.where(u.astype(bool), rows[None, :], 0).astype(np.uint32), axis=1)
        par = ((acc[:, None] >> np.arange(deg)[None, :]) & 1).astype(np.float32)
        assert np.array_equal(np.concatenate([d[key], par], 1), d[name + f"_k{k}_enc"]), key


def _encode_np(k, n, u):
    crc, n_polar, frozen, idx_rm, _ = _tables(k, n, "uplink")
    rows = polar5g.crc_generator_rows(crc, k)
    deg = polar5g.mysn.crc_params(crc)[0]
    acc = np.bitwise_xor.reduce(np.where(u.astype(bool), rows[None, :], 0).astype(np.uint32), axis=1)
    uc = np.concatenate([u, ((acc[:, None] >> np.arange(deg)[None, :]) & 1).astype(np.float32)], 1)
    c = oracle.polar_encode(uc, frozen, n_polar)
    return c[:, idx_rm]


def test_encoder_data_path_restated(g):
    for k, n in _cases(g, "ul"):
        tag = f"ul_{k}_{n}"
        assert np.array_equal(_encode_np(k, n, g[tag + "_u"]), g[tag + "_c"]), tag


def test_rate_recovery_table_restated(g):
    """The folded recovery table applied in numpy reproduces the reference's mother-code LLRs
    (dec.py:621-654) bit for bit: puncturing, shortening (-100) and repetition sums included."""
    for k, n in _cases(g, "ul"):
        tag = f"ul_{k}_{n}"
        with contextlib.redirect_stdout(io.StringIO()):
            enc = polar5g.Polar5GEncoder(k, n)
            dec = polar5g.Polar5GDecoder(enc, dec_type="SC")
        a, b, f = dec._rec
        x = g[tag + "_llr"]
        got = np.where(a[None, :] >= 0, x[:, np.maximum(a, 0)], f[None, :])
        rep = b >= 0
        got[:, rep] = x[:, a[rep]] + x[:, b[rep]]
        assert np.array_equal(got.astype(np.float32), g[tag + "_llr_mother"]), tag


def test_module_api_errors():
    with contextlib.redirect_stdout(io.StringIO()):
        enc = polar5g.Polar5GEncoder(64, 128)
        with pytest.raises(ValueError):
            polar5g.Polar5GDecoder(enc, dec_type="BP")
        with pytest.raises(NotImplementedError):
            polar5g.Polar5GDecoder(enc, dec_type="hybSCL")
        with pytest.raises(AssertionError):
            polar5g.Polar5GDecoder(enc, return_crc_status=1)
    assert (enc.k, enc.n, enc.k_polar, enc.n_polar, enc.enc_crc.crc_degree) == (64, 128, 75, 128, "CRC11")
    with pytest.raises(AssertionError):
        polar5g.Polar5GEncoder(64, 128, channel_type="sidelink")
