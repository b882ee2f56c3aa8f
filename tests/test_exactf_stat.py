"""Exact-boxplus parity at statistical power, CPU side: the recipe and the oracle.

tests/golden/exactf_stat.npz (made by tests/golden/make_golden_exactf.py from the reference's my_sn
SC_Dec / SCL_Dec / Polar5GDecoder, my_sn/fec/polar/dec.py:13-157, :158-537, :539-667) holds per
input set the recipe, a hash of the logits and one hash per decoded row.  Here:
  * the recipe regenerates every set's logits bit for bit (llr_sha) -- the precondition of the
    GPU comparison (tests/test_exactf_gpu.py), which regenerates them on the box;
  * the C oracle (glibc exp/log, the checker) reproduces the reference's rows at a mismatch rate
    the one-sided binomial gate accepts (<= 1e-4 for SC), and at exactly
    the mismatch count the fixture recorded when it was made (same oracle, same inputs).
"""
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def fx():
    import sys
    sys.path.insert(0, GOLDEN)
    import exactf_recipe
    return np.load(os.path.join(GOLDEN, "exactf_stat.npz")), exactf_recipe


def _sets(d, kind):
    return sorted(f[:-5] for f in d.files if f.endswith("_meta") and f.startswith(kind + "_"))


def _frozen(k, n):
    fs = np.load(os.path.join(GOLDEN, "frozen_sets.npz"))
    return fs[f"k{k}_n{n}"].astype(np.int64)


def test_row_hash_properties(fx):
    _, R = fx
    rng = np.random.default_rng(0)
    b = rng.integers(0, 2, (500, 523)).astype(np.uint8)
    h = R.row_hash(b)
    assert len(set(h.tolist())) == 500
    c = b.copy()
    c[np.arange(500), rng.integers(0, 523, 500)] ^= 1  # one flipped bit per row
    assert (R.row_hash(c) != h).all()
    assert np.array_equal(R.row_hash(b.astype(np.float32)), h)  # 0/1 floats hash as bytes
    assert np.array_equal(R.row_hash(np.asfortranarray(b)), h)


def test_recipe_encoder_matches_oracle(fx):
    _, R = fx
    fp = _frozen(128, 256)
    u, x, _ = R.awgn_codewords(fp, 256, 64, 2.0, 3)
    assert np.array_equal(x, oracle.polar_encode(u.astype(np.float32), fp, 256).astype(np.uint8))


@pytest.mark.parametrize("k,n", [(128, 256), (512, 1024)])
def test_sc_sets_oracle_rate(fx, k, n):
    d, R = fx
    names = [s for s in _sets(d, "sc") if s.startswith(f"sc_{k}_{n}_")]
    assert len(names) == 3
    mism = rows = 0
    fp = _frozen(k, n)
    for s in names:
        k_, n_, nrows, seed = (int(v) for v in d[s + "_meta"])
        llr = R.awgn_logits(fp, n, nrows, float(d[s + "_ebno"]), seed)
        assert R.llr_sha(llr) == str(d[s + "_llr_sha"]), s
        got = oracle.sc_decode(llr, fp, f_mode=1)
        m = int((R.row_hash(got) != d[s + "_hash"]).sum())
        assert m == int(d[s + "_oracle_mismatch"]), s
        mism += m
        rows += nrows
    assert R.binom_upper_ok(mism, rows, 1e-4), (mism, rows)


def test_scl_sets_oracle_rate(fx):
    d, R = fx
    for s in _sets(d, "scl"):
        k, n, nrows, seed = (int(v) for v in d[s + "_meta"])
        if n > 256:
            continue  # the (512,1024) sets: tests/test_exactf_gpu.py (oracle time)
        fp = _frozen(k, n)
        llr = R.awgn_logits(fp, n, nrows, float(d[s + "_ebno"]), seed)
        assert R.llr_sha(llr) == str(d[s + "_llr_sha"]), s
        got, pm = oracle.scl_decode_mysn(llr, fp, 8, fast_scl=True, exact_f=True)
        ok = R.row_hash(got) == d[s + "_hash"]
        assert int((~ok).sum()) == int(d[s + "_oracle_mismatch"]), s
        assert np.abs(pm.min(axis=1)[ok] - d[s + "_pm"][ok]).max() < 1e-6, s
