"""Deterministic AWGN inputs and row hashes for the exact-boxplus statistical fixtures
(tests/golden/exactf_stat.npz, made by make_golden_exactf.py; checked by tests/test_exactf_*.py).

TEST INFRASTRUCTURE ONLY.  The fixtures store, per input set, the recipe parameters, a hash of the
logits and one 32-bit hash per decoded row -- not the logits (tens of MB) nor the bits.  Both the
fixture script (in the build container, with the reference) and the tests (anywhere, without it)
regenerate the logits with `awgn_logits`: numpy's PCG64 stream and IEEE double arithmetic, so
the float32 logits are bit-identical on every host with this numpy (the stored `llr_sha` is
checked before any decision is compared).

Model: information bits u ~ Bernoulli(1/2) at the code's information positions, x = u G_n (the
XOR butterfly of my_sn/fec/polar/enc.py:85-96), Gray-QPSK components (1 - 2x)/sqrt(2), AWGN of
variance no/2 per component with no = 1/(10^(EbN0/10) * (k/n) * 2) (my_sn/trans/ebno.py:21-24),
and the demapper's logits log P(b=1)/P(b=0) = -2 sqrt(2) y / no (mapping.py:225-241 for Gray
QPSK) -- the System_AWGN_model chain (awgn_model.py:33-44) restated in numpy.
"""
import hashlib

import numpy as np


def polar_encode(u_full):
    """x = u G_n over GF(2) for uint8 rows of length n (u at every position, frozen ones 0)."""
    x = np.array(u_full, dtype=np.uint8, copy=True)
    n = x.shape[1]
    h = 1
    while h < n:
        x = x.reshape(x.shape[0], n // (2 * h), 2, h)
        x[:, :, 0, :] ^= x[:, :, 1, :]
        x = x.reshape(-1, n)
        h *= 2
    return x


def ebno_to_no(ebno_db, k, n):
    return 1.0 / (10.0 ** (ebno_db / 10.0) * (k / n) * 2.0)


def awgn_codewords(frozen_pos, n, rows, ebno_db, seed):
    """(u [rows, k] uint8, x [rows, n] uint8, logits [rows, n] float32) of one input set."""
    info = np.setdiff1d(np.arange(n), np.asarray(frozen_pos, dtype=np.int64))
    rng = np.random.default_rng(seed)
    u = rng.integers(0, 2, size=(rows, len(info)), dtype=np.uint8)
    full = np.zeros((rows, n), dtype=np.uint8)
    full[:, info] = u
    x = polar_encode(full)
    return u, x, logits_of(x, ebno_to_no(ebno_db, len(info), n), rng)


def logits_of(x, no, rng):
    """AWGN logits of code bits x (uint8 [rows, m]) at noise variance no, drawing from rng."""
    s = (1.0 - 2.0 * x.astype(np.float64)) * np.sqrt(0.5)
    y = s + rng.standard_normal(size=x.shape) * np.sqrt(no / 2.0)
    return (-2.0 * np.sqrt(2.0) * y / no).astype(np.float32)


def awgn_logits(frozen_pos, n, rows, ebno_db, seed):
    return awgn_codewords(frozen_pos, n, rows, ebno_db, seed)[2]


def llr_sha(llr):
    return hashlib.sha256(np.ascontiguousarray(llr, dtype=np.float32).tobytes()).hexdigest()[:16]


_M1 = np.uint64(0x9E3779B97F4A7C15)
_M2 = np.uint64(0xBF58476D1CE4E5B9)


def row_hash(bits):
    """One uint32 per row of a 0/1 array [rows, k]: the packed row bytes folded in 64-bit words
    (multiply-xorshift), so two rows hash equal iff they are equal (up to 2^-32 collisions)."""
    b = np.ascontiguousarray(np.asarray(bits) != 0, dtype=np.uint8)
    rows, k = b.shape
    packed = np.ascontiguousarray(np.packbits(b, axis=1))  # [rows, ceil(k/8)]
    pad = (-packed.shape[1]) % 8
    if pad:
        packed = np.concatenate([packed, np.zeros((rows, pad), dtype=np.uint8)], axis=1)
    words = packed.view(">u8").astype(np.uint64)  # [rows, W], byte order fixed
    h = np.full(rows, np.uint64(k), dtype=np.uint64)
    with np.errstate(over="ignore"):
        for j in range(words.shape[1]):
            h = (h ^ words[:, j]) * _M1
            h ^= h >> np.uint64(31)
            h *= _M2
            h ^= h >> np.uint64(29)
    return (h >> np.uint64(32)).astype(np.uint32)


def binom_upper_ok(mismatches, rows, p0, alpha=1e-3):
    """One-sided binomial gate: True unless `mismatches` of `rows` is significantly above rate
    p0, i.e. P(X >= mismatches | Bin(rows, p0)) >= alpha."""
    from scipy.stats import binom
    if mismatches == 0:
        return True
    return float(binom.sf(mismatches - 1, rows, p0)) >= alpha
