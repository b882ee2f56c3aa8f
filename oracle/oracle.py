"""ctypes wrapper around oracle/_build/libpolar_oracle.so (CPU restatement of the reference).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg as the checker.  The product decoders (polar_amd) never import this module.
Pinned against tests/golden/*.npz by tests/test_oracle.py.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libpolar_oracle.so")
_lib = None


def build(force=False):
    """Compile the oracle with gcc (make in oracle/)."""
    src = os.path.join(_HERE, "polar_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE], stdout=subprocess.DEVNULL)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        i32, i64 = ctypes.c_int, ctypes.c_int64
        L.orc_sc_decode.argtypes = [i32, P, i32, P, i64, P, i32]
        L.orc_sc_decode_lmax.argtypes = [i32, P, i32, ctypes.c_float, P, i64, P, i32]
        L.orc_scl_decode.argtypes = [i32, P, i32, P, i64, P, P, i32]
        L.orc_scl_decode_lazy.argtypes = [i32, P, i32, P, i64, P, P, i32]
        L.orc_polar_encode.argtypes = [i32, P, P, i64, P]
        L.orc_scl_decode_mysn.argtypes = [i32, P, i32, P, i64, P, P, i32, i32, i32, ctypes.c_uint32, ctypes.c_double,
                                          i32]
        L.orc_crc_encode.argtypes = [P, i64, i32, i32, ctypes.c_uint32, P]
        L.orc_crc_check.argtypes = [P, i64, i32, i32, ctypes.c_uint32, P]
        L.orc_np_pairwise_sum.argtypes = [P, i32]
        L.orc_np_pairwise_sum.restype = ctypes.c_double
        for f in (L.orc_sc_decode, L.orc_sc_decode_lmax, L.orc_scl_decode, L.orc_scl_decode_lazy, L.orc_polar_encode,
                  L.orc_scl_decode_mysn, L.orc_crc_encode, L.orc_crc_check):
            f.restype = i32
        _lib = L
    return _lib


def frozen_mask(frozen_pos, n):
    m = np.zeros(n, dtype=np.uint8)
    m[np.asarray(frozen_pos, dtype=np.int64)] = 1
    return m


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def sc_decode(llr_logits, frozen_pos, f_mode=0, nthreads=0, llr_max=30.0):
    """SC decode (polar_sc.py SC_Dec semantics).  llr_logits: [bs, n] float32 logits.
    Returns float32 [bs, k] 0/1 bits.  llr_max: the clipping bound (the reference's is 30)."""
    x = np.ascontiguousarray(llr_logits, dtype=np.float32)
    bs, n = x.shape
    fm = frozen_mask(frozen_pos, n)
    k = int(n - fm.sum())
    out = np.empty((bs, k), dtype=np.float32)
    r = lib().orc_sc_decode_lmax(n, _ptr(fm), int(f_mode), ctypes.c_float(llr_max), _ptr(x), bs, _ptr(out),
                                 int(nthreads))
    if r < 0:
        raise ValueError("orc_sc_decode rejected its arguments")
    return out


def scl_decode(llr_logits, frozen_pos, list_size=8, nthreads=0, lazy=False):
    """SCL decode (polar_scl.py SCL_Dec semantics, stable tie order).
    Returns (bits float32 [bs,k], sorted msg_pm float64 [bs, 2L])."""
    x = np.ascontiguousarray(llr_logits, dtype=np.float32)
    bs, n = x.shape
    fm = frozen_mask(frozen_pos, n)
    k = int(n - fm.sum())
    out = np.empty((bs, k), dtype=np.float32)
    pm = np.empty((bs, 2 * list_size), dtype=np.float64)
    fn = lib().orc_scl_decode_lazy if lazy else lib().orc_scl_decode
    r = fn(n, _ptr(fm), int(list_size), _ptr(x), bs, _ptr(out), _ptr(pm), int(nthreads))
    if r < 0:
        raise ValueError("orc_scl_decode rejected its arguments")
    return out, pm


def polar_encode(u_bits, frozen_pos, n):
    """Polar encoding (x_run enc.py semantics).  u_bits: [bs, k] 0/1 -> float32 [bs, n]."""
    u = np.ascontiguousarray(u_bits, dtype=np.float32)
    bs = u.shape[0]
    fm = frozen_mask(frozen_pos, n)
    out = np.empty((bs, n), dtype=np.float32)
    lib().orc_polar_encode(n, _ptr(fm), _ptr(u), bs, _ptr(out))
    return out


# 5G CRC polynomials, 3GPP TS 38.212 Sec. 5.1 as listed in my_sn/fec/crc.py:38-52 (exponents)
CRC_POLYS = {"CRC24A": [24, 23, 18, 17, 14, 11, 10, 7, 6, 5, 4, 3, 1, 0], "CRC24B": [24, 23, 6, 5, 1, 0],
             "CRC24C": [24, 23, 21, 20, 17, 15, 13, 12, 8, 4, 2, 1, 0], "CRC16": [16, 12, 5, 0],
             "CRC11": [11, 10, 9, 5, 0], "CRC6": [6, 5, 0]}


def crc_params(name):
    """(degree, generator mask without the leading term) of a 5G CRC polynomial."""
    ex = CRC_POLYS[name]
    deg = ex[0]
    return deg, sum(1 << e for e in ex if e < deg)


def crc_encode(bits, name):
    """CRCEncoder.forward (crc.py:85-104): [bs, k] 0/1 -> [bs, k + deg] float32."""
    x = np.ascontiguousarray(bits, dtype=np.float32)
    bs, k = x.shape
    deg, g = crc_params(name)
    out = np.empty((bs, k + deg), dtype=np.float32)
    assert lib().orc_crc_encode(_ptr(x), bs, k, deg, g, _ptr(out)) == 0
    return out


def crc_check(bits, name):
    """CRCDecoder validity (crc.py:119-138): [bs, k+deg] -> bool [bs]."""
    x = np.ascontiguousarray(bits, dtype=np.float32)
    bs, n = x.shape
    deg, g = crc_params(name)
    v = np.empty(bs, dtype=np.uint8)
    assert lib().orc_crc_check(_ptr(x), bs, n, deg, g, _ptr(v)) == 0
    return v.astype(bool)


def np_pairwise_sum(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return lib().orc_np_pairwise_sum(_ptr(a), int(a.shape[0]))


def scl_decode_mysn(llr_logits, frozen_pos, list_size=8, fast_scl=True, exact_f=True, crc=None, nthreads=0,
                    llr_max=30.0):
    """my_sn SCL_Dec.forward (dec.py:158-537): exact f, fast-SCL, optional CRC-aided pick.
    llr_max: the decoder's clipping bound (self._llr_max, dec.py:213): f and metric clipping, the
    dead-path metric (:420-422) and the CRC penalty llr_max*k (:517).
    Returns (bits float32 [bs,k], msg_pm float64 [bs,2L]: sorted, then CRC-penalised in place)."""
    x = np.ascontiguousarray(llr_logits, dtype=np.float32)
    bs, n = x.shape
    fm = frozen_mask(frozen_pos, n)
    k = int(n - fm.sum())
    out = np.empty((bs, k), dtype=np.float32)
    pm = np.empty((bs, 2 * list_size), dtype=np.float64)
    deg, g = crc_params(crc) if crc else (0, 0)
    r = lib().orc_scl_decode_mysn(n, _ptr(fm), int(list_size), _ptr(x), bs, _ptr(out), _ptr(pm), int(bool(fast_scl)),
                                  int(bool(exact_f)), deg, g, float(llr_max), int(nthreads))
    if r < 0:
        raise ValueError("orc_scl_decode_mysn rejected its arguments")
    return out, pm
