"""5G NR polar coding wrapper: drop-ins for my_sn/fec/polar

  generate_5g_ranking  <-> my_sn/fec/polar/utils.py:6-71   (3GPP TS 38.212 Table 5.3.1.2-1)
  generate_rm_code     <-> my_sn/fec/polar/utils.py:73-101  (Reed-Muller frozen set)
  PolarEncoder         <-> my_sn/fec/polar/enc.py:7-114     (mother-code encoder)
  Polar5GEncoder       <-> my_sn/fec/polar/enc.py:115-392   (CRC, rate matching, interleavers)
  Polar5GDecoder       <-> my_sn/fec/polar/dec.py:539-666   (rate recovery, SC / CRC-aided SCL)

The index tables (sub-block / channel / input interleavers, puncturing, shortening, repetition,
frozen set) are computed once on the host at construction, following 38.212 Sec. 5.3.1 and 5.4.1
exactly as the reference does (including its choices: no PC bits for 12 <= k <= 19, no
downlink input interleaving in forward).  The per-codeword data path runs on the GPU:
CRC attachment (pl_crc_attach), polar encoding (pl_polar_encode), rate matching
(pl_gather_rows), rate recovery (pl_rate_recover) and the my_sn SC / SCL decoders
(polar_amd.mysn).  There is no CPU path.

Differences from the reference, where it cannot run as shipped:
  * CRCEncoder cannot be constructed (crc.py:81 reads self.device, never set), so neither can
    Polar5GEncoder; here both work (the CRC is pinned by tests/golden/crc.npz).
  * return_crc_status=True reaches breakpoint() / CRCDecoder(tc.from_numpy(tensor)) in the
    reference (dec.py:655-666, crc.py:119-121); here it returns the CRC status (True = all
    parity bits match), the semantics its docstring states.  Parity unpinned for that output.
  * dec_type "hybSCL" cannot be constructed in the reference (SCL_Dec has no ind_iil_inv
    argument, dec.py:587-590); here it raises NotImplementedError.
"""
import ctypes
import math
import os

import numpy as np
import torch as tc
from torch import nn

from . import _lib, mysn, ops
from .crc import CRCEncoder
from .decoders import _gpu_for

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "polar5g_ranking.npy")
_RANKING = None

# 38.212 Table 5.4.1.1-1: sub-block interleaver pattern P(i)
SUBBLOCK_PERM = np.array([0, 1, 2, 4, 3, 5, 6, 7, 8, 16, 9, 17, 10, 18, 11, 19, 12, 20, 13, 21, 14, 22, 15, 23,
                          24, 25, 26, 28, 27, 29, 30, 31])
# 38.212 Table 5.3.1.1-1: input bit interleaver pattern (K_IL,max = 164)
INPUT_IL_MAX = np.array([
    0, 2, 4, 7, 9, 14, 19, 20, 24, 25, 26, 28, 31, 34, 42, 45, 49, 50, 51, 53, 54, 56, 58, 59, 61, 62, 65, 66, 67,
    69, 70, 71, 72, 76, 77, 81, 82, 83, 87, 88, 89, 91, 93, 95, 98, 101, 104, 106, 108, 110, 111, 113, 115, 118,
    119, 120, 122, 123, 126, 127, 129, 132, 134, 138, 139, 140, 1, 3, 5, 8, 10, 15, 21, 27, 29, 32, 35, 43, 46, 52,
    55, 57, 60, 63, 68, 73, 78, 84, 90, 92, 94, 96, 99, 102, 105, 107, 109, 112, 114, 116, 121, 124, 128, 130, 133,
    135, 141, 6, 11, 16, 22, 30, 33, 36, 44, 47, 64, 74, 79, 85, 97, 100, 103, 117, 125, 131, 136, 142, 12, 17, 23,
    37, 48, 75, 80, 86, 137, 143, 13, 18, 38, 144, 39, 145, 40, 146, 41, 147, 148, 149, 150, 151, 152, 153, 154,
    155, 156, 157, 158, 159, 160, 161, 162, 163])


def _ranking_table():
    """[1024, 2] (reliability rank, sub-channel index) of 38.212 Table 5.3.1.2-1."""
    global _RANKING
    if _RANKING is None:
        _RANKING = np.load(_DATA, allow_pickle=False).astype(np.int64)
    return _RANKING


def generate_5g_ranking(k, n, sort=True, strict=True):
    """[frozen_pos, info_pos] of the 5G polar code (utils.py:6-71): the n-k least reliable
    sub-channels < n are frozen.  Unsorted output lists positions from least to most reliable."""
    if strict:
        assert k < 1025, "k cant > 1024."
        assert n < 1025, "n cant > 1024."
        assert n > 31, "n cant < 32."
        assert n >= k, "Invalid coderate (>1)."
        assert np.log2(n) == int(np.log2(n)), "n must be a power of 2."
    t = _ranking_table()
    order = t[np.argsort(t[:, 0]), 1]  # sub-channels, least reliable first
    order = order[order < n]
    frozen_pos = order[: n - k].copy()
    info_pos = order[n - k:].copy()
    if sort:
        info_pos = np.sort(info_pos)
        frozen_pos = np.sort(frozen_pos)
    return [frozen_pos.astype(int), info_pos.astype(int)]


def generate_rm_code(r, m):
    """[frozen_pos, info_pos, n, k, d_min] of the (r, m) Reed-Muller code as a polar code
    (utils.py:73-101): the rows of F2^{(x)m} whose index has binary weight < m - r are frozen."""
    assert r <= m, "order r cannot be larger than m."
    n = 2 ** m
    d_min = 2 ** (m - r)
    k = sum(math.comb(m, i) for i in range(r + 1))
    w = np.array([bin(i).count("1") for i in range(n)])
    frozen_vec = w < m - r
    frozen_pos = np.arange(n)[frozen_vec]
    info_pos = np.arange(n)[~frozen_vec]
    assert len(info_pos) == k, "Error: resulting k is inconsistent."
    return frozen_pos, info_pos, n, k, d_min


def subblock_interleaving(u):
    """Sub-block interleaver of 38.212 Sec. 5.4.1.1 (enc.py:196-216): y[n] = u[J(n)]."""
    u = np.asarray(u)
    k = u.shape[-1]
    assert np.mod(k, 32) == 0, "len for sub-block interleaving must be a multiple of 32."
    m = np.arange(k)
    j = SUBBLOCK_PERM[(32 * m) // k] * (k // 32) + np.mod(m, k // 32)
    return u[j]


def channel_interleaver(c):
    """Triangular channel interleaver of 38.212 Sec. 5.4.1.3 (enc.py:217-242): write c row-wise
    into rows of length T, T-1, ..., read column-wise skipping the unfilled cells."""
    c = np.asarray(c)
    e = c.shape[-1]
    t = 0
    while t * (t + 1) / 2 < e:
        t += 1
    row_start = np.concatenate([[0], np.cumsum(np.arange(t, 0, -1))])  # first index of row i
    order = []
    for j in range(t):
        for i in range(t - j):
            idx = row_start[i] + j
            if idx < e:
                order.append(idx)
    return c[np.asarray(order, dtype=np.int64)]


def input_interleaver(c):
    """Input bit interleaver of 38.212 Sec. 5.3.1.1 (enc.py:243-263), K <= 164."""
    c = np.asarray(c)
    k = len(c)
    assert k <= 164, "Input interleaver only defined for length of 164."
    sel = INPUT_IL_MAX[INPUT_IL_MAX >= 164 - k] - (164 - k)
    return c[sel].astype(int)


def crc_generator_rows(crc_degree, k):
    """The k x L CRC generator of crc.py:54-73 (row m = parity of the unit vector e_m), one
    uint32 per row with bit c = parity column c."""
    deg, mask = mysn.crc_params(crc_degree)
    # MSB-first coefficient vector [x^deg ... x^0] of crc.py:_select_crc_pol
    pol = np.array([1] + [(mask >> (deg - 1 - i)) & 1 for i in range(deg)], dtype=np.int64)
    rows = np.zeros(k, dtype=np.uint32)
    x = np.zeros(deg, dtype=np.int64)
    x[0] = 1
    for i in range(k):
        x = np.concatenate([x, [0]])
        if x[0] == 1:
            x = np.bitwise_xor(x, pol)
        x = x[1:]
        rows[k - i - 1] = np.uint32(sum(int(b) << c for c, b in enumerate(x)))
    return rows


def _rate_match_tables(k_target, n_target, channel_type):
    """Polar5GEncoder._init_rate_match (enc.py:264-358): CRC, mother code, frozen set and the
    rate-matching gather indices."""
    assert n_target >= k_target, "n must be larger or equal k."
    assert n_target >= 18, "n<18 is not supported by the 5G Polar coding scheme."
    assert k_target <= 1013, "k too large - no codeword segmentation supported at the moment."
    assert n_target <= 1088, "n too large - no codeword segmentation supported at the moment."
    if channel_type == "uplink":
        if 12 <= k_target <= 19:
            crc_pol, k_crc = "CRC6", 6
        elif k_target >= 20:
            crc_pol, k_crc = "CRC11", 11
        else:
            raise ValueError("k_target<12 is not supported in 5G NR for uplink; please use 'channel coding of "
                             "small block len' scheme from Sec. 5.3.3 in 3GPP 38.212 instead.")
        if k_target <= 19:
            print("Warning: For 12<=k<=19 additional 3 parity-check bits are defined in 38.212. "
                  "we didn't implement that")
    else:
        assert k_target <= 140, "k too large for downlink channel config."
        assert n_target >= 25, "n too small for downlink channel config with 24 bit CRC."
        assert n_target <= 576, "n too large for downlink channel configuration."
        crc_pol, k_crc = "CRC24C", 24
    k_polar = k_target + k_crc
    assert k_polar <= n_target, "Device is not expected to be configured with k_polar + k_crc + n_pc > n_target."
    n_min, n_max = 5, 10
    if n_target <= (9 / 8) * 2 ** (np.ceil(np.log2(n_target)) - 1) and k_polar / n_target < 9 / 16:
        n1 = np.ceil(np.log2(n_target)) - 1
    else:
        n1 = np.ceil(np.log2(n_target))
    n2 = np.ceil(np.log2(8 * k_polar))
    n_polar = int(2 ** np.max((np.min([n1, n2, n_max]), n_min)))
    punct = k_polar / n_target <= 7 / 16
    prefrozen = []
    if n_target < n_polar:
        if punct:
            n_int = int(32 * np.ceil((n_polar - n_target) / 32))
            pat = subblock_interleaving(np.arange(n_int))
            prefrozen += [int(v) for v in pat[: n_polar - n_target]]
            if n_target >= 3 * n_polar / 4:
                t = int(np.ceil(3 / 4 * n_polar - n_target / 2) - 1)
            else:
                t = int(np.ceil(9 / 16 * n_polar - n_target / 4) - 1)
            prefrozen += list(range(t))
        else:
            n_int = int(32 * np.ceil(n_polar / 32))
            pat = subblock_interleaving(np.arange(n_int))
            prefrozen += [int(v) for v in pat[n_target:n_polar]]
    prefrozen = np.unique(np.asarray(prefrozen, dtype=np.int64))
    ranking, _ = generate_5g_ranking(0, n_polar, sort=False)
    cand = ranking[~np.isin(ranking, prefrozen)]  # reliability order kept (setdiff1d, assume_unique)
    info_pos = np.sort(cand[::-1][:k_polar]).astype(int)
    frozen_pos = np.setdiff1d(np.arange(n_polar), info_pos, assume_unique=True)
    ind_input_int = input_interleaver(np.arange(k_polar)) if channel_type == "downlink" else None
    ind_sub_int = subblock_interleaving(np.arange(n_polar))
    if n_target >= n_polar:
        idx_c = np.mod(np.arange(n_target), n_polar)  # repetition
    elif punct:
        idx_c = np.arange(n_target) + n_polar - n_target
    else:
        idx_c = np.arange(n_target)  # shortening
    if channel_type == "uplink":
        idx_rm = ind_sub_int[idx_c[channel_interleaver(np.arange(n_target))]]
    else:
        idx_rm = ind_sub_int[idx_c]
    return crc_pol, n_polar, frozen_pos, idx_rm.astype(int), ind_input_int


def _to_dev_i32(a, dev):
    return tc.as_tensor(np.ascontiguousarray(a, dtype=np.int32), device=dev)


class PolarEncoder(nn.Module):
    """my_sn polar encoder (enc.py:7-114): u [bs, k] -> x = u G_n [bs, n] (HIP butterfly)."""

    def __init__(self, frozen_pos, n, dtype=tc.float32, device='cpu'):
        super().__init__()
        self.device = device
        self.dtype = dtype
        assert np.log2(n) == int(np.log2(n)), "n must be a power of 2."
        frozen_pos = np.asarray(frozen_pos)
        self._k = n - len(frozen_pos)
        self._n = n
        self._frozen_pos = frozen_pos
        assert self._k <= self._n, "Invalid coderate (>1)."
        self.info_pos = np.setdiff1d(np.arange(self._n), frozen_pos)
        assert self._k == len(self.info_pos), "Internal error: invalid info_pos generated."
        self._mask = np.zeros(n, dtype=np.uint8)
        self._mask[frozen_pos.astype(np.int64)] = 1
        self._plans = _lib.PlanSet()

    @property
    def k(self):
        return self._k

    @property
    def n(self):
        return self._n

    @property
    def frozen_pos(self):
        return self._frozen_pos

    def plan(self, device=None):
        """The encoding plan on `device` (default: the current GPU); plans are device-bound."""
        return self._plans.get(device, self._make_plan)

    def _make_plan(self, dev):
        return _lib.Plan(self._n, self._mask, 1, _lib.PL_F_MINSUM, flags=_lib.PL_PLAN_GENERIC, device=dev)

    def _encode_dev(self, u):
        return ops.polar_encode(self.plan(u.device), u)

    def forward(self, u):
        assert u.shape[-1] == self._k, "Last dim must be len k."
        dev = _gpu_for(u, self.device)
        x = self._encode_dev(u.reshape(-1, self._k).to(dev, tc.float32))
        return x.reshape(*u.shape[:-1], self._n).to(device=u.device, dtype=self.dtype)


class Polar5GEncoder(PolarEncoder):
    """5G NR polar encoder with CRC and rate matching (enc.py:115-392)."""

    def __init__(self, k, n, channel_type="uplink", verbose=False, dtype=tc.float32, device='cpu'):
        k, n = int(k), int(n)
        assert n >= k, "Invalid coderate (>1)."
        assert channel_type in ("uplink", "downlink"), "Unsupported channel_type."
        self._channel_type = channel_type
        self._k_target, self._n_target = k, n
        self._verbose = verbose
        crc_pol, n_polar, frozen_pos, idx_rm, idx_input = _rate_match_tables(k, n, channel_type)
        super().__init__(frozen_pos, n_polar, dtype=dtype, device=device)
        self._frozen_pos = frozen_pos
        self._ind_rate_matching = idx_rm
        self._ind_input_int = idx_input
        self._crc_degree = crc_pol
        self._crc_length = mysn.crc_params(crc_pol)[0]
        self._enc_crc = CRCEncoder(crc_pol, k, dtype=dtype, device=device)  # enc.py:156
        self._g_rows = self._enc_crc.g_rows
        self._dev_tables = {}
        if verbose:
            print(f"Code params after rate-matching: k = {k}, n = {n}")
            print(f"Polar mother code: k_polar = {self.k_polar}, n_polar = {n_polar}")
            print("Using", crc_pol)
            print("Frozen positions: ", frozen_pos)
            print("Channel type: " + channel_type)

    @property
    def enc_crc(self):
        """The CRC encoder (polar_amd.crc.CRCEncoder, enc.py:156-158)."""
        return self._enc_crc

    @property
    def crc_degree(self):
        return self._crc_degree

    @property
    def crc_length(self):
        return self._crc_length

    @property
    def k_target(self):
        return self._k_target

    @property
    def n_target(self):
        return self._n_target

    @property
    def k_polar(self):
        return self._k

    @property
    def n_polar(self):
        return self._n

    @property
    def k(self):
        return self._k_target

    @property
    def n(self):
        return self._n_target

    # the interleavers as methods, like the reference (enc.py:196-263)
    subblock_interleaving = staticmethod(subblock_interleaving)
    channel_interleaver = staticmethod(channel_interleaver)
    input_interleaver = staticmethod(input_interleaver)

    def tables(self, dev):
        """Device copies of the CRC generator rows and the rate-matching gather index."""
        key = str(dev)
        if key not in self._dev_tables:
            self._dev_tables[key] = (tc.as_tensor(self._g_rows.view(np.int32), device=dev),
                                     _to_dev_i32(self._ind_rate_matching, dev))
        return self._dev_tables[key]

    def crc_attach(self, u):
        """[bs, k_target] -> [bs, k_target + crc_length] on the GPU (crc.py:85-104)."""
        ops._require_cuda(u, "u")
        u = u.to(tc.float32).contiguous()
        g, _ = self.tables(u.device)
        out = tc.empty((u.shape[0], self._k_target + self._crc_length), dtype=tc.float32, device=u.device)
        with tc.cuda.device(u.device):
            _lib.check(_lib.lib().pl_crc_attach(ctypes.c_void_p(u.data_ptr()), u.shape[0], self._k_target,
                                                ctypes.c_void_p(g.data_ptr()), self._crc_length,
                                                ctypes.c_void_p(out.data_ptr()), _lib.current_stream_ptr(u.device)),
                       "pl_crc_attach")
        return out

    def forward(self, u):
        bs = u.shape[0]
        assert u.shape[-1] == self.k, "Last dim must be len k."
        if self._channel_type == "downlink":
            raise Exception('error...')  # enc.py:375-377: downlink forward is not implemented upstream
        dev = _gpu_for(u, self.device)
        u2 = u.reshape(-1, self._k_target).to(dev, tc.float32)
        c = self._encode_dev(self.crc_attach(u2))
        _, idx = self.tables(dev)
        out = tc.empty((c.shape[0], self._n_target), dtype=tc.float32, device=dev)
        with tc.cuda.device(dev):
            _lib.check(_lib.lib().pl_gather_rows(ctypes.c_void_p(c.data_ptr()), c.shape[0], self._n,
                                                 ctypes.c_void_p(idx.data_ptr()), self._n_target,
                                                 ctypes.c_void_p(out.data_ptr()), _lib.current_stream_ptr(dev)),
                       "pl_gather_rows")
        out_shape = list(u.shape[:-1]) + [self._n_target]
        out_shape[0] = -1
        del bs
        return out.reshape(out_shape).to(device=u.device, dtype=self.dtype)


class Polar5GDecoder(nn.Module):
    """5G NR polar decoder: rate recovery + SC / CRC-aided SCL + CRC removal (dec.py:539-666)."""

    def __init__(self, enc_polar, dec_type="SC", list_size=8, return_crc_status=False, output_dtype=tc.float32):
        super().__init__()
        assert isinstance(enc_polar, Polar5GEncoder), "enc_polar must be a Polar5GEncoder."
        self._output_dtype = output_dtype
        self._n_target, self._k_target = enc_polar.n_target, enc_polar.k_target
        self._n_polar, self._k_polar = enc_polar.n_polar, enc_polar.k_polar
        self._k_crc = enc_polar.enc_crc.crc_length
        self._bil = enc_polar._channel_type == "uplink"
        self._iil = False
        self._llr_max = 100  # dec.py:568: internal max LLR (shortened positions)
        self._enc_polar = enc_polar
        self._dec_type = dec_type
        self._init_interleavers()
        if dec_type == "SC":
            print("Warning: CRC cant be used with SC dec and. Please use SCL dec.")
            self._polar_dec = mysn.SC_Dec(enc_polar._frozen_pos, self._n_polar)
        elif dec_type == "SCL":
            self._polar_dec = mysn.SCL_Dec(enc_polar._frozen_pos, self._n_polar,
                                           crc_degree=enc_polar.enc_crc.crc_degree, list_size=list_size)
        elif dec_type == "hybSCL":
            raise NotImplementedError("hybSCL: the reference cannot construct it (dec.py:587-590)")
        else:
            raise ValueError("Unknown value for dec_type.")
        assert isinstance(return_crc_status, bool), "return_crc_status must be bool."
        self._return_crc_status = return_crc_status
        self._build_recovery()
        self._dev_tables = {}

    def _init_interleavers(self):
        """Inverse interleaver patterns for rate recovery (dec.py:597-611)."""
        self.ind_ch_int_inv = np.argsort(channel_interleaver(np.arange(self._n_target)))
        self.ind_sub_int_inv = np.argsort(subblock_interleaving(np.arange(self._n_polar)))
        self.ind_iil_inv = None

    def _build_recovery(self):
        """Fold de-interleaving, de-puncturing / de-shortening / repetition combining and the
        sub-block de-interleaver (dec.py:621-654) into one table over the N mother positions:
        out[j] = fill[j] if a[j] < 0 else llr[a[j]] (+ llr[b[j]] if b[j] >= 0)."""
        N, E = self._n_polar, self._n_target
        chmap = self.ind_ch_int_inv if self._bil else np.arange(E)
        a = np.full(N, -1, dtype=np.int64)
        b = np.full(N, -1, dtype=np.int64)
        fill = np.zeros(N, dtype=np.float32)
        dem_a = np.full(N, -1, dtype=np.int64)
        dem_b = np.full(N, -1, dtype=np.int64)
        dem_f = np.zeros(N, dtype=np.float32)
        if E >= N:  # repetition: llr_1 + llr_3 on the first n_rep positions
            # (for E > 2N the reference's concat has n_rep > N columns and the sub-block gather
            # keeps the first N: a third copy is dropped, dec.py:627-633; reproduced here)
            n_rep = min(E - N, N)
            dem_a[:] = chmap[np.arange(N)]
            dem_b[:n_rep] = chmap[N + np.arange(n_rep)]
        elif self._k_polar / E <= 7 / 16:  # puncturing: N - E zero LLRs first
            dem_a[N - E:] = chmap[np.arange(E)]
        else:  # shortening: N - E LLRs of -llr_max (logits) last
            dem_a[:E] = chmap[np.arange(E)]
            dem_f[E:] = -self._llr_max
        j = self.ind_sub_int_inv
        a[:], b[:], fill[:] = dem_a[j], dem_b[j], dem_f[j]
        self._rec = (a, b, fill)

    def tables(self, dev):
        key = str(dev)
        if key not in self._dev_tables:
            a, b, f = self._rec
            self._dev_tables[key] = (_to_dev_i32(a, dev), _to_dev_i32(b, dev), tc.as_tensor(f, device=dev))
        return self._dev_tables[key]

    def rate_recover(self, llr_ch):
        """[bs, n_target] logits on the GPU -> [bs, n_polar] mother-code logits."""
        ops._require_cuda(llr_ch, "llr_ch")
        x = llr_ch.to(tc.float32).contiguous()
        a, b, f = self.tables(x.device)
        out = tc.empty((x.shape[0], self._n_polar), dtype=tc.float32, device=x.device)
        with tc.cuda.device(x.device):
            _lib.check(_lib.lib().pl_rate_recover(ctypes.c_void_p(x.data_ptr()), x.shape[0], self._n_target,
                                                  ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                                                  ctypes.c_void_p(f.data_ptr()), self._n_polar,
                                                  ctypes.c_void_p(out.data_ptr()), _lib.current_stream_ptr(x.device)),
                       "pl_rate_recover")
        return out

    @property
    def k_target(self):
        return self._k_target

    @property
    def n_target(self):
        return self._n_target

    @property
    def k_polar(self):
        return self._k_polar

    @property
    def n_polar(self):
        return self._n_polar

    @property
    def llr_max(self):
        return self._llr_max

    @property
    def dec_type(self):
        return self._dec_type

    @property
    def polar_dec(self):
        return self._polar_dec

    def forward(self, inputs):
        inputs = inputs.to(tc.float32)
        input_shape = inputs.shape
        assert len(input_shape) > 1
        llr_ch = inputs.reshape([-1, self._n_target])
        dev = _gpu_for(llr_ch, getattr(self._enc_polar, "device", None))
        llr_dec = self.rate_recover(llr_ch.to(dev))
        # the mother decoder returns on its own device (SCL_Dec: self.device, polar_scl.py:234)
        u_hat_crc = self._polar_dec(llr_dec).to(dev)
        u_hat = u_hat_crc[:, : self._k_target]
        output_shape = [*input_shape]
        output_shape[-1] = self._k_target
        output_shape[0] = -1
        u_hat = u_hat.reshape(output_shape).to(device=inputs.device, dtype=self._output_dtype)
        if not self._return_crc_status:
            return u_hat
        recoded = self._enc_polar.crc_attach(u_hat_crc[:, : self._k_target].contiguous())
        ok = (recoded[:, self._k_target:] == u_hat_crc[:, self._k_target:]).all(dim=-1)
        crc_shape = output_shape[:-1]
        return u_hat, ok.reshape(crc_shape).to(device=inputs.device, dtype=self._output_dtype)
