"""5G CRC drop-ins for my_sn/fec/crc.py and my_sn/fec/utils.py (SURVEY §2 row "my_sn/fec/crc.py").

  CRCEncoder  <-> my_sn/fec/crc.py:6-109    (G-matrix CRC of the 5G polynomials :38-52)
  CRCDecoder  <-> my_sn/fec/crc.py:111-138  (re-encode, valid iff every parity bit is 0)
  int_mod_2   <-> my_sn/fec/utils.py:2-13

The generator (crc.py:54-73: the CRC of every unit vector, built in O(k) by successive polynomial
division) is computed once per length on the host (polar5g.crc_generator_rows, one uint32 per row,
bit c = parity column c) and the per-word work runs on the GPU: pl_crc_attach (one wave per word,
XOR of the rows of the 1 bits, butterfly reduction over the wave) for the encoder, pl_crc_check
(same XOR over the whole received word, one byte per word) for the decoder.  There is no CPU path;
CPU tensors and NumPy arrays are moved to the GPU and the results back to where the inputs were.

Differences from the reference, where it cannot run as shipped:
  * CRCEncoder.build reads self.device, which is never set (crc.py:81), so the reference cannot be
    constructed; here it can, with the CRC of crc.py (pinned by tests/golden/crc.npz, generated
    with that one attribute set at run time).
  * A change of the last input dimension rebuilds the generator as crc.py:93-95 intends, without
    the breakpoint() at :94.
  * CRCDecoder re-encodes the received word with a generator of the word's own length held by
    the decoder; the reference does the same through its encoder (crc.py:132), which rebuilds the
    encoder in place and so changes encoder.k / encoder.n as a side effect.  Here the encoder is
    left as it was.  NumPy in -> NumPy out as in the reference (crc.py:125, :138); torch tensors
    are accepted too and give tensors on the input's device.
  * Inputs are hard bits in {0, 1}; a word bit counts as 1 when it is non-zero (the reference's
    x @ G followed by int_mod_2 agrees on {0, 1} inputs).
"""
import ctypes

import numpy as np
import torch as tc
from torch import nn

from . import _lib, mysn
from .decoders import _gpu_for


def int_mod_2(x):
    """x mod 2 of integer-valued inputs, result in x's dtype (my_sn/fec/utils.py:2-13: cast to int32,
    AND with 1, cast back)."""
    return tc.bitwise_and(x.to(tc.int32), 1).to(x.dtype)


def _crc_pol_msb_first(crc_degree):
    """crc.py:_select_crc_pol :38-53: coefficients [x^L ... x^0] as an int array, and L."""
    deg, mask = mysn.crc_params(crc_degree)
    return np.array([1] + [(mask >> (deg - 1 - i)) & 1 for i in range(deg)], dtype=int), deg


class _Rows:
    """Device copies of the generator rows for one word length."""

    def __init__(self, crc_degree, length):
        from .polar5g import crc_generator_rows
        self.length = length
        self.host = crc_generator_rows(crc_degree, length)
        self._dev = {}

    def on(self, dev):
        key = str(dev)
        if key not in self._dev:
            self._dev[key] = tc.as_tensor(self.host.view(np.int32), device=dev)
        return self._dev[key]


def _as_tensor(inputs):
    if isinstance(inputs, np.ndarray):
        return tc.from_numpy(np.ascontiguousarray(inputs)), True
    return inputs, False


class CRCEncoder(nn.Module):
    """Adds the CRC parity bits of a 5G polynomial to the last dimension (crc.py:6-109).

    crc_degree: one of CRC24A, CRC24B, CRC24C, CRC16, CRC11, CRC6; k: information bits per word;
    dtype: output dtype; device: GPU used when the inputs are on the CPU (default: the current one).
    forward(inputs [..., k]) -> [..., k + crc_length].
    """

    def __init__(self, crc_degree, k, dtype=tc.float32, device='cpu'):
        super().__init__()
        assert isinstance(crc_degree, str), "crc_degree must be str"
        self.dtype = dtype
        self.device = device
        self._crc_degree = crc_degree
        self._crc_pol, self._crc_length = _crc_pol_msb_first(crc_degree)
        self._k = k
        self._n = None
        self.build([None, k])

    @property
    def crc_degree(self):
        return self._crc_degree

    @property
    def crc_length(self):
        return self._crc_length

    @property
    def crc_pol(self):
        return self._crc_pol

    @property
    def k(self):
        return self._k

    @property
    def n(self):
        return self._n

    @property
    def g_rows(self):
        """The k x crc_length generator of crc.py:54-73, one uint32 per row (bit c = column c)."""
        return self._rows.host

    def build(self, input_shape):
        """Generator for the last dimension of input_shape (crc.py:76-83)."""
        k = input_shape[-1]
        assert k is not None, "Shape of last dimension cannot be None."
        self._rows = _Rows(self._crc_degree, int(k))
        self._k = int(k)
        self._n = self._k + self._crc_length

    def _attach(self, x):
        """[rows, k] fp32 on the GPU -> [rows, k + L] fp32 (pl_crc_attach)."""
        out = tc.empty((x.shape[0], self._n), dtype=tc.float32, device=x.device)
        with tc.cuda.device(x.device):
            _lib.check(_lib.lib().pl_crc_attach(ctypes.c_void_p(x.data_ptr()), x.shape[0], self._k,
                                                ctypes.c_void_p(self._rows.on(x.device).data_ptr()),
                                                self._crc_length, ctypes.c_void_p(out.data_ptr()),
                                                _lib.current_stream_ptr(x.device)), "pl_crc_attach")
        return out

    def forward(self, inputs):
        inputs, from_numpy = _as_tensor(inputs)
        assert len(inputs.shape) > 1
        if inputs.shape[-1] != self._k:
            self.build(inputs.shape)  # crc.py:93-95 (without its breakpoint)
        dev = _gpu_for(inputs, self.device)
        x = inputs.reshape(-1, self._k).to(device=dev, dtype=tc.float32).contiguous()
        out = self._attach(x).reshape(*inputs.shape[:-1], self._n)
        if from_numpy:
            return out.to(self.dtype).cpu().numpy()
        return out.to(device=inputs.device, dtype=self.dtype)


class CRCDecoder(nn.Module):
    """Checks and strips the CRC (crc.py:111-138).

    forward(inputs [..., k + crc_length]) -> (x [..., k], crc_valid [..., 1] bool).
    """

    def __init__(self, crc_encoder, dtype=tc.float32):
        super().__init__()
        assert isinstance(crc_encoder, CRCEncoder), "crc_encoder must be an instance of CRCEncoder."
        self._encoder = crc_encoder
        self.dtype = dtype
        self._rows = {}

    def _rows_for(self, length):
        if length not in self._rows:
            self._rows[length] = _Rows(self._encoder.crc_degree, length)
        return self._rows[length]

    def forward(self, inputs):
        inputs, from_numpy = _as_tensor(inputs)
        assert len(inputs.shape) >= 2, "Input tensor must have at least rank 2."
        L = self._encoder.crc_length
        assert inputs.shape[-1] >= L, f"Last dimension of inputs must be at least {L}."
        length = inputs.shape[-1]
        x_info = inputs[..., :-L]
        dev = _gpu_for(inputs, self._encoder.device)
        w = inputs.reshape(-1, length).to(device=dev, dtype=tc.float32).contiguous()
        valid = tc.empty(w.shape[0], dtype=tc.uint8, device=dev)
        with tc.cuda.device(dev):
            _lib.check(_lib.lib().pl_crc_check(ctypes.c_void_p(w.data_ptr()), w.shape[0], length,
                                               ctypes.c_void_p(self._rows_for(length).on(dev).data_ptr()), L,
                                               ctypes.c_void_p(valid.data_ptr()), _lib.current_stream_ptr(dev)),
                       "pl_crc_check")
        valid = valid.to(tc.bool).reshape(*inputs.shape[:-1], 1)
        if from_numpy:
            return x_info.numpy(), valid.cpu().numpy()
        return x_info, valid.to(inputs.device)
