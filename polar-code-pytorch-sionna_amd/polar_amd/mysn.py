"""Drop-ins for the library API decoders of the reference (my_sn/fec/polar/dec.py).

  SC_Dec   <-> my_sn/fec/polar/dec.py:13-157    exact log-domain boxplus f (dec.py:33-46)
  SCL_Dec  <-> my_sn/fec/polar/dec.py:158-537   exact f, fast-SCL rate-0/repetition pruning
               (use_fast_scl, :367-376), optional CRC-aided pick (crc_degree, :507-518)

Both run in libpolar_mi355x.so on a ROCm GPU (SC: the per-code specialised kernel in exact-f mode;
SCL: the subtree kernel scl_tree_kernel.hip with exact f / fast-SCL / CRC for 32 <= n <= 1024,
the generic scl_kernel.hip otherwise -- n = 2048 with list_size <= 16, the largest list state
that fits one CU's LDS; larger codes raise ValueError at construction).  Differences from the reference are stated where
they exist:
  * The reference's CRCEncoder cannot be constructed as shipped (crc.py:81 reads self.device,
    which is never set), so SCL_Dec(crc_degree=...) raises there; here it works, with the CRC of
    crc.py (pinned by tests/golden/crc.npz, generated with that one attribute set at run time).
  * use_hybrid_sc and return_crc_status raise NotImplementedError, as the reference does
    ("not implement...", dec.py:497-498, :534-535).
  * Path-metric ties are broken in the stable (metric, index) order (the reference's np.argsort is
    unstable and host-dependent, see polar_scl.py notes in DESIGN.md §4).
"""
import numpy as np
import torch as tc
from torch import nn

from . import _lib, ops
from .decoders import _frozen_mask, _gpu_for, check_supported

# 5G CRC polynomials (my_sn/fec/crc.py:38-52 / 3GPP TS 38.212 Sec. 5.1), exponents
CRC_POLYS = {"CRC24A": [24, 23, 18, 17, 14, 11, 10, 7, 6, 5, 4, 3, 1, 0], "CRC24B": [24, 23, 6, 5, 1, 0],
             "CRC24C": [24, 23, 21, 20, 17, 15, 13, 12, 8, 4, 2, 1, 0], "CRC16": [16, 12, 5, 0],
             "CRC11": [11, 10, 9, 5, 0], "CRC6": [6, 5, 0]}


def crc_params(crc_degree):
    """(degree, generator mask without x^degree) of a 5G CRC name (crc.py:_select_crc_pol)."""
    if crc_degree not in CRC_POLYS:
        raise ValueError("Invalid CRC Polynomial")
    ex = CRC_POLYS[crc_degree]
    return ex[0], sum(1 << e for e in ex if e < ex[0])


class SC_Dec(nn.Module):
    """my_sn SC decoder with the exact boxplus f (reference: my_sn/fec/polar/dec.py:13-157)."""

    def __init__(self, frozen_pos, n, output_dtype=tc.float32, device='cpu'):
        super().__init__()
        self.output_dtype = output_dtype
        self.n = n
        self.frozen_pos = frozen_pos
        self.k = self.n - len(self.frozen_pos)
        fp, mask = _frozen_mask(frozen_pos, n)
        self.info_pos = np.setdiff1d(np.arange(self.n), fp)
        assert self.k == len(self.info_pos), "Internal error: invalid " "info_pos generated."
        self.llr_max = 30.
        self._frozen_ind = mask.astype(np.float64)
        self._use_fast_sc = False
        self.device = device
        self._mask = mask
        check_supported(n)
        self._plans = _lib.PlanSet()

    def plan(self, device=None):
        """The decoding plan on `device` (default: the current GPU); plans are device-bound."""
        return self._plans.get(device, self._make_plan)

    def _make_plan(self, dev):
        return _lib.Plan(self.n, self._mask, 1, _lib.PL_F_EXACT, self.llr_max, device=dev)

    def forward(self, inputs):
        inputs = inputs.to(dtype=tc.float32)
        assert inputs.shape[-1] == self.n, "Last input dim must be of len n."
        assert len(inputs.shape) > 1
        input_shape = inputs.shape
        llr = inputs.reshape([-1, self.n])
        dev = _gpu_for(llr, self.device)
        u_hat = ops.sc_decode(self.plan(dev), llr.to(dev, non_blocking=True))
        output_shape = list(input_shape)
        output_shape[-1] = self.k
        output_shape[0] = -1
        return u_hat.reshape(output_shape).to(device=inputs.device, dtype=self.output_dtype)


class SCL_Dec(nn.Module):
    """my_sn SC-list decoder (reference: my_sn/fec/polar/dec.py:158-537).

    After forward(), `msg_pm` holds the metrics the reference leaves behind: [bs, 2L] float64,
    sorted, with the CRC penalty added in place when a CRC is used (dec.py:515-518 modifies the
    array _decode_np_batch returned, which is self.msg_pm).
    """

    def __init__(self, frozen_pos, n, list_size=8, crc_degree=None, use_hybrid_sc=False, use_fast_scl=True,
                 return_crc_status=False, output_dtype=tc.float32, device='cpu'):
        super().__init__()
        self.device = device
        if output_dtype not in (tc.float16, tc.float32, tc.float64):
            raise ValueError('output_dtype must be {tf.float16, tf.float32, tf.float64}.')
        self.output_dtype = output_dtype
        n = int(n)
        assert len(frozen_pos) <= n, "Num. of elements in frozen_pos cannot be greater than n."
        assert np.log2(n) == int(np.log2(n)), "n must be a power of 2."
        assert np.log2(list_size) == int(np.log2(list_size)), "list_size must be a power of 2."
        self._use_fast_scl = bool(use_fast_scl)
        self._use_hybrid_sc = False
        self._n = n
        self._frozen_pos = frozen_pos
        self._k = self._n - len(self._frozen_pos)
        self._list_size = list_size
        fp, mask = _frozen_mask(frozen_pos, n)
        self._info_pos = np.setdiff1d(np.arange(self._n), fp)
        self._llr_max = 30.
        assert self._k == len(self._info_pos), "Internal error: invalid info_pos generated."
        self._frozen_ind = mask.astype(np.float64)
        self._n_stages = int(np.log2(self._n))
        if crc_degree is not None:
            self._use_crc = True
            self._crc = crc_params(crc_degree)
            self._k_crc = self._crc[0]
        else:
            self._use_crc = False
            self._crc = (0, 0)
            self._k_crc = 0
        assert self._k >= self._k_crc, "Value of k is too small for given CRC_degree."
        if (crc_degree is None) and return_crc_status:
            raise ValueError("Returning CRC status requires given crc_degree.")
        self._return_crc_status = return_crc_status
        if use_hybrid_sc:
            raise NotImplementedError("use_hybrid_sc: not implemented in the reference either (dec.py:497-498)")
        self._mask = mask
        check_supported(n, list_size)
        self._plans = _lib.PlanSet()
        self._pm = None

    @property
    def n(self):
        return self._n

    @property
    def k(self):
        return self._k

    @property
    def k_crc(self):
        return self._k_crc

    @property
    def frozen_pos(self):
        return self._frozen_pos

    @property
    def info_pos(self):
        return self._info_pos

    @property
    def llr_max(self):
        return self._llr_max

    @property
    def list_size(self):
        return self._list_size

    @property
    def msg_pm(self):
        return None if self._pm is None else self._pm.cpu().numpy()

    def plan(self, device=None):
        """The decoding plan on `device` (default: the current GPU); plans are device-bound."""
        return self._plans.get(device, self._make_plan)

    def _make_plan(self, dev):
        flags = _lib.PL_PLAN_FAST_SCL if self._use_fast_scl else 0
        p = _lib.Plan(self._n, self._mask, self._list_size, _lib.PL_F_EXACT, self._llr_max, flags=flags, device=dev)
        if self._use_crc:
            p.set_crc(*self._crc)
        return p

    def forward(self, inputs):
        assert inputs.dtype == self.output_dtype, "Invalid input dtype."
        inputs = inputs.to(tc.float32)
        assert inputs.shape[-1] == self._n, "Last input dimension must be of length n."
        assert inputs.dim() > 1
        if self._return_crc_status:
            raise NotImplementedError("return_crc_status: not implemented in the reference either (dec.py:534-535)")
        input_shape = inputs.shape
        llr = inputs.reshape([-1, self._n])
        dev = _gpu_for(llr, self.device)
        u_hat, self._pm = ops.scl_decode(self.plan(dev), llr.to(dev, non_blocking=True), return_pm=True)
        output_shape = list(input_shape)
        output_shape[-1] = self.k
        output_shape[0] = -1
        return u_hat.reshape(output_shape).to(self.output_dtype).to(device=self.device)
