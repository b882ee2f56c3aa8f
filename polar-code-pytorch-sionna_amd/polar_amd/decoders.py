"""Drop-in SC / SCL decoder modules with the reference's constructor and forward() contracts.

  SC_Dec   <-> x_run_sn_polar/polar/polar_sc.py:5-133   (min-sum f; `mode` is inert as in :46)
  SCL_Dec  <-> x_run_sn_polar/polar/polar_scl.py:5-234  (min-sum f, fp64 path metrics)

Decoding always runs in libpolar_mi355x.so on a ROCm GPU.  CPU input tensors (the reference
harness produces them) are copied to the GPU and the result is copied back, so the modules can
replace the reference ones unchanged; GPU inputs stay on the GPU.  Without a GPU the forward
raises: there is no CPU decoder in the product path.
"""
import numpy as np
import torch as tc
from torch import nn

from . import _lib, ops


def _frozen_mask(frozen_pos, n):
    fp = frozen_pos.detach().cpu().numpy() if isinstance(frozen_pos, tc.Tensor) else np.asarray(frozen_pos)
    m = np.zeros(n, dtype=np.uint8)
    m[fp.astype(np.int64)] = 1
    return fp, m


def check_supported(n, list_size=1):
    """Raise ValueError at construction for codes no MI355X kernel decodes (the C library's
    limits, include/polar_mi355x.h: n <= 2048; list decoding at n = 2048 needs list_size <= 16)."""
    n, list_size = int(n), int(list_size)
    if n > 2048 or (list_size > 1 and n > 1024 and list_size > 16):
        what = "SC" if list_size == 1 else f"SCL (list_size {list_size})"
        raise ValueError(f"{what} decoding of n = {n} is not supported by the MI355X kernels "
                         "(n <= 2048; list_size <= 16 at n = 2048)")


def _gpu_for(inputs, module_device):
    if inputs.device.type == "cuda":
        return inputs.device
    d = tc.device(module_device) if module_device is not None else tc.device("cpu")
    if d.type == "cuda":
        return d
    if not tc.cuda.is_available():
        raise RuntimeError("polar_amd decoders run only on a ROCm GPU (MI355X); none is visible")
    return tc.device("cuda", tc.cuda.current_device())


class SC_Dec(nn.Module):
    """Successive-cancellation decoder (reference: x_run_sn_polar/polar/polar_sc.py:5-133)."""

    def __init__(self, frozen_pos, n, output_dtype=tc.float32, device='cpu', mode='llr'):
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
        self.mode = mode
        self.device = device
        self._n_stages = int(np.log2(n))
        self._mask = mask
        check_supported(n)
        self._plans = _lib.PlanSet()

    def plan(self, device=None):
        """The decoding plan on `device` (default: the current GPU); plans are device-bound."""
        return self._plans.get(device, self._make_plan)

    def _make_plan(self, dev):
        return _lib.Plan(self.n, self._mask, 1, _lib.PL_F_MINSUM, self.llr_max, device=dev)

    def forward(self, inputs):
        if self.mode not in ("llr", "max"):  # polar_sc.py:44-45 raises inside f
            raise Exception('error...')
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
    """SC-list decoder (reference: x_run_sn_polar/polar/polar_scl.py:5-234).

    crc_degree / use_hybrid_sc / use_fast_scl / return_crc_status are accepted and, exactly as in
    the x_run reference, not used.  After forward(), `msg_pm` holds the final sorted path metrics
    [bs, 2L] (float64 numpy), as the reference leaves in self.msg_pm (polar_scl.py:204).
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
    def frozen_pos(self):
        return self._frozen_pos

    @property
    def msg_pm(self):
        return None if self._pm is None else self._pm.cpu().numpy()

    def plan(self, device=None):
        """The decoding plan on `device` (default: the current GPU); plans are device-bound."""
        return self._plans.get(device, self._make_plan)

    def _make_plan(self, dev):
        return _lib.Plan(self._n, self._mask, self._list_size, _lib.PL_F_MINSUM, self._llr_max, device=dev)

    def forward(self, inputs):
        assert inputs.dtype == self.output_dtype, "Invalid input dtype."
        inputs = inputs.to(tc.float32)
        assert inputs.shape[-1] == self._n, "Last input dim must be of len n."
        assert inputs.dim() > 1
        input_shape = inputs.shape
        llr = inputs.reshape([-1, self._n])
        dev = _gpu_for(llr, self.device)
        u_hat, self._pm = ops.scl_decode(self.plan(dev), llr.to(dev, non_blocking=True), return_pm=True)
        output_shape = list(input_shape)
        output_shape[-1] = self.k
        output_shape[0] = -1
        return u_hat.reshape(output_shape).to(self.output_dtype).to(device=self.device)
