"""LLR producer for the decoder: bits -> polar encoder -> QPSK -> AWGN -> logits (any torch device).

Numerically this follows the reference blocks op for op, in the same RNG call order, so that on
the CPU device it reproduces the reference's LLRs bit for bit (pinned by tests/golden/harness_c1.npz):
  ebnodb2no        my_sn/trans/ebno.py:2-24
  BinarySource     my_sn/trans/binary_source.py:14-19           (randint, float32)
  QamConstell      my_sn/trans/mapping.py:7-48, :49-95          (Gray QPSK, unit energy)
  Mapper           my_sn/trans/mapping.py:97-149
  AWGN             my_sn/trans/channel/awgn.py:6-29 + my_sn/utils.py:2-17 (two torch.normal draws)
  Demapper         my_sn/trans/mapping.py:151-241              (logsumexp, logits log P1/P0)
  System_AWGN_model  x_run_sn_polar/z_sys_model/awgn_model.py:17-44
On a GPU the same ops run on device (different RNG stream, same distribution) and the encoder is
the HIP XOR-butterfly kernel (bit-identical to the reference's dense c@G % 2, enc.py:42).

FusedAWGN is the same system model as ONE HIP kernel (pl_awgn_qpsk_llr, csrc/channel_kernel.hip):
Philox4x32-10 bits and noise, encoder, mapper, channel and demapper fused -- the production
producer on a GPU (statistical parity with the reference; System_AWGN_model keeps the op-by-op
numerics and RNG order for the CPU-device reproduction of the reference).
"""
import numpy as np
import torch as tc
from torch import nn


def ebnodb2no(ebno_db, n_bits_per_sym, coderate):
    ebno = 10. ** (ebno_db / 10.)
    return 1 / (ebno * coderate * n_bits_per_sym / 1)


def splitmix64(x):
    """splitmix64's finaliser (Steele, Lea, Flood 2014): a bijection of 64-bit words."""
    m = 2 ** 64 - 1
    z = x & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def _qam_points(n_bits_per_sym):
    """Gray-labelled, unit-energy QAM points as complex64 numpy (mapping.py:7-48 arithmetic)."""
    assert n_bits_per_sym % 2 == 0 and n_bits_per_sym > 0

    def pam(b):
        if len(b) > 1:
            return (1 - 2 * b[0]) * (2 ** len(b[1:]) - pam(b[1:]))
        return 1 - 2 * b[0]

    c = np.zeros([2 ** n_bits_per_sym], dtype=np.complex64)
    for i in range(2 ** n_bits_per_sym):
        b = np.array(list(np.binary_repr(i, n_bits_per_sym)), dtype=np.int16)
        c[i] = pam(b[0::2]) + 1j * pam(b[1::2])
    m = n_bits_per_sym // 2
    var = 1 / (2 ** (m - 2)) * np.sum(np.linspace(1, 2 ** m - 1, 2 ** (m - 1)) ** 2)
    c /= np.sqrt(var)
    return c


class QamConstellation(nn.Module):
    def __init__(self, n_bits_per_symbol=2, device='cpu'):
        super().__init__()
        self.n_bits_per_sym = int(n_bits_per_symbol)
        self.dtype = tc.complex64
        self.device = device
        p = tc.from_numpy(_qam_points(self.n_bits_per_sym)).to(dtype=tc.complex64, device=device)
        self._points = tc.stack([tc.real(p), tc.imag(p)], dim=0).to(tc.float32)

    @property
    def points(self):
        x = tc.complex(self._points[0], self._points[1])
        energy = tc.mean(tc.abs(x) ** 2)
        return x / tc.sqrt(energy).to(dtype=self.dtype)


class BinarySource(nn.Module):
    def __init__(self, dtype=tc.float32, device='cpu', generator=None):
        super().__init__()
        self.dtype, self.device, self.generator = dtype, device, generator

    def forward(self, shape):
        return tc.randint(0, 2, size=shape, device=self.device, dtype=self.dtype, generator=self.generator)


class Mapper(nn.Module):
    def __init__(self, constell):
        super().__init__()
        self.constell = constell
        m = constell.n_bits_per_sym
        self._base = 2 ** tc.tensor(range(m - 1, -1, -1), device=constell.device)

    def forward(self, bits):
        m = self.constell.n_bits_per_sym
        shape = [-1] + list(bits.shape[1:-1]) + [int(bits.shape[-1] / m), m]
        idx = tc.sum(bits.reshape(shape).to(tc.int32) * self._base, dim=-1)
        return self.constell.points[idx]


class AWGN(nn.Module):
    def __init__(self, device='cpu', generator=None):
        super().__init__()
        self.device, self.generator = device, generator

    def forward(self, inputs):
        x, no = inputs
        # utils.py:11-15 passes a 0-dim fp32 tensor; the arg parser reads it as this same double
        std = float(tc.sqrt(tc.tensor(1.0 / 2, dtype=tc.float32)))
        kw = dict(size=x.shape, dtype=tc.float32, device=self.device)
        if self.generator is not None:
            kw["generator"] = self.generator
        xr = tc.normal(mean=0, std=std, **kw)
        xi = tc.normal(mean=0, std=std, **kw)
        noise = tc.complex(xr, xi)
        no = tc.as_tensor(no).reshape([1] * len(x.shape)) if tc.is_tensor(no) and no.dim() == 0 else no
        noise *= tc.sqrt(tc.as_tensor(no).to(dtype=tc.float32)).to(dtype=noise.dtype, device=self.device)
        return x + noise


class Demapper(nn.Module):
    """Exact (logsumexp) demapper: logits log(P(b=1)/P(b=0)) per bit."""

    def __init__(self, constell):
        super().__init__()
        self.constell = constell
        m = constell.n_bits_per_sym
        npts = 2 ** m
        a = np.array([list(np.binary_repr(i, m)) for i in range(npts)], dtype=np.int16)
        c0 = np.stack([np.where(a[:, i] == 0)[0] for i in range(m)], axis=1)
        c1 = np.stack([np.where(a[:, i] == 1)[0] for i in range(m)], axis=1)
        self._c0 = tc.tensor(c0, dtype=tc.int64)
        self._c1 = tc.tensor(c1, dtype=tc.int64)

    def forward(self, inputs):
        y, no = inputs
        pts = self.constell.points.reshape([1] * len(y.shape) + [-1])
        sq = tc.abs(y.unsqueeze(dim=-1) - pts) ** 2
        no_t = tc.as_tensor(no)
        no_t = no_t.reshape(list(no_t.shape) + [1] * (len(sq.shape) - no_t.dim())).to(y.device)
        e = -sq / no_t
        llr = tc.logsumexp(e[..., self._c1.to(e.device)], dim=-2) - tc.logsumexp(e[..., self._c0.to(e.device)], dim=-2)
        return llr.reshape(list(y.shape[:-1]) + [y.shape[-1] * self.constell.n_bits_per_sym])


class DenseEncoder(nn.Module):
    """c[:, info_pos] = u; (c @ G) % 2 -- the reference harness encoder (enc.py:30-43), any device."""

    def __init__(self, frozen_pos, n, G, device='cpu'):
        super().__init__()
        fp = frozen_pos.cpu().numpy() if tc.is_tensor(frozen_pos) else np.asarray(frozen_pos)
        self.n = n
        self.info_pos = tc.from_numpy(np.setdiff1d(np.arange(n), fp)).to(device)
        self.G = G.to(device)

    def forward(self, u):
        c = tc.zeros([u.shape[0], self.n], dtype=tc.float32, device=u.device)
        c[..., self.info_pos] = u
        return (c @ self.G % 2).to(tc.float32)


class GpuEncoder(nn.Module):
    """Polar encoder on the GPU through the HIP butterfly kernel (same output as DenseEncoder)."""

    def __init__(self, frozen_pos, n):
        super().__init__()
        from . import _lib
        from .frozen import frozen_mask
        self._n, self._mask = n, frozen_mask(frozen_pos, n)
        self._plans = _lib.PlanSet()

    def _make_plan(self, dev):
        from . import _lib
        return _lib.Plan(self._n, self._mask, 1, flags=_lib.PL_PLAN_GENERIC, device=dev)

    def forward(self, u):
        from . import ops
        return ops.polar_encode(self._plans.get(u.device, self._make_plan), u)


class System_AWGN_model(nn.Module):
    """bits -> encoder -> QPSK -> AWGN -> demapper -> decoder (awgn_model.py:17-44)."""

    def __init__(self, n, k, encoder, decoder, cw_estimates=False, device='cpu', generator=None):
        super().__init__()
        self.cw_estimates = cw_estimates
        self.n_bits_per_sym = 2
        self.n, self.k = n, k
        self.coderate = self.k / self.n
        self.constell = QamConstellation(self.n_bits_per_sym, device=device)
        self.mapper = Mapper(self.constell)
        self.demapper = Demapper(self.constell)
        self.binary_src = BinarySource(device=device, generator=generator)
        self.awgn_channel = AWGN(device=device, generator=generator)
        self.encoder, self.decoder = encoder, decoder

    def llrs(self, batch_size, ebno_db):
        """The channel half of forward(): (bits, codewords, logits)."""
        no = ebnodb2no(ebno_db, self.n_bits_per_sym, self.coderate)
        bits = self.binary_src([batch_size, self.k])
        codewords = self.encoder(bits)
        x = self.mapper(codewords)
        y = self.awgn_channel([x, no])
        return bits, codewords, self.demapper([y, no])

    def forward(self, batch_size, ebno_db):
        bits, codewords, llr = self.llrs(batch_size, ebno_db)
        bits_hat = self.decoder(llr)
        if self.cw_estimates:
            return codewords, bits_hat
        return bits, bits_hat


class FusedAWGN(nn.Module):
    """System_AWGN_model (awgn_model.py:17-44) with the whole producer -- bits, polar encoder, QPSK
    mapper, AWGN, demapper -- as one HIP kernel per call (pl_awgn_qpsk_llr).

    Same interface: forward(batch_size, ebno_db) -> (bits, bits_hat) (or (codewords, bits_hat)
    with cw_estimates), llrs(batch_size, ebno_db) -> (bits, None, logits).  Randomness is Philox
    keyed by `seed`.  A draw is keyed by (SNR point, iteration): forward / llrs / error_counts take
    stream=(point, iteration) (sim_ber passes its loop indices, so a speculatively launched
    iteration never shifts another point's codewords); without it every call draws the next
    iteration of point 0 (`iteration` counts those calls).  The key is `seed` in the first run and
    changes with every run sim_ber makes over the model (`epoch`, next_epoch(): sim_ber mutates the model it is
    given, once per call, also when the call raises).  Stream row r of a draw is codeword
    row0 + r; the point lives in the row's high 32 bits (counter word 1), so row0 + batch_size
    must stay below 2^32.  `row0` offsets the rows (a rank's shard of a multi-GPU batch)."""

    keyed_streams = True  # sim_ber: draws depend on (point, iteration), not on call order

    def __init__(self, n, k, frozen_pos, decoder, device=None, seed=42, row0=0, cw_estimates=False,
                 sim_kernel=True):
        super().__init__()
        self.sim_kernel = bool(sim_kernel)  # error_counts: the fused producer+decoder kernel when the plan has it
        from . import _lib
        from .frozen import frozen_mask
        self.n, self.k = int(n), int(k)
        self.n_bits_per_sym = 2
        self.coderate = self.k / self.n
        self.decoder = decoder
        self.cw_estimates = cw_estimates
        self.seed, self.row0, self.iteration = int(seed), int(row0), 0
        self.epoch = 0  # runs of sim_ber over this model so far (next_epoch): part of the Philox key
        if not 0 <= self.row0 < 2 ** 32:
            raise ValueError(f"row0 must be in [0, 2^32), got {row0}")
        self._mask = frozen_mask(frozen_pos, self.n)
        assert self.n - int(self._mask.sum()) == self.k, "k must equal n - len(frozen_pos)"
        self.device = tc.device(device) if device is not None else tc.device("cuda", tc.cuda.current_device())
        self._plans = _lib.PlanSet()

    def next_epoch(self):
        """Start a new run: the following draws use a fresh Philox key (sim_ber calls this once
        per run, so repeating a sweep over the same model does not repeat its codewords; the
        reference draws them from its advancing global RNG)."""
        self.epoch += 1

    def key(self):
        """The Philox key of the current epoch: the seed itself in epoch 0 (the pinned streams),
        otherwise splitmix64(seed + epoch * golden gamma) -- a bijective mixer, so distinct epochs
        of one seed get distinct keys, and related seeds (seed vs seed ^ gamma) do not replay each
        other's epochs the way a plain seed ^ epoch * gamma key would."""
        if self.epoch == 0:
            return self.seed & (2 ** 64 - 1)
        return splitmix64((self.seed + self.epoch * 0x9E3779B97F4A7C15) & (2 ** 64 - 1))

    def _make_plan(self, dev):
        from . import _lib
        return _lib.Plan(self.n, self._mask, 1, flags=_lib.PL_PLAN_GENERIC, device=dev)

    def _draw(self, batch_size, stream):
        """(iteration, first stream row) of a draw of batch_size codewords."""
        if stream is None:
            point, it = 0, self.iteration
            self.iteration += 1
        else:
            point, it = int(stream[0]), int(stream[1])
        if not 0 <= it < 2 ** 32:
            raise ValueError(f"Monte-Carlo iteration must be in [0, 2^32), got {it}")
        if not 0 <= point < 2 ** 31:
            raise ValueError(f"SNR point index must be in [0, 2^31), got {point}")
        if self.row0 + int(batch_size) > 2 ** 32:
            raise ValueError("row0 + batch_size must not exceed 2^32 (the point index is the row's high word)")
        return it, self.row0 + (point << 32)

    def llrs(self, batch_size, ebno_db, stream=None):
        from . import ops
        no = float(ebnodb2no(float(ebno_db), self.n_bits_per_sym, self.coderate))
        it, row0 = self._draw(batch_size, stream)
        bits, llr = ops.awgn_qpsk_llr(self._plans.get(self.device, self._make_plan), int(batch_size), no,
                                      self.key(), it, row0)
        return bits, None, llr

    def forward(self, batch_size, ebno_db, stream=None):
        bits, _, llr = self.llrs(batch_size, ebno_db, stream)
        bits_hat = self.decoder(llr)
        if self.cw_estimates:
            from . import ops
            return ops.polar_encode(self._plans.get(self.device, self._make_plan), bits), bits_hat
        return bits, bits_hat

    def error_counts(self, batch_size, ebno_db, counts=None, stream=None):
        """One Monte-Carlo iteration straight to the harness's counters: [bit errors, block errors]
        (int64 [2] on the device, accumulated into counts) of decoding a fresh batch -- what
        count_errors / count_block_errors (my_sn/sim.py:7-18) give on forward()'s output.
          * pl_sc_sim_count (sim_kernel=True and a specialised plan with 64 channel slots per
            lane): the whole iteration inside the SC kernel, nothing written to HBM but the
            counters; its Philox streams are its own (the same model, not forward()'s draw).
          * otherwise pl_awgn_qpsk_llr_bits + pl_sc_decode_count: the producer writes the logits
            and the information bits packed, the decoder compares its decisions with them -- the
            same draw as forward() for this iteration.
        Returns None (nothing drawn) when the decoder is not this package's SC_Dec on a specialised
        plan; sim_ber then runs forward() and counts separately."""
        from . import _lib, ops
        from .decoders import SC_Dec
        dec = self.decoder
        if self.cw_estimates or type(dec) is not SC_Dec or dec.mode not in ("llr", "max"):
            return None
        plan = dec.plan(self.device)
        if plan.kernel()[0] != "specialized":
            return None
        no = float(ebnodb2no(float(ebno_db), self.n_bits_per_sym, self.coderate))
        it, row0 = self._draw(batch_size, stream)
        if self.sim_kernel:
            try:
                return ops.sc_sim_count(plan, int(batch_size), no, self.key(), it, row0, counts)
            except _lib.PolarLibError as e:
                if e.code != _lib.PL_ENOTSUP:
                    raise
                self.sim_kernel = False  # this plan's kernel has no fused entry: the two-kernel path
        ubits, llr = ops.awgn_qpsk_llr_bits(self._plans.get(self.device, self._make_plan), int(batch_size), no,
                                            self.key(), it, row0)
        return ops.sc_decode_count(plan, llr, ubits, counts)


def philox4x32_10(ctr, key):
    """Random123 Philox4x32-10 on numpy uint32 arrays: ctr [..., 4], key [..., 2] -> [..., 4].
    The host restatement of csrc/channel_kernel.hip's generator (tests pin the kernel's bit
    placement against it; the Random123 known-answer vectors pin this function)."""
    c = np.array(ctr, dtype=np.uint64)
    k0 = np.array(key[..., 0], dtype=np.uint64)
    k1 = np.array(key[..., 1], dtype=np.uint64)
    m32 = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[..., 0]
        p1 = np.uint64(0xCD9E8D57) * c[..., 2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & m32
        hi1, lo1 = p1 >> np.uint64(32), p1 & m32
        c = np.stack([hi1 ^ c[..., 1] ^ k0, lo1, hi0 ^ c[..., 3] ^ k1, lo0], axis=-1)
        k0 = (k0 + np.uint64(0x9E3779B9)) & m32
        k1 = (k1 + np.uint64(0xBB67AE85)) & m32
    return c.astype(np.uint32)


def fused_info_bits(seed, iteration, rows, k):
    """The information bits pl_awgn_qpsk_llr draws for stream rows `rows` (1-D int64): bit r of a
    row is bit r % 32 of Philox word r // 32, word q = component q % 4 of the block with counter
    (row, iteration, q // 4) -- returned as float32 [len(rows), k]."""
    rows = np.asarray(rows, dtype=np.int64).reshape(-1)
    nq = (k + 31) // 32
    q = np.arange(nq)
    ctr = np.zeros((len(rows), nq, 4), dtype=np.uint64)
    ctr[..., 0] = (rows & 0xFFFFFFFF)[:, None]
    ctr[..., 1] = (rows >> 32)[:, None]
    ctr[..., 2] = np.uint64(iteration & 0xFFFFFFFF)
    ctr[..., 3] = (q >> 2)[None, :]
    key = np.zeros((len(rows), nq, 2), dtype=np.uint64)
    key[..., 0] = seed & 0xFFFFFFFF
    key[..., 1] = (seed >> 32) & 0xFFFFFFFF
    words = philox4x32_10(ctr, key)               # [rows, nq, 4]
    w = words[:, q, q & 3]                        # [rows, nq]
    bits = (w[..., None] >> np.arange(32, dtype=np.uint32)) & 1
    return bits.reshape(len(rows), nq * 32)[:, :k].astype(np.float32)
