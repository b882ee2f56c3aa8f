"""Tensor-level entry points over the C ABI (device tensors in, device tensors out).

Every function here launches a hand-written gfx950 kernel from libpolar_mi355x.so on the
current torch stream of the tensor's device; nothing runs on the CPU and there is no fallback.
"""
import ctypes

import torch

from . import _lib


def _require_cuda(t, name):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise RuntimeError(f"{name} must be a tensor on a ROCm GPU (got "
                           f"{getattr(t, 'device', type(t))}); the MI355X decoder has no CPU path")


def _counts(counts, device):
    """The int64 device counters a counting kernel accumulates into with 64-bit atomics: created
    if None, else checked (contiguous int64 with >= 2 elements on `device`), so a host, narrower
    or foreign-device tensor never reaches the kernel as a raw pointer."""
    if counts is None:
        return torch.zeros(2, dtype=torch.int64, device=device)
    if not isinstance(counts, torch.Tensor) or counts.dtype != torch.int64 or not counts.is_contiguous() \
            or counts.numel() < 2 or counts.device != torch.device(device):
        raise ValueError(f"counts must be a contiguous int64 tensor of >= 2 elements on {device}, got "
                         f"{getattr(counts, 'dtype', type(counts))} {tuple(getattr(counts, 'shape', ()))} on "
                         f"{getattr(counts, 'device', None)}")
    return counts


def _out_kind(dtype):
    if dtype == torch.float32:
        return _lib.PL_OUT_F32
    if dtype == torch.uint8:
        return _lib.PL_OUT_U8
    raise ValueError(f"unsupported decoder output dtype {dtype}")


def sc_decode(plan, llr_logits, out=None, out_dtype=torch.float32):
    """SC-decode [bs, n] fp32 logits on the GPU -> [bs, k] bits (polar_sc.py:113-133 semantics)."""
    _require_cuda(llr_logits, "llr_logits")
    x = llr_logits
    if x.dtype != torch.float32 or not x.is_contiguous():
        x = x.to(torch.float32).contiguous()
    if x.dim() != 2 or x.shape[1] != plan.n:
        raise ValueError(f"llr_logits must be [bs, {plan.n}], got {tuple(x.shape)}")
    bs = x.shape[0]
    if out is None:
        out = torch.empty((bs, plan.k), dtype=out_dtype, device=x.device)
    elif out.shape != (bs, plan.k) or not out.is_contiguous() or out.device != x.device:
        raise ValueError("out must be a contiguous [bs, k] tensor on the input's device")
    kind = _out_kind(out.dtype)
    with torch.cuda.device(x.device):
        st = _lib.current_stream_ptr(x.device)
        _lib.check(_lib.lib().pl_sc_decode(plan.handle, ctypes.c_void_p(x.data_ptr()), bs,
                                           ctypes.c_void_p(out.data_ptr()), kind, st), "pl_sc_decode")
    return out


def scl_workspace(plan, bs, device):
    """A device workspace of pl_scl_workspace_size(plan, bs) bytes (reusable across calls)."""
    ws_bytes = int(_lib.lib().pl_scl_workspace_size(plan.handle, bs))
    return torch.empty((max(ws_bytes, 1),), dtype=torch.uint8, device=device)


def scl_decode(plan, llr_logits, out=None, out_dtype=torch.float32, return_pm=False, workspace=None):
    """SCL-decode [bs, n] fp32 logits -> [bs, k] bits (+ sorted path metrics [bs, 2L] fp64).
    workspace: optional uint8 device tensor from scl_workspace() (allocated per call if None)."""
    _require_cuda(llr_logits, "llr_logits")
    x = llr_logits
    if x.dtype != torch.float32 or not x.is_contiguous():
        x = x.to(torch.float32).contiguous()
    if x.dim() != 2 or x.shape[1] != plan.n:
        raise ValueError(f"llr_logits must be [bs, {plan.n}], got {tuple(x.shape)}")
    bs = x.shape[0]
    if out is None:
        out = torch.empty((bs, plan.k), dtype=out_dtype, device=x.device)
    kind = _out_kind(out.dtype)
    pm = torch.empty((bs, 2 * plan.list_size), dtype=torch.float64, device=x.device) if return_pm else None
    L = _lib.lib()
    ws_bytes = int(L.pl_scl_workspace_size(plan.handle, bs))
    ws = workspace if workspace is not None else scl_workspace(plan, bs, x.device)
    if ws.device != x.device or ws.numel() < ws_bytes:
        raise ValueError(f"workspace must hold {ws_bytes} bytes on {x.device}")
    with torch.cuda.device(x.device):
        st = _lib.current_stream_ptr(x.device)
        _lib.check(L.pl_scl_decode(plan.handle, ctypes.c_void_p(x.data_ptr()), bs, ctypes.c_void_p(out.data_ptr()),
                                   kind, ctypes.c_void_p(pm.data_ptr() if pm is not None else 0),
                                   ctypes.c_void_p(ws.data_ptr()), ws_bytes, st), "pl_scl_decode")
    return (out, pm) if return_pm else out


def polar_encode(plan, u_bits, out=None):
    """Encode [bs, k] 0/1 fp32 information bits -> [bs, n] fp32 codewords (enc.py:30-43)."""
    _require_cuda(u_bits, "u_bits")
    u = u_bits
    if u.dtype != torch.float32 or not u.is_contiguous():
        u = u.to(torch.float32).contiguous()
    if u.dim() != 2 or u.shape[1] != plan.k:
        raise ValueError(f"u_bits must be [bs, {plan.k}], got {tuple(u.shape)}")
    bs = u.shape[0]
    if out is None:
        out = torch.empty((bs, plan.n), dtype=torch.float32, device=u.device)
    with torch.cuda.device(u.device):
        st = _lib.current_stream_ptr(u.device)
        _lib.check(_lib.lib().pl_polar_encode(plan.handle, ctypes.c_void_p(u.data_ptr()), bs,
                                              ctypes.c_void_p(out.data_ptr()), st), "pl_polar_encode")
    return out


def awgn_qpsk_llr(plan, bs, no, seed, iteration, row0=0, with_bits=True):
    """The fused System_AWGN_model producer (pl_awgn_qpsk_llr) on the plan's device: returns
    (u [bs, k] fp32 0/1 or None, logits [bs, n] fp32) for rows row0.. of the (seed, iteration)
    stream."""
    dev = plan.device
    no = float(no)
    if not no > 0.0:
        raise ValueError(f"noise variance must be positive, got {no}")
    if not 0 <= int(iteration) < 2 ** 32:
        raise ValueError(f"iteration must be in [0, 2^32) (the Philox counter word), got {iteration}")
    llr = torch.empty((bs, plan.n), dtype=torch.float32, device=dev)
    u = torch.empty((bs, plan.k), dtype=torch.float32, device=dev) if with_bits else None
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().pl_awgn_qpsk_llr(plan.handle, int(seed) & (2 ** 64 - 1), int(iteration) & (2 ** 64 - 1),
                                               int(row0), int(bs), no,
                                               ctypes.c_void_p(u.data_ptr() if u is not None else 0),
                                               ctypes.c_void_p(llr.data_ptr()), _lib.current_stream_ptr(dev)),
                   "pl_awgn_qpsk_llr")
    return u, llr


def awgn_qpsk_llr_bits(plan, bs, no, seed, iteration, row0=0):
    """pl_awgn_qpsk_llr_bits: the fused producer with the information bits packed -- returns
    (ubits [bs, ceil(k/32)] int32 words, bit m % 32 of word m // 32 = bit m; logits [bs, n] fp32).
    Same stream and logits as awgn_qpsk_llr."""
    dev = plan.device
    no = float(no)
    if not no > 0.0:
        raise ValueError(f"noise variance must be positive, got {no}")
    if not 0 <= int(iteration) < 2 ** 32:
        raise ValueError(f"iteration must be in [0, 2^32) (the Philox counter word), got {iteration}")
    llr = torch.empty((bs, plan.n), dtype=torch.float32, device=dev)
    ubits = torch.empty((bs, (plan.k + 31) // 32), dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().pl_awgn_qpsk_llr_bits(plan.handle, int(seed) & (2 ** 64 - 1),
                                                    int(iteration) & (2 ** 64 - 1), int(row0), int(bs), no,
                                                    ctypes.c_void_p(ubits.data_ptr()), ctypes.c_void_p(llr.data_ptr()),
                                                    _lib.current_stream_ptr(dev)),
                   "pl_awgn_qpsk_llr_bits")
    return ubits, llr


def pack_bits(bits):
    """[..., k] 0/1 tensor -> [rows, ceil(k/32)] int32 words in pl_sc_decode_count's layout."""
    k = bits.shape[-1]
    b = (bits.reshape(-1, k) != 0).to(torch.int64)
    nq = (k + 31) // 32
    b = torch.nn.functional.pad(b, (0, nq * 32 - k)).reshape(-1, nq, 32)
    w = (b << torch.arange(32, device=b.device, dtype=torch.int64)).sum(-1)
    return torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32)



def sc_decode_count(plan, llr_logits, ref_bits, counts=None):
    """pl_sc_decode_count: SC decode fused with count_errors / count_block_errors (my_sn/sim.py:7-18)
    against packed reference bits (awgn_qpsk_llr_bits / pack_bits); accumulates [bit errors, block
    errors] into counts (int64 [2] on the device, created if None) and returns it.  Raises
    PolarLibError (PL_ENOTSUP) for a plan on the generic SC kernel."""
    _require_cuda(llr_logits, "llr_logits")
    x = llr_logits
    if x.dtype != torch.float32 or not x.is_contiguous():
        x = x.to(torch.float32).contiguous()
    if x.dim() != 2 or x.shape[1] != plan.n:
        raise ValueError(f"llr_logits must be [bs, {plan.n}], got {tuple(x.shape)}")
    bs = x.shape[0]
    nq = (plan.k + 31) // 32
    if ref_bits.shape != (bs, nq) or ref_bits.dtype != torch.int32 or ref_bits.device != x.device:
        raise ValueError(f"ref_bits must be int32 [{bs}, {nq}] on the input's device")
    ref = ref_bits.contiguous()
    counts = _counts(counts, x.device)
    ws_bytes = int(_lib.lib().pl_sc_count_workspace_size(plan.handle, bs))
    ws = torch.empty((max(ws_bytes, 4),), dtype=torch.uint8, device=x.device)  # per call: stream-safe
    with torch.cuda.device(x.device):
        _lib.check(_lib.lib().pl_sc_decode_count(plan.handle, ctypes.c_void_p(x.data_ptr()), bs,
                                                 ctypes.c_void_p(ref.data_ptr()), ctypes.c_void_p(counts.data_ptr()),
                                                 ctypes.c_void_p(ws.data_ptr()), ws_bytes,
                                                 _lib.current_stream_ptr(x.device)), "pl_sc_decode_count")
    return counts


def sc_sim_count(plan, bs, no, seed, iteration, row0=0, counts=None, dump=False):
    """pl_sc_sim_count: one Monte-Carlo iteration inside the specialised SC kernel -- information
    bits, encoder, QPSK, AWGN and logits generated in the decoder's registers, decoded and counted
    (System_AWGN_model.forward + my_sn/sim.py:84-100).  Accumulates [bit errors, block errors] into
    counts (int64 [2] on the plan's device, created if None) and returns it; with dump=True returns
    (counts, u [bs, k] fp32, logits [bs, n] fp32) as generated.  Raises PolarLibError (PL_ENOTSUP)
    for plans without the fused entry (generic kernel, or not 64 channel slots per lane)."""
    dev = plan.device
    no = float(no)
    if not no > 0.0:
        raise ValueError(f"noise variance must be positive, got {no}")
    bs = int(bs)
    if not 0 <= int(iteration) < 2 ** 32:
        raise ValueError(f"iteration must be in [0, 2^32) (the Philox counter word), got {iteration}")
    counts = _counts(counts, dev)
    u = llr = None
    if dump:
        u = torch.empty((bs, plan.k), dtype=torch.float32, device=dev)
        llr = torch.empty((bs, plan.n), dtype=torch.float32, device=dev)
    ws_bytes = int(_lib.lib().pl_sc_count_workspace_size(plan.handle, bs))
    ws = torch.empty((max(ws_bytes, 4),), dtype=torch.uint8, device=dev)  # per call: stream-safe
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().pl_sc_sim_count(plan.handle, int(seed) & (2 ** 64 - 1), int(iteration) & (2 ** 64 - 1),
                                              int(row0), bs, no, ctypes.c_void_p(counts.data_ptr()),
                                              ctypes.c_void_p(ws.data_ptr()), ws_bytes,
                                              ctypes.c_void_p(llr.data_ptr() if dump else None),
                                              ctypes.c_void_p(u.data_ptr() if dump else None),
                                              _lib.current_stream_ptr(dev)), "pl_sc_sim_count")
    return (counts, u, llr) if dump else counts


def count_errors(a, b, counts=None):
    """[bit errors, block errors] (int64, on the device) of two [..., k] 0/1 fp32 tensors
    (my_sn/sim.py:7-18 count_errors / count_block_errors in one pass); accumulates into counts."""
    _require_cuda(a, "a")
    _require_cuda(b, "b")
    if a.shape != b.shape or a.device != b.device:
        raise ValueError("count_errors: tensors must have the same shape and device")
    k = a.shape[-1] if a.dim() else 1
    x = a.to(torch.float32).contiguous()
    y = b.to(torch.float32).contiguous()
    rows = x.numel() // k if k else 0
    counts = _counts(counts, a.device)
    with torch.cuda.device(a.device):
        _lib.check(_lib.lib().pl_count_errors(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), rows, k,
                                              ctypes.c_void_p(counts.data_ptr()), _lib.current_stream_ptr(a.device)),
                   "pl_count_errors")
    return counts


class LaunchGraph:
    """`launches` back-to-back calls of fn() (decodes of resident batches: ops.sc_decode /
    scl_decode with `out` -- and for SCL `workspace` -- given, so nothing is allocated) captured
    once into a HIP graph and replayed as one submission.  Small batches are launch-bound: at
    (128,256) x 4096 a decode is ~7.5 us per launch issued one by one and ~6.5 us per launch
    replayed (profiles/r05i_graph_time.txt; an empty kernel: ~3 us vs ~1.7 us).  The graph
    holds the buffers' addresses: refill the same tensors in place between replays.  The graph
    also keeps fn -- and with it the plan, tensors and workspace its closure holds -- alive for as
    long as it exists: a plan destroyed under a captured graph would unload the code object its
    kernel launches come from, and freed tensors would be replayed into."""

    def __init__(self, fn, launches, device=None):
        if launches < 1:
            raise ValueError("launches must be >= 1")
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.launches = int(launches)
        self.fn = fn  # keep-alive of everything the captured launches point at (see above)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # one eager call first: plans load their code object lazily
            fn()
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.device(dev), torch.cuda.graph(self.graph):
            for _ in range(self.launches):
                fn()

    def replay(self):
        self.graph.replay()


def shader_clock_ghz(device=None, iters=16384):
    """The shader clock of one CU now (pl_clock_probe: one wave's dependent VALU chain timed by
    s_memtime against the 100 MHz s_memrealtime), in GHz, measured on the current stream of
    `device` -- so it runs right after whatever was queued before it.  Diagnostics for bench.py."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    ticks = torch.zeros(3, dtype=torch.int64, device=dev)
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().pl_clock_probe(ctypes.c_void_p(ticks.data_ptr()), int(iters),
                                             _lib.current_stream_ptr(dev)), "pl_clock_probe")
    t = ticks.cpu()
    return 0.1 * float(t[0]) / max(float(t[1]), 1.0)
