"""Parity of the my_sn decoder drop-ins on the GPU.

  polar_amd.mysn.SCL_Dec <-> my_sn/fec/polar/dec.py:158-537 (exact f, fast-SCL, CRC-aided pick)
  polar_amd.mysn.SC_Dec  <-> my_sn/fec/polar/dec.py:13-157  (exact f)

The exact boxplus f is log/exp arithmetic, so the GPU (ocml fp64) and the reference (numpy) can
differ in the last ulp; the bits are gated by a one-sided binomial test on the row-mismatch count
(level 1e-3) at the rate tests/test_exactf_gpu.py establishes with 5,000 reference rows
(P0_SCL = 6e-4, the 95 % bound of the C oracle's own rate there), against both the reference
fixtures and the C oracle (glibc), with path metrics within 1e-6 on agreeing rows.  The
CRC-aided pick and the fast-SCL node sums (numpy pairwise order) are exact given the same
metrics.
"""
import glob
import os
import sys

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
from exactf_recipe import binom_upper_ok  # noqa: E402

P0_SCL = 6e-4  # exact-f SCL row-mismatch rate gate (tests/test_exactf_gpu.py: the oracle's 95 % bound)
P0_SC = 1e-4  # exact-f SC
CASES = [("mysn_scl_L8_32_64", {}), ("mysn_scl_L8_128_256", {}), ("mysn_scl_nofast_L4_32_64", {"fast": False}),
         ("mysn_scl_crc11_L8_32_64", {"crc": "CRC11"}), ("mysn_scl_crc24c_L8_128_256", {"crc": "CRC24C"})]


@pytest.fixture(scope="module")
def pa():
    import polar_amd
    assert torch.cuda.is_available()
    return polar_amd


@pytest.mark.parametrize("fname,kw", CASES, ids=[c[0] for c in CASES])
def test_mysn_scl_golden(pa, fname, kw):
    from polar_amd import mysn
    d = np.load(os.path.join(GOLDEN, fname + ".npz"))
    n, L = int(d["n"]), int(d["L"])
    fp = torch.from_numpy(d["frozen_pos"].astype(np.int64))
    dec = mysn.SCL_Dec(fp, n, list_size=L, use_fast_scl=kw.get("fast", True), crc_degree=kw.get("crc"))
    rows = agree = 0
    for name in [k[4:] for k in d.files if k.startswith("llr_")]:
        x = torch.from_numpy(d["llr_" + name])
        got = dec(x).numpy().astype(np.uint8)
        pm = dec.msg_pm
        ok = (got == d["bits_stable_" + name]).all(1)
        rows += len(ok)
        agree += int(ok.sum())
        assert np.abs(pm[ok] - d["pm_stable_" + name][ok]).max() < 1e-6, name
    assert binom_upper_ok(rows - agree, rows, P0_SCL), (agree, rows)


@pytest.mark.parametrize("log_n", [3, 5, 6, 7, 8, 9, 10])
@pytest.mark.parametrize("L", [2, 8])
@pytest.mark.parametrize("fast", [True, False])
def test_mysn_scl_random_code_vs_oracle(pa, log_n, L, fast):
    """Arbitrary frozen sets.  Min-sum f: bit-exact and metrics to 1e-9, on AWGN codewords with
    every 9th LLR rounded (exact ties and zeros).  Exact f: row mismatches against the oracle
    within the binomial gate at P0_SCL, metrics to 1e-6 on agreeing rows -- on unrounded AWGN
    codewords of random codes that freeze at least the n/4 least reliable positions.  (With an
    information bit at one of those, its LLR after log2(n) exact-f levels is rounding noise of
    the f formula, e.g. ~1e-16 of either sign, and the list's choice is decided by it: the C
    oracle itself changes 30-75 % of such rows at n = 1024 when 1/4 of its fp64 exp/log results
    move by one ulp, and 0-1 of 37 on these codes.)"""
    from polar_amd import _lib, ops
    n = 1 << log_n
    # every shape runs, n = 1024 at L = 8 included (the configs[3] shape, with and without fast-SCL):
    # the C oracle decodes these 37 rows in ~0.03 s
    rng = np.random.default_rng(log_n * 7 + L + fast)
    k = n // 2
    fp = np.sort(rng.permutation(n)[: n - k])
    bs = 37
    u = rng.integers(0, 2, (bs, k)).astype(np.float32)
    cw = oracle.polar_encode(u, fp, n)
    llr = ((2 * cw - 1) * 2.0 + rng.standard_normal(cw.shape) * 1.4).astype(np.float32)
    llr[:, ::9] = np.round(llr[:, ::9])  # exact ties and zeros
    flags = _lib.PL_PLAN_FAST_SCL if fast else 0
    want, wpm = oracle.scl_decode_mysn(llr, fp, L, fast_scl=fast, exact_f=False)
    plan = _lib.Plan(n, pa.frozen_mask(fp, n), L, _lib.PL_F_MINSUM, flags=flags)
    got, pm = ops.scl_decode(plan, torch.from_numpy(llr).cuda(), return_pm=True)
    assert np.array_equal(got.cpu().numpy(), want)
    assert np.abs(pm.cpu().numpy() - wpm).max() < 1e-9
    base = pa.reference_frozen_pos(n - n // 4, n).numpy()  # the n/4 least reliable positions (froze.py)
    fp = np.sort(np.concatenate([base, rng.choice(np.setdiff1d(np.arange(n), base), n // 4, replace=False)]))
    cw = oracle.polar_encode(u, fp, n)
    llr_awgn = ((2 * cw - 1) * 2.0 + rng.standard_normal(cw.shape) * 1.4).astype(np.float32)
    want, wpm = oracle.scl_decode_mysn(llr_awgn, fp, L, fast_scl=fast, exact_f=True)
    plan = _lib.Plan(n, pa.frozen_mask(fp, n), L, _lib.PL_F_EXACT, flags=flags)
    got, pm = ops.scl_decode(plan, torch.from_numpy(llr_awgn).cuda(), return_pm=True)
    ok = (got.cpu().numpy() == want).all(1)
    assert binom_upper_ok(int((~ok).sum()), len(ok), P0_SCL), ok.mean()
    assert np.abs(pm.cpu().numpy()[ok] - wpm[ok]).max() < 1e-6


@pytest.mark.parametrize("lmax", [7.5, 100.0, 300.0])
@pytest.mark.parametrize("kernel", ["subtree", "generic"])
def test_mysn_scl_exact_f_llr_max_vs_oracle(pa, lmax, kernel):
    """Exact f at llr_max far from 30 (my_sn dec.py:213): the f's exponentials take arguments down
    to -2 llr_max (softplus.h fex_exp: the 2^(j/64) table and the shifter's integer range), the clip
    folds into min(|x|, llr_max).  Strong channel LLRs so the clip binds at 7.5 and node values
    reach hundreds.  (Above llr_max ~355 the reference's own float64 exp(xc + yc) overflows and its
    f turns +inf where ours stays finite: DESIGN.md section 7.)  Row mismatches against the C oracle
    within the P0_SCL gate, metrics to 1e-6 on agreeing rows, on both SCL kernels, fast-SCL on."""
    from polar_amd import _lib, ops
    k, n, L, bs = 128, 256, 8, 64
    rng = np.random.default_rng(int(lmax) + (kernel == "generic"))
    fp = pa.reference_frozen_pos(k, n).numpy()
    u = rng.integers(0, 2, (bs, k)).astype(np.float32)
    cw = oracle.polar_encode(u, fp, n)
    llr = ((2 * cw - 1) * 6.0 + rng.standard_normal(cw.shape) * 3.0).astype(np.float32)
    flags = _lib.PL_PLAN_FAST_SCL | (_lib.PL_PLAN_GENERIC if kernel == "generic" else 0)
    want, wpm = oracle.scl_decode_mysn(llr, fp, L, fast_scl=True, exact_f=True, llr_max=lmax)
    plan = _lib.Plan(n, pa.frozen_mask(fp, n), L, _lib.PL_F_EXACT, llr_max=lmax, flags=flags)
    got, pm = ops.scl_decode(plan, torch.from_numpy(llr).cuda(), return_pm=True)
    ok = (got.cpu().numpy() == want).all(1)
    assert binom_upper_ok(int((~ok).sum()), len(ok), P0_SCL), ok.mean()
    assert np.abs(pm.cpu().numpy()[ok] - wpm[ok]).max() < 1e-6
    assert np.isfinite(pm.cpu().numpy()).all()


def test_mysn_scl_minsum_fast_is_exact_vs_oracle(pa):
    """Fast-SCL with the min-sum f has no transcendental in the tree: bits must be identical."""
    from polar_amd import _lib, ops
    for (k, n) in ((32, 64), (128, 256), (512, 1024)):
        fp = pa.reference_frozen_pos(k, n).numpy()
        rng = np.random.default_rng(n)
        llr = (rng.standard_normal((24, n)) * 2 + 1).astype(np.float32)
        want, wpm = oracle.scl_decode_mysn(llr, fp, 8, fast_scl=True, exact_f=False)
        plan = _lib.Plan(n, pa.frozen_mask(fp, n), 8, _lib.PL_F_MINSUM, flags=_lib.PL_PLAN_FAST_SCL)
        got, pm = ops.scl_decode(plan, torch.from_numpy(llr).cuda(), return_pm=True)
        assert np.array_equal(got.cpu().numpy(), want), (k, n)
        assert np.abs(pm.cpu().numpy() - wpm).max() < 1e-9


@pytest.mark.parametrize("k", [0, 1, 2])
def test_mysn_scl_fast_pruned_root_vs_oracle(pa, k):
    """Fast-SCL on codes whose root is itself pruned (k = 0: rate-0 root, k = 1: repetition root;
    k = 2: pruned children of the root), where a node sum spans the whole codeword."""
    from polar_amd import _lib, ops
    for n in (32, 256):
        fp = np.arange(n - k) if k < 2 else np.setdiff1d(np.arange(n), [n // 2 - 1, n - 1])
        rng = np.random.default_rng(n + k)
        llr = (rng.standard_normal((29, n)) * 2 + 0.5).astype(np.float32)
        want, wpm = oracle.scl_decode_mysn(llr, fp, 4, fast_scl=True, exact_f=False)
        plan = _lib.Plan(n, pa.frozen_mask(fp, n), 4, _lib.PL_F_MINSUM, flags=_lib.PL_PLAN_FAST_SCL)
        got, pm = ops.scl_decode(plan, torch.from_numpy(llr).cuda(), return_pm=True)
        assert np.array_equal(got.cpu().numpy(), want), (k, n)
        assert np.abs(pm.cpu().numpy() - wpm).max() < 1e-9, (k, n)


def test_mysn_scl_crc_pick_vs_oracle(pa):
    """CRC-aided pick on CRC-carrying codewords: exact vs the oracle's pick (min-sum f, no
    transcendental differences), and the CRC raises the block success rate."""
    from polar_amd import _lib, ops
    k, n, L = 128, 256, 8
    fp = pa.reference_frozen_pos(k, n).numpy()
    info = np.setdiff1d(np.arange(n), fp)
    rng = np.random.default_rng(9)
    u = oracle.crc_encode(rng.integers(0, 2, (200, k - 24)).astype(np.float32), "CRC24C")
    cw = oracle.polar_encode(u, fp, n)
    llr = ((2 * cw - 1) * 1.6 + rng.standard_normal(cw.shape) * 1.5).astype(np.float32)
    want, wpm = oracle.scl_decode_mysn(llr, fp, L, fast_scl=True, exact_f=False, crc="CRC24C")
    plan = _lib.Plan(n, pa.frozen_mask(fp, n), L, _lib.PL_F_MINSUM, flags=_lib.PL_PLAN_FAST_SCL)
    from polar_amd.mysn import crc_params
    plan.set_crc(*crc_params("CRC24C"))
    got, pm = ops.scl_decode(plan, torch.from_numpy(llr).cuda(), return_pm=True)
    got = got.cpu().numpy()
    assert np.array_equal(got, want)
    assert np.abs(pm.cpu().numpy() - wpm).max() < 1e-9
    plain = _lib.Plan(n, pa.frozen_mask(fp, n), L, _lib.PL_F_MINSUM, flags=_lib.PL_PLAN_FAST_SCL)
    nocrc = ops.scl_decode(plain, torch.from_numpy(llr).cuda()).cpu().numpy()
    assert (got == u).all(1).sum() >= (nocrc == u).all(1).sum()


def test_mysn_sc_module(pa):
    from polar_amd import mysn
    d = np.load(os.path.join(GOLDEN, "sc_128_256.npz"))
    dec = mysn.SC_Dec(torch.from_numpy(d["frozen_pos"].astype(np.int64)), 256)
    got = dec(torch.from_numpy(d["llr_awgn2"])).numpy().astype(np.uint8)
    assert got.shape == d["exact_awgn2"].shape
    assert binom_upper_ok(int((got != d["exact_awgn2"]).any(1).sum()), len(got), P0_SC)


@pytest.mark.parametrize("kernel", ["subtree", "generic"])
@pytest.mark.parametrize("fast", [True, False])
@pytest.mark.parametrize("L,lmax", [(4, 7.5), (8, 7.5), (8, 300.0)])
def test_mysn_scl_crc_llr_max_vs_oracle(pa, kernel, fast, L, lmax):
    """llr_max != 30 (my_sn dec.py:213 self._llr_max): it clips f and the metric terms, sets the
    dead-path metric (:420-422) and the CRC penalty llr_max*k (:517).  Min-sum f: bit-exact and
    metrics to 1e-9 against the oracle run with the same llr_max, on both SCL kernels.  At L = 8 the
    subtree kernel selects by the speculative push (scl_tree_kernel.hip PL_SCL_SPEC), whose key
    covers metrics in [2^-44, 2^20): llr_max = 300 makes metrics far below 2^-44 (softplus(-300) ~
    5e-131), outside the key's range, where only the order check and the 64-bit re-rank keep the
    selection exact."""
    from polar_amd import _lib, ops
    from polar_amd.mysn import crc_params
    k, n = 128, 256
    fp = pa.reference_frozen_pos(k, n).numpy()
    rng = np.random.default_rng(17)
    u = oracle.crc_encode(rng.integers(0, 2, (160, k - 11)).astype(np.float32), "CRC11")
    cw = oracle.polar_encode(u, fp, n)
    llr = ((2 * cw - 1) * 2.5 + rng.standard_normal(cw.shape) * 3.0).astype(np.float32)
    want, wpm = oracle.scl_decode_mysn(llr, fp, L, fast_scl=fast, exact_f=False, crc="CRC11", llr_max=lmax)
    flags = (_lib.PL_PLAN_FAST_SCL if fast else 0) | (_lib.PL_PLAN_GENERIC if kernel == "generic" else 0)
    plan = _lib.Plan(n, pa.frozen_mask(fp, n), L, _lib.PL_F_MINSUM, llr_max=lmax, flags=flags)
    assert plan.kernel()[0] == ("scl_subtree" if kernel == "subtree" else "generic")
    plan.set_crc(*crc_params("CRC11"))
    got, pm = ops.scl_decode(plan, torch.from_numpy(llr).cuda(), return_pm=True)
    assert np.array_equal(got.cpu().numpy(), want)
    assert np.abs(pm.cpu().numpy() - wpm).max() < 1e-9
    # the penalty really is llr_max*k: some row failed its CRC and carries it
    assert (wpm.max(1) >= lmax * k).any()


@pytest.mark.parametrize("L", [2, 4, 8, 16])
@pytest.mark.parametrize("fast", [False, True])
def test_scl_n2048_vs_oracle(pa, L, fast):
    """n = 2048 list decoding (generic kernel, list state in LDS up to L = 16): min-sum f,
    bit-exact and metrics to 1e-9 against the oracle (x_run semantics without fast-SCL, my_sn
    fast-SCL semantics with it)."""
    from polar_amd import _lib, ops
    n, k = 2048, 1024
    fp = pa.reference_frozen_pos(k, n).numpy()
    rng = np.random.default_rng(L + 3 * fast)
    bs = 6 if L >= 8 else 12
    u = rng.integers(0, 2, (bs, k)).astype(np.float32)
    cw = oracle.polar_encode(u, fp, n)
    llr = ((2 * cw - 1) * 1.8 + rng.standard_normal(cw.shape) * 1.3).astype(np.float32)
    llr[:, ::13] = np.round(llr[:, ::13])
    if fast:
        want, wpm = oracle.scl_decode_mysn(llr, fp, L, fast_scl=True, exact_f=False)
    else:
        want, wpm = oracle.scl_decode(llr, fp, L, lazy=True)
    plan = _lib.Plan(n, pa.frozen_mask(fp, n), L, _lib.PL_F_MINSUM, flags=_lib.PL_PLAN_FAST_SCL if fast else 0)
    assert plan.kernel()[0] == "generic"
    got, pm = ops.scl_decode(plan, torch.from_numpy(llr).cuda(), return_pm=True)
    assert np.array_equal(got.cpu().numpy(), want)
    assert np.abs(pm.cpu().numpy() - wpm).max() < 1e-9


def test_scl_n2048_module_and_limits(pa):
    """The x_run SCL_Dec drop-in decodes n = 2048 (L <= 16) and rejects L = 32 at construction."""
    n, k = 2048, 1024
    fp = pa.reference_frozen_pos(k, n)
    dec = pa.SCL_Dec(fp, n, list_size=4)
    rng = np.random.default_rng(5)
    x = torch.from_numpy((rng.standard_normal((3, n)) * 2).astype(np.float32))
    want, wpm = oracle.scl_decode(x.numpy(), fp.numpy(), 4, lazy=True)
    assert np.array_equal(dec(x).numpy(), want)
    assert np.abs(dec.msg_pm - wpm).max() < 1e-9
    with pytest.raises(ValueError, match="list_size"):
        pa.SCL_Dec(fp, n, list_size=32)


@pytest.mark.parametrize("n,k,fast", [(1024, 512, True), (1024, 512, False), (512, 256, True), (256, 128, True)])
def test_exact_scl_chain_cache_is_transparent(pa, n, k, fast):
    """The exact-f subtree kernel's workspace caches (leftmost chain, four-outcome tables) change no
    bit and no metric: decoding with the workspace equals decoding with NULL (both recomputed in
    every virtual pass), including a tail wave (bs not a multiple of the codewords per wave)."""
    import ctypes

    from polar_amd import _lib, ops
    fp = pa.reference_frozen_pos(k, n).numpy()
    flags = _lib.PL_PLAN_FAST_SCL if fast else 0
    plan = _lib.Plan(n, pa.frozen_mask(fp, n), 8, _lib.PL_F_EXACT, flags=flags)
    bs = 67
    v = plan_v(n)  # per codeword: the leftmost chain, then the four-outcome tables (scl_tree_kernel.hip)
    per_cw = (n - (n >> v)) + (2 * n - 4 * (n >> v) if v >= 2 else 0)
    assert int(_lib.lib().pl_scl_workspace_size(plan.handle, bs)) == 68 * per_cw * 8
    g = torch.Generator(device="cuda").manual_seed(n + fast)
    llr = (torch.randn((bs, n), device="cuda", generator=g) * 2.0 + 0.8).contiguous()
    bits, pm = ops.scl_decode(plan, llr, return_pm=True)
    out = torch.empty((bs, k), device="cuda")
    pm0 = torch.empty((bs, 16), device="cuda", dtype=torch.float64)
    L = _lib.lib()
    _lib.check(L.pl_scl_decode(plan.handle, ctypes.c_void_p(llr.data_ptr()), bs, ctypes.c_void_p(out.data_ptr()),
                               _lib.PL_OUT_F32, ctypes.c_void_p(pm0.data_ptr()), None, 0,
                               _lib.current_stream_ptr(llr.device)), "pl_scl_decode")
    torch.cuda.synchronize()
    assert torch.equal(bits, out)
    assert torch.equal(pm, pm0)


def plan_v(n):
    """Virtual stages of the subtree kernel at code length n (scl_tree_kernel.hip pick_v)."""
    S = n.bit_length() - 1
    v = min(S - 1 - 4, 4)
    if v == 4 and S != 10:
        v = 3
    return max(v, 0)


def test_exact_scl_workspace_chunks(pa):
    """A batch above the workspace chunk (16384 codewords) runs as consecutive launches over one
    chunk-sized workspace: the same bits and metrics as one launch without the workspace, and the
    workspace size stops growing with the batch."""
    import ctypes

    from polar_amd import _lib, ops
    n, k = 256, 128
    fp = pa.reference_frozen_pos(k, n).numpy()
    plan = _lib.Plan(n, pa.frozen_mask(fp, n), 8, _lib.PL_F_EXACT, flags=_lib.PL_PLAN_FAST_SCL)
    L = _lib.lib()
    assert int(L.pl_scl_workspace_size(plan.handle, 16384)) == int(L.pl_scl_workspace_size(plan.handle, 40000))
    bs = 16384 + 37
    g = torch.Generator(device="cuda").manual_seed(11)
    llr = (torch.randn((bs, n), device="cuda", generator=g) * 2.0 + 0.8).contiguous()
    bits, pm = ops.scl_decode(plan, llr, return_pm=True)
    out = torch.empty((bs, k), device="cuda")
    pm0 = torch.empty((bs, 16), device="cuda", dtype=torch.float64)
    _lib.check(L.pl_scl_decode(plan.handle, ctypes.c_void_p(llr.data_ptr()), bs, ctypes.c_void_p(out.data_ptr()),
                               _lib.PL_OUT_F32, ctypes.c_void_p(pm0.data_ptr()), None, 0,
                               _lib.current_stream_ptr(llr.device)), "pl_scl_decode")
    torch.cuda.synchronize()
    assert torch.equal(bits, out)
    assert torch.equal(pm, pm0)
