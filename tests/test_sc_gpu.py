"""Parity of the HIP SC decoder (libpolar_mi355x.so via the C ABI) with the reference.

  * golden fixtures from the reference (tests/golden/sc_*.npz): bit-exact, min-sum
  * the pinned CPU oracle on seeded random inputs, every supported n: bit-exact
  * full-size (512,1024) x 65536 batch: noiseless encode->decode round trip + oracle on a sample
  * edge cases: bs = 0 / 1 / ragged, k = 0 / n, exact zeros, saturation, uint8 output, CPU input
  * exact-boxplus mode: statistical gate (see tests/test_oracle.py for why)
Both SC kernels are held to the same bar: the code-specialised one (default; pre-built for the
reference codes, compiled with hiprtc at plan time for any other code) and the generic one.
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


@pytest.fixture(scope="module")
def pa():
    import polar_amd
    assert torch.cuda.is_available(), "GPU tests need a ROCm GPU"
    return polar_amd


KINDS = ("specialized", "generic")


def _plan(pa, fp, n, f_mode=0, L=1, kind="specialized"):
    from polar_amd import _lib
    # specialised: only pre-built code objects (build.py), never a compile on the GPU box
    flags = _lib.PL_PLAN_GENERIC if kind == "generic" else _lib.PL_PLAN_CACHE_ONLY
    plan = _lib.Plan(n, pa.frozen_mask(fp, n), L, f_mode, flags=flags)
    assert plan.kernel()[0] == kind, plan.kernel()
    return plan


def _sets(d):
    return [k[4:] for k in d.files if k.startswith("llr_")]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "sc_*.npz"))), ids=os.path.basename)
def test_sc_golden_bit_exact(pa, path, kind):
    d = np.load(path)
    n = int(d["n"])
    plan = _plan(pa, d["frozen_pos"], n, kind=kind)
    for name in _sets(d):
        x = torch.from_numpy(d["llr_" + name]).cuda()
        bits = pa.ops.sc_decode(plan, x)
        torch.cuda.synchronize()
        got = bits.cpu().numpy().astype(np.uint8)
        assert np.array_equal(got, d["bits_" + name]), f"{name}: {int((got != d['bits_' + name]).any(1).sum())} rows differ"


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("log_n", list(range(1, 12)))
@pytest.mark.parametrize("rate", [0.25, 0.5, 0.75])
def test_sc_random_vs_oracle(pa, log_n, rate, kind):
    """Arbitrary frozen sets at every n = 2 ... 2048 and three rates, both SC kernels (the
    specialised ones are pre-built by build.test_random_codes, so nothing compiles on the box)."""
    n = 1 << log_n
    rng = np.random.default_rng(log_n * 10 + int(rate * 4))
    k = max(1, int(n * rate))
    fp = np.sort(rng.permutation(n)[: n - k])  # arbitrary frozen set: exercises all node patterns
    bs = 300 + log_n  # ragged: not a multiple of the per-block codeword count
    llr = (rng.standard_normal((bs, n)) * 3).astype(np.float32)
    llr[rng.random((bs, n)) < 0.05] = 0.0
    want = oracle.sc_decode(llr, fp)
    plan = _plan(pa, fp, n, kind=kind)
    got = pa.ops.sc_decode(plan, torch.from_numpy(llr).cuda()).cpu().numpy()
    assert np.array_equal(got, want)
    got8 = pa.ops.sc_decode(plan, torch.from_numpy(llr).cuda(), out_dtype=torch.uint8).cpu().numpy()
    assert np.array_equal(got8, want.astype(np.uint8))


@pytest.mark.parametrize("kind", KINDS)
def test_sc_reference_frozen_all_shapes(pa, kind):
    fs = np.load(os.path.join(GOLDEN, "frozen_sets.npz"))
    rng = np.random.default_rng(5)
    for key in fs.files:
        k, n = (int(v[1:]) for v in key.split("_"))
        if n > 2048:
            continue
        fp = fs[key]
        llr = (rng.standard_normal((129, n)) * 2 + 0.5).astype(np.float32)
        got = pa.ops.sc_decode(_plan(pa, fp, n, kind=kind), torch.from_numpy(llr).cuda()).cpu().numpy()
        assert np.array_equal(got, oracle.sc_decode(llr, fp)), key
        # ties, exact zeros and saturation: every shortcut's fallback path
        t = (np.round(rng.standard_normal((129, n)) * 2) * 0.5).astype(np.float32)
        t[:, ::5] *= 100.0
        got = pa.ops.sc_decode(_plan(pa, fp, n, kind=kind), torch.from_numpy(t).cuda()).cpu().numpy()
        assert np.array_equal(got, oracle.sc_decode(t, fp)), key


@pytest.mark.parametrize("kind", KINDS)
def test_sc_root_half_types(pa, kind):
    """n = 1024 codes whose root halves are rate-0 / rate-1 / repetition / SPC / a general node:
    every branch of the virtual root (and of the LDS channel half, sc_static.h Ch).  Pre-built by
    build() (polar_amd.build.root_half_codes), so the specialised kernels never compile here."""
    from polar_amd import _lib, build
    rng = np.random.default_rng(11)
    llr = (rng.standard_normal((257, 1024)) * 2.5).astype(np.float32)
    llr[:, ::9] = np.round(llr[:, ::9])  # exact zeros and ties
    llr[:5] *= 40.0  # saturation
    x = torch.from_numpy(llr).cuda()
    for name, m in build.root_half_codes():
        fp = np.nonzero(m)[0]
        flags = _lib.PL_PLAN_GENERIC if kind == "generic" else _lib.PL_PLAN_CACHE_ONLY
        plan = _lib.Plan(1024, m, 1, 0, flags=flags)
        assert plan.kernel()[0] == kind, (name, plan.kernel())
        got = pa.ops.sc_decode(plan, x).cpu().numpy()
        assert np.array_equal(got, oracle.sc_decode(llr, fp)), name


def test_sc_full_batch_roundtrip_and_sample(pa):
    """(512,1024) at the bench batch: size-independent property + oracle on a sample."""
    fp = pa.reference_frozen_pos(512, 1024).numpy()
    plan = _plan(pa, fp, 1024)
    g = torch.Generator(device="cuda").manual_seed(3)
    bs = 65536
    u = torch.randint(0, 2, (bs, 512), device="cuda", generator=g).to(torch.float32)
    cw = pa.ops.polar_encode(plan, u)
    logits = (2.0 * cw - 1.0) * 3.0  # noiseless: logits > 0 <=> bit 1
    assert torch.equal(pa.ops.sc_decode(plan, logits), u)
    noisy = logits + torch.randn(logits.shape, device="cuda", generator=g) * 2.0
    got = pa.ops.sc_decode(plan, noisy)
    idx = torch.randint(0, bs, (512,), device="cuda", generator=g)
    sample = noisy[idx].cpu().numpy()
    assert np.array_equal(got[idx].cpu().numpy(), oracle.sc_decode(sample, fp))


def test_sc_edge_cases(pa):
    n = 64
    fp = pa.reference_frozen_pos(32, 64).numpy()
    plan = _plan(pa, fp, n)
    empty = pa.ops.sc_decode(plan, torch.empty((0, n), device="cuda"))
    assert empty.shape == (0, 32)
    one = (torch.randn(1, n) * 2).cuda()
    assert np.array_equal(pa.ops.sc_decode(plan, one).cpu().numpy(), oracle.sc_decode(one.cpu().numpy(), fp))
    # all frozen (k = 0) and nothing frozen (k = n)
    p0 = _plan(pa, np.arange(n), n)
    assert pa.ops.sc_decode(p0, one).shape == (1, 0)
    pn = _plan(pa, np.array([], dtype=np.int64), n)
    x = (torch.randn(77, n) * 2)
    x[:, ::7] = 0.0
    assert np.array_equal(pa.ops.sc_decode(pn, x.cuda()).cpu().numpy(), oracle.sc_decode(x.numpy(), []))
    # saturation far beyond the +-30 clip and signed zeros
    y = (torch.randn(200, n) * 500)
    y[:, 3] = -0.0
    assert np.array_equal(pa.ops.sc_decode(plan, y.cuda()).cpu().numpy(), oracle.sc_decode(y.numpy(), fp))
    with pytest.raises(ValueError):
        pa.ops.sc_decode(plan, torch.zeros((4, n + 1), device="cuda"))


def test_sc_dropin_module_matches_reference_contract(pa):
    d = np.load(os.path.join(GOLDEN, "sc_32_64.npz"))
    fp = torch.from_numpy(d["frozen_pos"].astype(np.int64))
    dec = pa.SC_Dec(fp, 64)
    x = torch.from_numpy(d["llr_rand"])  # CPU tensor, as the reference harness passes
    out = dec(x)
    assert out.device.type == "cpu" and out.dtype == torch.float32 and out.shape == (x.shape[0], 32)
    assert np.array_equal(out.numpy().astype(np.uint8), d["bits_rand"])
    out3 = dec(x.reshape(4, -1, 64))  # [..., n] input -> [-1, ..., k] output (polar_sc.py:129-132)
    assert out3.shape == (4, x.shape[0] // 4, 32)
    with pytest.raises(AssertionError):
        dec(torch.zeros(64))
    with pytest.raises(AssertionError):
        dec(torch.zeros(3, 63))
    assert dec(x.cuda()).device.type == "cuda"


@pytest.mark.parametrize("kind", KINDS)
def test_sc_exact_mode_statistical(pa, kind):
    """Exact-boxplus SC (my_sn dec.py:39-43) on the golden shapes' AWGN and saturation sets:
    row mismatches against the reference within the one-sided binomial gate at rate 1e-4
    (the statistical-power version is tests/test_exactf_gpu.py).  The
    random N(0, 4) sets are left out: there the cancellation in f decides ~4 % of rows by the
    last ulp even between two correctly rounded libms (the C oracle: 59 of 1440)."""
    sys.path.insert(0, GOLDEN)
    from exactf_recipe import binom_upper_ok
    mism = rows = 0
    for path in sorted(glob.glob(os.path.join(GOLDEN, "sc_*.npz"))):
        d = np.load(path)
        plan = _plan(pa, d["frozen_pos"], int(d["n"]), f_mode=1, kind=kind)
        for name in _sets(d):
            if not (name.startswith("awgn") or name == "sat"):
                continue
            got = pa.ops.sc_decode(plan, torch.from_numpy(d["llr_" + name]).cuda()).cpu().numpy().astype(np.uint8)
            mism += int((got != d["exact_" + name]).any(1).sum())
            rows += len(got)
    assert rows >= 2000 and binom_upper_ok(mism, rows, 1e-4), (mism, rows)


@pytest.mark.parametrize("kind", KINDS)
def test_sc_exact_large_llr_max_overflows_like_the_reference(pa, kind):
    """Exact-f SC plans with llr_max > 43: xc + yc then leaves exp's finite range,
    log(1 + exp(xc + yc)) must be +inf as in torch (log(inf) = inf), not NaN, and the decisions
    follow.  n = 2 and 4, every frozen pattern, llr_max 60 and 80 (< 88.7, so exp(llr_max) and
    exp(x) + exp(y) stay finite and f is never inf - inf; f can only overflow to +inf, and g never
    adds two infinities of opposite sign at n <= 4): neither decoder reaches a NaN and the oracle
    (glibc expf/logf, same llr_max) is exact.  Inputs of magnitude 30-80: most f overflow.  (Above
    88.7 the reference itself produces inf - inf = NaN LLRs and NaN output bits.)"""
    from polar_amd import _lib
    g = np.random.default_rng(7)
    for lmax in (60.0, 80.0):
        for n in (2, 4):
            x = (g.uniform(30.0, lmax, (512, n)) * g.choice([-1.0, 1.0], (512, n))).astype(np.float32)
            x[:16] = np.float32(lmax) * np.sign(x[:16])  # saturated rows
            for code in range(1, 1 << n):  # k >= 1
                mask = np.array([(code >> i) & 1 for i in range(n)], dtype=np.uint8) ^ 1
                fp = np.flatnonzero(mask)
                flags = _lib.PL_PLAN_GENERIC if kind == "generic" else _lib.PL_PLAN_CACHE_ONLY
                plan = _lib.Plan(n, mask, 1, _lib.PL_F_EXACT, lmax, flags=flags)
                assert plan.kernel()[0] == kind, plan.kernel()
                got = pa.ops.sc_decode(plan, torch.from_numpy(x).cuda()).cpu().numpy()
                want = oracle.sc_decode(x, fp, f_mode=1, llr_max=lmax)
                assert np.array_equal(got, want), (lmax, n, code, int((got != want).any(1).sum()))


def test_sc_specialized_jit_for_an_arbitrary_code(pa, tmp_path, monkeypatch):
    """A code with no pre-built kernel: compiled by hiprtc at plan creation, cached, bit-exact."""
    from polar_amd import _lib
    monkeypatch.setenv("PL_KERNEL_CACHE", str(tmp_path))
    rng = np.random.default_rng(77)
    n = 1024
    fp = np.sort(rng.permutation(n)[:400])
    plan = _lib.Plan(n, pa.frozen_mask(fp, n), 1, 0)
    kind, path = plan.kernel()
    assert kind == "specialized" and path.startswith(str(tmp_path)), (kind, path)
    llr = (rng.standard_normal((4099, n)) * 2.5).astype(np.float32)
    llr[:, ::11] = np.round(llr[:, ::11])
    got = pa.ops.sc_decode(plan, torch.from_numpy(llr).cuda()).cpu().numpy()
    assert np.array_equal(got, oracle.sc_decode(llr, fp))
    # second plan for the same code: cache hit, same file; cache-only plans never compile
    assert _lib.Plan(n, pa.frozen_mask(fp, n), 1, 0, flags=_lib.PL_PLAN_CACHE_ONLY).kernel() == (kind, path)
    fp2 = np.sort(rng.permutation(n)[:401])
    assert _lib.Plan(n, pa.frozen_mask(fp2, n), 1, 0, flags=_lib.PL_PLAN_CACHE_ONLY).kernel()[0] == "generic"


def test_plans_are_device_bound(pa):
    """Plans record their device (pl_plan_device); modules keep one plan per device.  With two or
    more GPUs: a plan refuses a stream of another device (PL_EINVAL -> ValueError), and a module
    decodes on a non-current device with that device's own plan."""
    import polar_amd
    from polar_amd import _lib, ops
    fp = polar_amd.reference_frozen_pos(128, 256)
    p0 = _lib.Plan(256, pa.frozen_mask(fp.numpy(), 256), 1, 0, device=0)
    assert p0.device == torch.device("cuda", 0)
    dec = polar_amd.SC_Dec(fp, 256)
    x = torch.randn((40, 256), generator=torch.Generator().manual_seed(3)) * 2
    want = oracle.sc_decode(x.numpy(), fp.numpy())
    assert np.array_equal(dec(x).numpy(), want)
    assert np.array_equal(dec(x.cuda(0)).cpu().numpy(), want)
    assert dec.plan(0).device == torch.device("cuda", 0)
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU: cross-device checks need two")
    with torch.cuda.device(0):
        got = dec(x.cuda(1))
    assert got.device == torch.device("cuda", 1)
    assert np.array_equal(got.cpu().numpy(), want)
    assert dec.plan(1).device == torch.device("cuda", 1)
    with pytest.raises(ValueError, match="device-bound"):
        ops.sc_decode(p0, x.cuda(1))


def test_launch_graph_replays_bit_exact(pa):
    """ops.LaunchGraph: back-to-back SC (specialised, configs[1] shape) and SCL (L = 8, with its
    workspace) decodes of resident batches captured into one HIP graph; each replay leaves the
    same bits as the eager calls, also after the inputs are refilled in place."""
    from polar_amd import _lib, ops
    g = np.random.default_rng(11)
    fp = pa.reference_frozen_pos(128, 256)
    plan = _plan(pa, fp, 256)
    llr = torch.from_numpy(g.normal(0.0, 2.0, (4096, 256)).astype(np.float32)).cuda()
    out = torch.empty((4096, 128), device="cuda")
    lg = ops.LaunchGraph(lambda: ops.sc_decode(plan, llr, out=out), 3)
    for _ in range(2):
        out.zero_()
        lg.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ops.sc_decode(plan, llr)), "SC graph replay"
        llr.copy_(torch.from_numpy(g.normal(0.0, 2.0, (4096, 256)).astype(np.float32)))
    fp8 = pa.reference_frozen_pos(64, 128)
    p8 = _lib.Plan(128, pa.frozen_mask(fp8, 128), 8, 0)
    x = torch.from_numpy(g.normal(0.0, 2.0, (256, 128)).astype(np.float32)).cuda()
    o8 = torch.empty((256, 64), device="cuda")
    ws = ops.scl_workspace(p8, 256, x.device)
    lg8 = ops.LaunchGraph(lambda: ops.scl_decode(p8, x, out=o8, workspace=ws), 2)
    o8.zero_()
    lg8.replay()
    torch.cuda.synchronize()
    assert torch.equal(o8, ops.scl_decode(p8, x)), "SCL graph replay"


def test_launch_graph_keeps_its_plan_and_buffers_alive(pa):
    """the graph owns fn, so once the function that captured it has returned -- its
    plan, input and workspace referenced by nothing but the closure -- and the garbage collector
    has run, replay() is still valid: the replay writes the eager decode's bits into the buffer it
    captured."""
    import gc
    import weakref
    from polar_amd import _lib, ops

    def capture():
        g = np.random.default_rng(12)
        fp = pa.reference_frozen_pos(64, 128)
        plan = _lib.Plan(128, pa.frozen_mask(fp, 128), 8, 0)
        x = torch.from_numpy(g.normal(0.0, 2.0, (256, 128)).astype(np.float32)).cuda()
        want = ops.scl_decode(plan, x)
        out = torch.zeros((256, 64), device="cuda")
        ws = ops.scl_workspace(plan, 256, x.device)
        lg = ops.LaunchGraph(lambda: ops.scl_decode(plan, x, out=out, workspace=ws), 2)
        return lg, out, want, weakref.ref(plan)

    lg, probe, want, ref_plan = capture()
    gc.collect()
    assert ref_plan() is not None, "the graph must keep its plan alive"
    probe.zero_()
    lg.replay()
    torch.cuda.synchronize()
    assert torch.equal(probe, want)
    del lg
    gc.collect()
    assert ref_plan() is None, "the plan is released with the graph"


def test_shader_clock_probe(pa):
    """pl_clock_probe: s_memtime / s_memrealtime of one wave's chain gives a plausible MI355X shader
    clock (bench.py records it around its timed region)."""
    from polar_amd import ops
    ghz = ops.shader_clock_ghz()
    assert 0.5 < ghz < 3.0, ghz


def test_sc_exact_wide_range_code_object(pa, tmp_path, monkeypatch):
    """Exact-f plans get one code object per llr_max range (exactf.h PL_EXF_RANGE): llr_max 30 and
    60 on the same code load different specialised kernels, the llr_max = 60 one compiled on demand
    (out of process, into an empty cache); each equals the generic kernel (which tests the range
    in every f) bit for bit."""
    from polar_amd import _lib, ops
    monkeypatch.setenv("PL_KERNEL_CACHE", str(tmp_path))
    g = np.random.default_rng(5)
    n = 64
    fp = np.sort(g.permutation(n)[:28])
    mask = pa.frozen_mask(fp, n)
    x = torch.from_numpy((g.normal(0.0, 6.0, (1024, n))).astype(np.float32)).cuda()
    paths = []
    for lmax in (30.0, 60.0):
        p = _lib.Plan(n, mask, 1, _lib.PL_F_EXACT, lmax)
        kind, path = p.kernel()
        assert kind == "specialized", (lmax, kind)
        paths.append(path)
        gen = _lib.Plan(n, mask, 1, _lib.PL_F_EXACT, lmax, flags=_lib.PL_PLAN_GENERIC)
        assert torch.equal(ops.sc_decode(p, x), ops.sc_decode(gen, x)), lmax
    assert paths[0] != paths[1], paths
