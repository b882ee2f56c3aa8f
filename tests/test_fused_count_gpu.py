"""GPU tests of the harness fused into the decoder (pl_awgn_qpsk_llr_bits + pl_sc_decode_count):

  * the packed-bits producer draws the same stream: its logits are bit-identical to
    pl_awgn_qpsk_llr's and its words are the fp32 bit rows packed;
  * pl_sc_decode_count's [bit errors, block errors] equal count_errors / count_block_errors
    (my_sn/sim.py:7-18, via pl_count_errors) of pl_sc_decode's output against the same bits,
    exactly, for the bench code at 1, 2 and 4 dB, ragged batches, k not a multiple of 32, and
    rate-0 / rate-1 root halves (the LDS channel path);
  * sim_ber over FusedAWGN(sim_kernel=False) + SC_Dec takes the fused-count path and its counters
    equal the two-kernel path's for the same seed (the producer-in-kernel path, pl_sc_sim_count,
    is tested in tests/test_sim_kernel_gpu.py);
  * the same for the exact-f (my_sn SC_Dec) specialised kernels at (512,1024) and (128,256);
  * plans on the generic SC kernel report PL_ENOTSUP.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pa():
    import polar_amd
    assert torch.cuda.is_available()
    return polar_amd


def _plans(pa, fp, n, f_mode=0):
    from polar_amd import _lib
    m = pa.frozen_mask(fp, n)
    gen = _lib.Plan(n, m, 1, f_mode, flags=_lib.PL_PLAN_GENERIC)
    spec = _lib.Plan(n, m, 1, f_mode, flags=_lib.PL_PLAN_CACHE_ONLY)
    assert spec.kernel()[0] == "specialized", spec.kernel()
    return gen, spec


def _ebno_no(ebno, k, n):
    from polar_amd.channel import ebnodb2no
    return float(ebnodb2no(float(ebno), 2, k / n))


def test_packed_producer_same_stream(pa):
    from polar_amd import ops
    k, n = 512, 1024
    gen, _ = _plans(pa, pa.reference_frozen_pos(k, n).numpy(), n)
    no = _ebno_no(2.0, k, n)
    u, llr = ops.awgn_qpsk_llr(gen, 1000, no, 7, 3, 11)
    ub, llr2 = ops.awgn_qpsk_llr_bits(gen, 1000, no, 7, 3, 11)
    assert torch.equal(llr, llr2)
    assert torch.equal(ub, ops.pack_bits(u))


def _case(pa, fp, n, bs, ebno, seed, f_mode=0):
    from polar_amd import ops
    k = n - len(fp)
    gen, spec = _plans(pa, fp, n, f_mode)
    ub, llr = ops.awgn_qpsk_llr_bits(gen, bs, _ebno_no(ebno, k, n), seed, 0, 0)
    u, _ = ops.awgn_qpsk_llr(gen, bs, _ebno_no(ebno, k, n), seed, 0, 0)
    want = ops.count_errors(u, ops.sc_decode(spec, llr))
    got = ops.sc_decode_count(spec, llr, ub)
    assert got.tolist() == want.tolist(), (k, n, bs, ebno)
    ops.sc_decode_count(spec, llr, ub, counts=got)  # accumulates
    assert got.tolist() == [2 * v for v in want.tolist()]
    return want


@pytest.mark.parametrize("ebno", [1.0, 2.0, 4.0])
def test_decode_count_equals_decode_then_count_bench_code(pa, ebno):
    w = _case(pa, pa.reference_frozen_pos(512, 1024).numpy(), 1024, 65536, ebno, 42)
    assert w[1] > 0


@pytest.mark.parametrize("k,n,bs", [(512, 1024, 4099), (128, 256, 1000), (32, 64, 257), (48, 64, 333)])
def test_decode_count_ragged_and_k_not_multiple_of_32(pa, k, n, bs):
    from polar_amd import build
    if (k, n) == (48, 64):  # a pre-built random code (build.test_random_codes: log_n 6, rate 0.75)
        rng = np.random.default_rng(6 * 10 + 3)
        fp = np.sort(rng.permutation(n)[: n - k])
        assert any(np.array_equal(np.nonzero(m)[0], fp) for m, fm in build.test_random_codes() if len(m) == n)
    else:
        fp = pa.reference_frozen_pos(k, n).numpy()
    _case(pa, fp, n, bs, 2.0, 5)


@pytest.mark.parametrize("k,n,bs", [(512, 1024, 8195), (128, 256, 4096)])
def test_decode_count_exact_f(pa, k, n, bs):
    """the exact-f specialised kernels (my_sn SC_Dec's f; n >= 128 compiles the decode +
    count entry with the stage-(n/2) VGPR root, PL_SC_ROOT_MODE 1): sc_decode_count equals
    count_errors of the same plan's sc_decode, ragged batch included."""
    w = _case(pa, pa.reference_frozen_pos(k, n).numpy(), n, bs, 2.0, 17, f_mode=1)
    assert w[1] > 0


def test_decode_count_root_half_codes(pa):
    from polar_amd import build
    for name, m in build.root_half_codes():
        if name in ("REP_SPC", "R0_GEN", "GEN_R1"):
            _case(pa, np.nonzero(m)[0], 1024, 2053, 3.0, 9)


def test_sim_ber_fused_equals_two_kernel_path(pa):
    from polar_amd import channel, sim
    k, n = 512, 1024
    fp = pa.reference_frozen_pos(k, n)
    class ForwardOnly:  # the same keyed draws through forward() + pl_count_errors (no error_counts)
        keyed_streams = True

        def __init__(self, m):
            self.m = m

        def __call__(self, batch_size, ebno_db, stream=None):
            return self.m(batch_size, ebno_db, stream=stream)

    counts = []
    for fused in (True, False):
        model = channel.FusedAWGN(n, k, fp, pa.SC_Dec(fp, n), seed=3, sim_kernel=False)
        mc = model if fused else ForwardOnly(model)
        _, _, cnt = sim.sim_ber(mc, [2.5, 3.0, 3.5], 8192, 3, verbose=False, device="cuda", return_counts=True)
        counts.append(cnt)
    assert torch.equal(counts[0], counts[1]), counts


def test_generic_plan_is_not_supported(pa):
    from polar_amd import _lib, ops
    k, n = 512, 1024
    gen, _ = _plans(pa, pa.reference_frozen_pos(k, n).numpy(), n)
    ub, llr = ops.awgn_qpsk_llr_bits(gen, 64, 0.5, 1, 0, 0)
    with pytest.raises(_lib.PolarLibError):
        ops.sc_decode_count(gen, llr, ub)
