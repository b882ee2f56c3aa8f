"""GPU tests of the whole Monte-Carlo iteration inside the specialised SC kernel (pl_sc_sim_count,
sc_static.h OUT_SIM): System_AWGN_model.forward (awgn_model.py:33-44) generated in the decoder's
lane layout, decoded, and counted as my_sn/sim.py:84-100 does.

  * counters: exactly count_errors / count_block_errors (pl_count_errors) of pl_sc_decode's output
    on the kernel's own dumped logits against its dumped information bits -- for the bench code at
    1, 2, 3 dB, ragged batches, n = 64 ... 1024, and the rate-0 / rate-1 root halves;
  * information bits: bit-exact against a numpy restatement of the stream convention (Philox
    restated in polar_amd.channel.philox4x32_10, pinned by the Random123 known answers);
  * the encoder inside the kernel: the noiseless part of every logit has the sign of the code bit
    of polar_encode(u) (GpuEncoder), and the standardised noise is N(0, 1) (statistical, 4e6 draws);
  * row0 shifts the stream rows (a rank's shard); dumps do not change the counters;
  * FusedAWGN.error_counts and sim_ber take this path; plans without 64 channel slots per lane
    report PL_ENOTSUP and FusedAWGN falls back to the two-kernel path.
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


def _spec(pa, fp, n, f_mode=0):
    from polar_amd import _lib
    spec = _lib.Plan(n, pa.frozen_mask(fp, n), 1, f_mode, flags=_lib.PL_PLAN_CACHE_ONLY)
    assert spec.kernel()[0] == "specialized", spec.kernel()
    return spec


def _no(ebno, k, n):
    from polar_amd.channel import ebnodb2no
    return float(ebnodb2no(float(ebno), 2, k / n))


def _check_counts(pa, spec, bs, no, seed, it, row0=0):
    from polar_amd import ops
    cnt, u, llr = ops.sc_sim_count(spec, bs, no, seed, it, row0, dump=True)
    want = ops.count_errors(u, ops.sc_decode(spec, llr))
    assert cnt.tolist() == want.tolist(), (spec.n, spec.k, bs, no)
    plain = ops.sc_sim_count(spec, bs, no, seed, it, row0)
    assert plain.tolist() == cnt.tolist()
    return cnt, u, llr


@pytest.mark.parametrize("ebno", [1.0, 2.0, 3.0])
def test_counts_equal_decode_of_dump_bench_code(pa, ebno):
    k, n = 512, 1024
    spec = _spec(pa, pa.reference_frozen_pos(k, n).numpy(), n)
    cnt, _, _ = _check_counts(pa, spec, 8192, _no(ebno, k, n), 42, 3)
    assert 0 < int(cnt[1]) <= 8192 or ebno >= 3.0


@pytest.mark.parametrize("k,n,bs", [(512, 1024, 1001), (256, 512, 777), (128, 256, 4096), (32, 64, 100),
                                    (16, 64, 65), (256, 1024, 300), (1023, 1024, 129), (1, 1024, 257),
                                    (63, 64, 1)])
def test_counts_ragged_and_other_codes(pa, k, n, bs):
    spec = _spec(pa, pa.reference_frozen_pos(k, n).numpy(), n)
    _check_counts(pa, spec, bs, _no(1.5, k, n), 5, 1)


def test_root_half_codes(pa):
    from polar_amd.build import root_half_codes
    for _, mask in root_half_codes():
        fp = np.flatnonzero(mask)
        spec = _spec(pa, fp, 1024)
        _check_counts(pa, spec, 300, _no(1.0, 1024 - len(fp), 1024), 9, 0)


def _ref_info_bits(fp, n, k, seed, it, rows):
    """Information bits of stream rows `rows` in position order, restated with numpy Philox."""
    from polar_amd.channel import philox4x32_10
    G = n // 64
    mask = np.ones(n, dtype=bool)
    mask[fp] = False  # information positions
    rows = np.asarray(rows, dtype=np.int64)
    u = np.zeros((len(rows), n), dtype=np.uint8)
    for r in range(G):
        ctr = np.zeros((len(rows), 4), dtype=np.uint64)
        ctr[:, 0] = rows & 0xFFFFFFFF
        ctr[:, 1] = rows >> 32
        ctr[:, 2] = it
        ctr[:, 3] = 0x40000000 | (r >> 1)
        key = np.zeros((len(rows), 2), dtype=np.uint64)
        key[:, 0] = seed & 0xFFFFFFFF
        key[:, 1] = seed >> 32
        blk = philox4x32_10(ctr, key)
        for j in range(64):
            w = blk[:, 2 * (r & 1) + j // 32]
            u[:, r + G * j] = (w >> np.uint32(j % 32)) & 1
    u[:, ~mask] = 0
    return u[:, mask]


@pytest.mark.parametrize("k,n", [(512, 1024), (128, 256), (32, 64)])
def test_information_bits_stream(pa, k, n):
    from polar_amd import ops
    fp = pa.reference_frozen_pos(k, n).numpy()
    spec = _spec(pa, fp, n)
    seed, it = 0x1234_5678_9ABC, 7
    _, u, _ = ops.sc_sim_count(spec, 200, _no(2.0, k, n), seed, it, 13, dump=True)
    want = _ref_info_bits(fp, n, k, seed, it, np.arange(13, 213))
    assert np.array_equal(u.cpu().numpy().astype(np.uint8), want)


def test_encoder_and_noise_statistics(pa):
    from polar_amd import channel, ops
    k, n = 512, 1024
    fp = pa.reference_frozen_pos(k, n)
    spec = _spec(pa, fp.numpy(), n)
    no = _no(2.0, k, n)
    _, u, llr = ops.sc_sim_count(spec, 4096, no, 11, 2, dump=True)
    cw = channel.GpuEncoder(fp, n)(u)
    z = (llr - (2.0 / no) * (2 * cw - 1)) * (no ** 0.5) / 2  # standardised noise
    assert abs(float(z.mean())) < 3e-3 and abs(float(z.std()) - 1.0) < 3e-3
    assert abs(float((z[:, :-1] * z[:, 1:]).mean())) < 3e-3  # neighbouring positions uncorrelated
    assert abs(float((z[:, :-16] * z[:, 16:]).mean())) < 3e-3  # slots of one lane uncorrelated
    zz = z.flatten()
    assert abs(float((zz.abs() > 3).float().mean()) - 2.6998e-3) < 3e-4  # two-sided 3-sigma tail
    assert 0.45 < float(u.mean()) < 0.55


def test_row_offset_selects_stream_rows(pa):
    from polar_amd import ops
    k, n = 128, 256
    spec = _spec(pa, pa.reference_frozen_pos(k, n).numpy(), n)
    no = _no(2.0, k, n)
    _, u0, l0 = ops.sc_sim_count(spec, 40, no, 3, 5, 0, dump=True)
    _, u1, l1 = ops.sc_sim_count(spec, 30, no, 3, 5, 10, dump=True)
    assert torch.equal(u0[10:], u1) and torch.equal(l0[10:], l1)
    _, u2, _ = ops.sc_sim_count(spec, 40, no, 3, 6, 0, dump=True)
    assert not torch.equal(u0, u2)  # the iteration draws a fresh batch


def test_fused_awgn_and_sim_ber_take_this_path(pa):
    from polar_amd import channel, ops, sim
    k, n = 512, 1024
    fp = pa.reference_frozen_pos(k, n)
    dec = pa.SC_Dec(fp, n)
    model = channel.FusedAWGN(n, k, fp, dec, seed=3)
    no = _no(2.0, k, n)
    got = model.error_counts(2048, 2.0)
    want = ops.sc_sim_count(dec.plan(model.device), 2048, no, 3, 0, 0)
    assert model.sim_kernel and got.tolist() == want.tolist()
    ber, bler = sim.sim_ber(model, [1.0, 2.0], 4096, 4, verbose=False, device="cuda")
    assert float(bler[0]) > float(bler[1]) > 0.0


def test_plans_without_the_entry(pa):
    from polar_amd import _lib, channel, ops
    k, n = 512, 1024
    fp = pa.reference_frozen_pos(k, n)
    exact = _spec(pa, fp.numpy(), n, f_mode=1)  # exact-f layout: 128 slots per lane
    with pytest.raises(_lib.PolarLibError) as e:
        ops.sc_sim_count(exact, 64, 0.5, 1, 0)
    assert e.value.code == _lib.PL_ENOTSUP
    gen = _lib.Plan(n, pa.frozen_mask(fp, n), 1, flags=_lib.PL_PLAN_GENERIC)
    with pytest.raises(_lib.PolarLibError):
        ops.sc_sim_count(gen, 64, 0.5, 1, 0)
    # n = 2048 runs 128 slots per lane: FusedAWGN falls back to the two-kernel path
    fp2 = pa.reference_frozen_pos(1024, 2048)
    dec = pa.SC_Dec(fp2, 2048)
    model = channel.FusedAWGN(2048, 1024, fp2, dec, seed=1)
    cnt = model.error_counts(256, 2.0)
    assert cnt is not None and not model.sim_kernel
