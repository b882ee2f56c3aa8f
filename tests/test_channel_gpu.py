"""GPU tests of the fused Monte-Carlo producer and error counter (csrc/channel_kernel.hip):

  * information bits bit-exact against the numpy Philox restatement (tests/test_channel.py pins it
    to the Random123 known answers);
  * at very high SNR the logits' signs are exactly the codewords of the oracle's encoder (bits,
    encoder and Gray mapping exact);
  * logits have the reference demapper's distribution at 2 dB (mean (2/no)(2c-1), variance 4/no);
  * SC BLER through FusedAWGN matches the reference's measured BLER table within binomial bounds;
  * pl_count_errors equals the reference's count_errors / count_block_errors exactly.
The reference draws from torch's CPU generator, which no GPU stream reproduces: parity of the
producer is statistical by construction (the CPU-device System_AWGN_model keeps the bit-exact path).
"""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pa():
    import polar_amd
    assert torch.cuda.is_available()
    return polar_amd


def _plan(pa, fp, n):
    from polar_amd import _lib
    return _lib.Plan(n, pa.frozen_mask(fp, n), 1, flags=_lib.PL_PLAN_GENERIC)


@pytest.mark.parametrize("k,n", [(512, 1024), (128, 256), (4, 8), (11, 16), (1024, 2048), (0, 32), (32, 32)])
def test_fused_bits_and_codewords_exact(pa, k, n):
    from polar_amd import ops
    from polar_amd.channel import fused_info_bits
    rng = np.random.default_rng(n + k)
    fp = np.sort(rng.permutation(n)[: n - k]) if (k, n) not in ((512, 1024), (128, 256), (1024, 2048)) else \
        pa.reference_frozen_pos(k, n).numpy()
    plan = _plan(pa, fp, n)
    bs, seed, it, row0 = 301, 7, 3, 1000
    u, llr = ops.awgn_qpsk_llr(plan, bs, 1e-7, seed, it, row0)
    u = u.cpu().numpy()
    assert np.array_equal(u, fused_info_bits(seed, it, np.arange(row0, row0 + bs), k))
    cw = oracle.polar_encode(u, fp, n)
    assert np.array_equal((llr.cpu().numpy() > 0).astype(np.float32), cw)  # logits > 0 <=> bit 1
    # same (seed, iteration, rows) -> same draw; another iteration -> another draw
    u2, llr2 = ops.awgn_qpsk_llr(plan, bs, 1e-7, seed, it, row0)
    assert torch.equal(llr, llr2)
    _, llr3 = ops.awgn_qpsk_llr(plan, bs, 1e-7, seed, it + 1, row0)
    assert not torch.equal(llr, llr3) or k == 0


def test_fused_llr_distribution(pa):
    from polar_amd import ops
    from polar_amd.channel import ebnodb2no
    k, n = 512, 1024
    plan = _plan(pa, pa.reference_frozen_pos(k, n).numpy(), n)
    no = float(ebnodb2no(2.0, 2, k / n))
    u, llr = ops.awgn_qpsk_llr(plan, 4096, no, 11, 0)
    cw = torch.from_numpy(oracle.polar_encode(u.cpu().numpy(), pa.reference_frozen_pos(k, n).numpy(), n)).cuda()
    z = (llr - (2.0 / no) * (2 * cw - 1)) * (no ** 0.5) / 2  # standardised noise: N(0, 1)
    assert abs(float(z.mean())) < 0.005
    assert abs(float(z.var()) - 1.0) < 0.005
    assert abs(float((z ** 3).mean())) < 0.01 and abs(float((z ** 4).mean()) - 3.0) < 0.03


# reference x_run SC BLER, (128,256), bs=4096, seed 42 (measured on the reference)
REF_BLER_128_256 = {1.5: 0.9563, 2.0: 0.884, 2.5: 0.7344, 3.0: 0.5195}


@pytest.mark.parametrize("ebno", sorted(REF_BLER_128_256))
def test_fused_bler_matches_reference(pa, ebno):
    from polar_amd import channel, sim
    k, n, bs = 128, 256, 65536
    fp = pa.reference_frozen_pos(k, n)
    model = channel.FusedAWGN(n, k, fp, pa.SC_Dec(fp, n), seed=5)
    b, bh = model(bs, ebno)
    bler = float(sim.count_block_errors(b, bh)) / bs
    p = REF_BLER_128_256[ebno]
    sd = (p * (1 - p) / 4096 + p * (1 - p) / bs) ** 0.5
    assert abs(bler - p) < 5 * sd, (ebno, bler, p)


def test_count_errors_exact(pa):
    from polar_amd import ops, sim
    g = torch.Generator(device="cuda").manual_seed(1)
    for rows, k in ((1001, 37), (64, 512), (3, 1), (9000, 64)):
        a = torch.randint(0, 2, (rows, k), generator=g, device="cuda").float()
        b = a.clone()
        flip = torch.rand((rows, k), generator=g, device="cuda") < 0.01
        b[flip] = 1 - b[flip]
        c = ops.count_errors(a, b)
        assert c.tolist() == [int(sim.count_errors(a, b)), int(sim.count_block_errors(a, b))]
        ops.count_errors(a, b, counts=c)  # accumulates
        assert c.tolist() == [2 * int(sim.count_errors(a, b)), 2 * int(sim.count_block_errors(a, b))]


def test_sim_ber_with_fused_model(pa):
    """sim_ber over FusedAWGN: counters from pl_count_errors, the same stop rules."""
    from polar_amd import channel, sim
    k, n = 32, 64
    fp = pa.reference_frozen_pos(k, n)
    model = channel.FusedAWGN(n, k, fp, pa.SC_Dec(fp, n), seed=42)
    ber, bler, cnt = sim.sim_ber(model, [0.0, 2.0, 4.0], 4000, 5, target_block_errs=500, verbose=False,
                                 device="cuda", return_counts=True)
    assert (cnt[:, 3] % 4000 == 0).all() and cnt[0, 1] >= 500
    assert bler[0] > bler[1] > bler[2] > 0
