"""The simulation harness (caller side of the decoder) against the reference's config-1 run.

tests/golden/harness_c1.npz holds what the reference produced for config 1 of BASELINE.json
(x_run_sn_polar/main.py, (k,n)=(32,64), bs=100, mc_iter=1, seed 42, SC and SCL-8): the LLRs of
every Monte-Carlo iteration and the BER/BLER per SNR point (= the committed plot).  On the CPU
device our LLR producer must reproduce those LLRs bit for bit (same ops, same RNG call order).
CPU tests decode with the oracle (checker); the GPU test decodes with the HIP library.
"""
import os

import numpy as np
import pytest
import torch as tc

import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class _OracleDecoder(tc.nn.Module):
    """Test-only stand-in decoder (the checker), to run the harness without a GPU."""

    def __init__(self, frozen_pos, L=1):
        super().__init__()
        self.fp, self.L = np.asarray(frozen_pos), L
        self.seen = []

    def forward(self, llr):
        self.seen.append(llr.clone())
        x = llr.numpy()
        b = oracle.sc_decode(x, self.fp) if self.L == 1 else oracle.scl_decode(x, self.fp, self.L)[0]
        return tc.from_numpy(b)


def _model(dec, device='cpu'):
    from polar_amd import channel, frozen
    G, _, fp = frozen.get_Kern_frozen_bits(64, 32, frozen.F2)
    enc = channel.DenseEncoder(fp, 64, G, device=device)
    return channel.System_AWGN_model(64, 32, enc, dec, device=device), fp


@pytest.mark.parametrize("name,L", [("sc", 1), ("scl8", 8)])
def test_harness_config1_reproduces_reference(name, L):
    from polar_amd import sim
    d = np.load(os.path.join(GOLDEN, "harness_c1.npz"))
    from polar_amd import frozen
    fp = frozen.reference_frozen_pos(32, 64).numpy()
    dec = _OracleDecoder(fp, L)
    model, fp2 = _model(dec)
    assert np.array_equal(fp2.numpy(), fp)
    np.random.seed(42)
    tc.manual_seed(42)
    ber, bler = sim.sim_ber(model, d["ebno_db"], 100, max_mc_iter=1, target_block_errs=1000, verbose=False)
    llr = np.stack([s.numpy() for s in dec.seen])
    assert llr.shape == d[name + "_llr"].shape
    assert np.array_equal(llr, d[name + "_llr"]), "LLR producer diverged from the reference"
    np.testing.assert_array_equal(bler.numpy(), d[name + "_bler"])
    np.testing.assert_array_equal(ber.numpy(), d[name + "_ber"])


def test_published_table_values():
    """the committed plot's SC / SCL-8 BLER at 0..4.5 dB."""
    d = np.load(os.path.join(GOLDEN, "harness_c1.npz"))
    sc = [0.82, 0.75, 0.53, 0.48, 0.30, 0.29, 0.15, 0.16, 0.06, 0.01]
    scl = [0.56, 0.47, 0.33, 0.28, 0.07, 0.06, 0.03, 0.01, 0.00, 0.0]
    np.testing.assert_allclose(d["sc_bler"], sc, atol=1e-6)
    np.testing.assert_allclose(d["scl8_bler"], scl, atol=1e-6)


@pytest.mark.gpu
def test_harness_config1_on_gpu_decoder():
    """Same run with the drop-in HIP decoders (CPU LLRs -> GPU decode -> CPU bits)."""
    import polar_amd
    from polar_amd import frozen, sim
    d = np.load(os.path.join(GOLDEN, "harness_c1.npz"))
    fp = frozen.reference_frozen_pos(32, 64)
    for name, dec in (("sc", polar_amd.SC_Dec(fp, 64)), ("scl8", polar_amd.SCL_Dec(fp, 64, 8))):
        model, _ = _model(dec)
        np.random.seed(42)
        tc.manual_seed(42)
        ber, bler = sim.sim_ber(model, d["ebno_db"], 100, max_mc_iter=1, target_block_errs=1000, verbose=False)
        np.testing.assert_array_equal(bler.numpy(), d[name + "_bler"])
        np.testing.assert_array_equal(ber.numpy(), d[name + "_ber"])
