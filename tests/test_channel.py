"""Host-side pins of the fused Monte-Carlo producer (csrc/channel_kernel.hip): the numpy
Philox4x32-10 restatement against the Random123 known-answer vectors, and the information-bit
placement helper the GPU tests compare the kernel with."""
import numpy as np
import pytest

from polar_amd.channel import fused_info_bits, philox4x32_10

# Random123 kat_vectors, philox4x32_10: (counter, key) -> output
KAT = [([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
       ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
       ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1])]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_philox_known_answers(ctr, key, want):
    got = philox4x32_10(np.array(ctr, dtype=np.uint64), np.array(key, dtype=np.uint64))
    assert [int(v) for v in got] == want


def test_philox_vectorised_equals_scalar():
    rng = np.random.default_rng(0)
    ctr = rng.integers(0, 2 ** 32, (5, 3, 4), dtype=np.uint64)
    key = rng.integers(0, 2 ** 32, (5, 3, 2), dtype=np.uint64)
    got = philox4x32_10(ctr, key)
    for i in range(5):
        for j in range(3):
            assert np.array_equal(got[i, j], philox4x32_10(ctr[i, j], key[i, j]))


def test_fused_info_bits_layout():
    u = fused_info_bits(42, 3, np.arange(10, 20), 100)
    assert u.shape == (10, 100) and set(np.unique(u)) <= {0.0, 1.0}
    # row 12 alone gives the same bits (rows are independent streams), another iteration differs
    assert np.array_equal(fused_info_bits(42, 3, [12], 100)[0], u[2])
    assert not np.array_equal(fused_info_bits(42, 4, [12], 100)[0], u[2])
    # bit r is bit r % 32 of word r // 32 = component (r // 32) % 4 of block (r // 32) // 4
    w = philox4x32_10(np.array([12, 0, 3, 0], dtype=np.uint64), np.array([42, 0], dtype=np.uint64))
    assert [int(b) for b in u[2, 32:64]] == [(int(w[1]) >> i) & 1 for i in range(32)]
    assert abs(fused_info_bits(1, 0, np.arange(2000), 512).mean() - 0.5) < 0.01


def test_pack_bits_layout():
    """ops.pack_bits: bit m of a row = bit m % 32 of word m // 32 (pl_sc_decode_count's reference)."""
    import torch
    from polar_amd import ops
    rng = np.random.default_rng(4)
    for k in (1, 31, 32, 33, 48, 512):
        b = rng.integers(0, 2, (7, k))
        w = ops.pack_bits(torch.from_numpy(b).float()).numpy().view(np.uint32)
        assert w.shape == (7, (k + 31) // 32)
        for m in range(k):
            assert np.array_equal((w[:, m // 32] >> np.uint32(m % 32)) & 1, b[:, m])
