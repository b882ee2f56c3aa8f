"""sim_ber's windowed Monte-Carlo loop (polar_amd/sim.py) on CPU, against the reference stop rule.

The reference (my_sn/sim.py:79-133) reads its counters after every iteration and stops a point
at the first iteration whose running count reaches a target.  sim_ber launches windows of
iterations for models whose draws are keyed by (SNR point, iteration) and applies that rule on
the host afterwards.  KeyedModel is such a model on the CPU (numpy draws keyed per
(seed, point, iteration), stream rows row0 .. row0 + bs - 1, decoded by the oracle, the checker):
  * windowed counters == the one-iteration loop's, with targets that stop points mid-window,
    early stop, and max_mc_iter not a multiple of the window;
  * a hand-written restatement of the reference loop over the same draws gives the same table;
  * _next_window never overshoots max_mc_iter.
test_distributed.py runs the same model sharded over 2 gloo ranks.
"""
import numpy as np
import pytest
import torch as tc

import oracle


class KeyedModel(tc.nn.Module):
    """mc_fun with keyed draws: iteration ii of point p decodes stream rows row0 .. row0 + bs - 1
    of the (seed, p, ii) draw; codewords of global row r are the same whatever the batch split."""

    keyed_streams = True

    def __init__(self, k=32, n=64, seed=7, row0=0, rows_total=None):
        super().__init__()
        from polar_amd import frozen
        self.k, self.n, self.seed, self.row0 = k, n, seed, row0
        self.fp = frozen.reference_frozen_pos(k, n).numpy()
        self.rows_total = rows_total
        self.calls = []

    def _global_draw(self, point, it, rows, ebno_db):
        rng = np.random.default_rng([self.seed, point, it])
        u = rng.integers(0, 2, size=(rows, self.k)).astype(np.float32)
        x = oracle.polar_encode(u, self.fp, self.n)
        no = 1.0 / (10 ** (float(ebno_db) / 10) * (self.k / self.n) * 2)
        y = (1 - 2 * x) + np.sqrt(no / 2) * rng.standard_normal(size=x.shape)
        llr = (-4.0 * y / (2 * no)).astype(np.float32)  # logits log P(1)/P(0) for BPSK components
        return u, llr

    def forward(self, batch_size, ebno_db, stream=None):
        assert stream is not None, "sim_ber must key the draws of a keyed model"
        point, it = stream
        self.calls.append((point, it))
        total = self.rows_total or (self.row0 + batch_size)
        u, llr = self._global_draw(point, it, total, ebno_db)
        u, llr = u[self.row0:self.row0 + batch_size], llr[self.row0:self.row0 + batch_size]
        return tc.from_numpy(u), tc.from_numpy(oracle.sc_decode(llr, self.fp))


def reference_loop(model, ebno_dbs, bs, max_mc_iter, target_bit_errs=None, target_block_errs=None, early_stop=True):
    """my_sn/sim.py:79-133 restated over the keyed draws: counters [P, 4]."""
    from polar_amd import sim
    cnt = np.zeros((len(ebno_dbs), 4), dtype=np.int64)
    for i, e in enumerate(ebno_dbs):
        for ii in range(max_mc_iter):
            b, b_hat = model(bs, e, stream=(i, ii))
            cnt[i] += [int(sim.count_errors(b, b_hat)), int(sim.count_block_errors(b, b_hat)), b.numel(), b.shape[0]]
            if target_bit_errs is not None and cnt[i, 0] >= target_bit_errs:
                break
            if target_block_errs is not None and cnt[i, 1] >= target_block_errs:
                break
        if early_stop and cnt[i, 1] == 0:
            break
    return cnt


@pytest.mark.parametrize("targets", [dict(target_block_errs=25), dict(target_bit_errs=300), dict()])
def test_window_equals_sequential_and_reference(targets):
    from polar_amd import sim
    ebno = np.array([0.0, 2.0, 4.0, 6.0, 9.0])
    m = KeyedModel()
    _, _, c_win = sim.sim_ber(m, ebno, 16, max_mc_iter=11, verbose=False, return_counts=True, **targets)
    calls_win = len(m.calls)
    m1 = KeyedModel()
    _, _, c_seq = sim.sim_ber(m1, ebno, 16, max_mc_iter=11, verbose=False, return_counts=True, max_window=1,
                              **targets)
    want = reference_loop(KeyedModel(), ebno, 16, 11, **targets)
    np.testing.assert_array_equal(c_seq.numpy(), want)
    np.testing.assert_array_equal(c_win.numpy(), want)
    # the windowed loop may launch iterations past a stop, never fewer than the sequential loop
    assert calls_win >= len(m1.calls)
    assert all(it < 11 for _, it in m.calls)


def test_window_does_not_shift_later_points():
    """A point that stops mid-window leaves the draws of every later point unchanged."""
    from polar_amd import sim
    ebno = np.array([0.0, 1.0, 2.0])
    m = KeyedModel()
    _, _, c = sim.sim_ber(m, ebno, 8, max_mc_iter=40, target_block_errs=20, verbose=False, return_counts=True,
                          max_window=16)
    first = [it for p, it in m.calls if p == 0]
    assert max(first) + 1 > int(np.ceil(c[0, 3].item() / 8))  # speculative iterations were launched
    want = reference_loop(KeyedModel(), ebno, 8, 40, target_block_errs=20)
    np.testing.assert_array_equal(c.numpy(), want)


def test_next_window_bounds():
    from polar_amd.sim import _next_window
    acc = np.zeros(4, dtype=np.int64)
    w, done, seen = 0, 0, []
    while done < 100:
        w = _next_window(w, done, 100, acc, None, None, 64)
        seen.append(w)
        done += w
    assert done == 100 and seen[:4] == [1, 2, 4, 8] and max(seen) <= 64
    # a target about to be reached caps the window at the predicted need
    acc = np.array([0, 90, 0, 0])
    assert _next_window(32, 10, 1000, acc, None, 100, 64) == 3


def test_counts_argument_is_validated():
    """ops._counts: the counting kernels' 64-bit atomics only ever see a contiguous int64 tensor of
    >= 2 elements on the launch device (a caller's counts went straight to the kernel)."""
    from polar_amd import ops
    cpu = tc.device("cpu")
    assert ops._counts(None, cpu).tolist() == [0, 0]
    ok = tc.zeros(4, dtype=tc.int64)
    assert ops._counts(ok[:2], cpu) is not None
    for bad in (tc.zeros(2, dtype=tc.int32), tc.zeros(1, dtype=tc.int64), tc.zeros(4, dtype=tc.int64)[::2],
                [0, 0], tc.zeros((2, 2), dtype=tc.int64).t()):
        with pytest.raises(ValueError):
            ops._counts(bad, cpu)
    with pytest.raises(ValueError):
        ops._counts(ok, tc.device("meta"))


def test_fused_awgn_stream_keys():
    """FusedAWGN._draw: stream (point, iteration) -> (iteration, row0 + point << 32); range checks."""
    from polar_amd import channel, frozen
    fp = frozen.reference_frozen_pos(32, 64)
    m = channel.FusedAWGN(64, 32, fp, None, device="cpu", row0=100)
    assert m._draw(10, (3, 7)) == (7, 100 + (3 << 32))
    assert m._draw(10, None) == (0, 100) and m._draw(10, None) == (1, 100)  # call order, point 0
    for stream in ((0, 2 ** 32), (0, -1), (2 ** 31, 0)):
        with pytest.raises(ValueError):
            m._draw(10, stream)
    with pytest.raises(ValueError):
        m._draw(2 ** 32, (0, 0))
    with pytest.raises(ValueError):
        channel.FusedAWGN(64, 32, fp, None, device="cpu", row0=2 ** 32)


def test_fused_awgn_epochs_rekey_each_run():
    """sim_ber advances a keyed model's epoch once per run, so running the same sweep
    twice over one FusedAWGN draws fresh codewords; epoch 0 keeps the seed itself (the pinned
    streams of the GPU tests)."""
    from polar_amd import channel, frozen, sim

    class Keyed(channel.FusedAWGN):
        keys = []

        def error_counts(self, batch_size, ebno_db, counts=None, stream=None):
            return None  # no fused path: sim_ber calls forward()

        def forward(self, batch_size, ebno_db, stream=None):
            self.keys.append((self.key(), stream))
            b = tc.zeros((batch_size, self.k))
            return b, b

    fp = frozen.reference_frozen_pos(32, 64)
    m = Keyed(64, 32, fp, None, device="cpu", seed=42)
    assert m.key() == 42
    sim.sim_ber(m, [1.0], 4, max_mc_iter=2, verbose=False)
    sim.sim_ber(m, [1.0], 4, max_mc_iter=2, verbose=False)
    k1 = {k for k, _ in Keyed.keys[:2]}
    k2 = {k for k, _ in Keyed.keys[2:]}
    assert k1 == {42} and len(k2) == 1 and k2 != k1 and m.epoch == 2
    assert [s for _, s in Keyed.keys[:2]] == [s for _, s in Keyed.keys[2:]]  # same (point, iteration) streams
    keys = set()
    for _ in range(100):
        keys.add(m.key())
        m.next_epoch()
    assert len(keys) == 100


def test_counter_device_follows_the_group_backend():
    """an RCCL group reduces device tensors, so the counter block goes to the
    model's GPU (or the current one) whatever `device` says; gloo reduces on the host."""
    from polar_amd import sim

    class FakeDist:
        def __init__(self, backend):
            self.backend = backend

        def get_backend(self, group=None):
            return self.backend

    class M:
        device = tc.device("cuda", 3)

    assert sim._counter_device("cpu", None, None, M()) == tc.device("cpu")
    assert sim._counter_device("cpu", FakeDist("nccl"), None, M()) == tc.device("cuda", 3)
    assert sim._counter_device("cuda", FakeDist("gloo"), None, M()) == tc.device("cpu")


def test_epoch_keys_mix_and_interrupted_runs_advance():
    """epoch keys come from a mixing function (related seeds do not replay each other's
    epochs), and a sim_ber run that raises still advances the epoch (a retry draws fresh codewords)."""
    from polar_amd import channel, frozen, sim
    C = 0x9E3779B97F4A7C15
    fp = frozen.reference_frozen_pos(32, 64)
    a = channel.FusedAWGN(64, 32, fp, None, device="cpu", seed=42)
    b = channel.FusedAWGN(64, 32, fp, None, device="cpu", seed=42 ^ ((1 * C) ^ (2 * C)))
    a.epoch, b.epoch = 2, 1  # the XOR key gave (seed, 2) and (seed ^ (C ^ 2C), 1) the same key
    assert a.key() != b.key()
    keys = {channel.FusedAWGN(64, 32, fp, None, device="cpu", seed=s).key() for s in range(50)}
    assert len(keys) == 50  # epoch 0: the seed itself

    class Boom(channel.FusedAWGN):
        def error_counts(self, batch_size, ebno_db, counts=None, stream=None):
            return None

        def forward(self, batch_size, ebno_db, stream=None):
            raise KeyboardInterrupt

    m = Boom(64, 32, fp, None, device="cpu", seed=7)
    with pytest.raises(KeyboardInterrupt):
        sim.sim_ber(m, [1.0], 4, max_mc_iter=2, verbose=False)
    assert m.epoch == 1 and m.key() != 7
