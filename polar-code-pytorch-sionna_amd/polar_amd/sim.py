"""Monte-Carlo BER/BLER simulation (the caller side of the decoder), single- or multi-GPU.

Mirrors my_sn/sim.py:19-140 (sim_ber: error counters, target-error stop, early stop at the first
error-free SNR point, the same progress table) and my_sn/plotting.py:22-48 (PlotBER.simulate).

Counters stay on the device.  The reference reads them on the host after every Monte-Carlo
iteration (the stop rule, sim.py:107-123); here that read happens once per *window* of
iterations when the model's draws are keyed by (SNR point, iteration) rather than by call order
(`keyed_streams`, e.g. channel.FusedAWGN): the window's iterations are launched back to back into
per-iteration counter rows, reduced over ranks with one all_reduce of a [W, 4] int64 tensor, read
once, and the reference's stop rule is then applied iteration by iteration on the host; counts
of iterations after the stop are discarded.  Because iteration ii of point i draws the same
codewords whether or not later iterations were launched, the result is exactly the sequential
loop's.  Models whose draws depend on call order (the CPU-device System_AWGN_model, which follows
the reference's global torch RNG) keep the one-iteration window, so their RNG order is the
reference's.

With a torch.distributed process group (one rank per GPU, RCCL over xGMI) every rank simulates
its own batch_size codewords per iteration and the per-window counter block is summed over ranks;
every stop decision is taken on the reduced counts, so all ranks leave together.
"""
import time

import numpy as np
import torch as tc


def hard_decisions(llr):
    return tc.where(llr > 0, 1., 0.)


def count_block_errors(b, b_hat):
    return tc.sum(tc.any(tc.not_equal(b, b_hat).to(tc.int64), dim=-1))


def count_errors(b, b_hat):
    return tc.sum(tc.not_equal(b, b_hat).to(tc.int64))


_STATUS = ["not simulated", "reached max iter       ", "no errors - early stop",
           "reached target bit errors", "reached target block errors"]
_HEADER = ["EbNo [dB]", "BER", "BLER", "bit errors", "num bits", "block errors", "num blocks", "runtime [s]", "status"]

MAX_WINDOW = 64  # iterations launched per host read (keyed models)


def _row(cells, end):
    print("{: >9} |{: >11} |{: >11} |{: >12} |{: >12} |{: >13} |{: >12} |{: >12} |{: >10}".format(*cells), end=end)


def _model_of(mc_fun):
    return getattr(mc_fun, "__self__", mc_fun)


def _next_window(w, done, max_mc_iter, acc, target_bit_errs, target_block_errs, max_window):
    """Iterations to launch next: doubling from 1 up to max_window, never past max_mc_iter, and
    no more than ~1.25x the iterations the error rate so far predicts the targets still need."""
    w = min(max(1, 2 * w), max_window, max_mc_iter - done)
    if done > 0:
        for tgt, got in ((target_bit_errs, acc[0]), (target_block_errs, acc[1])):
            if tgt is not None and got > 0:
                need = (tgt - got) * done / got  # iterations at the observed rate
                w = min(w, max(1, int(np.ceil(1.25 * need)) + 1))
    return max(1, w)


def sim_ber(mc_fun, ebno_dbs, batch_size, max_mc_iter, soft_estimates=False, target_bit_errs=None,
            target_block_errs=None, early_stop=True, verbose=True, dtype=tc.complex64, device='cpu',
            process_group=None, return_counts=False, max_window=None):
    """Returns (ber, bler) float tensors per SNR point, like my_sn/sim.py:sim_ber.

    With process_group set, each rank simulates its own batch_size codewords per iteration and the
    counters are summed over ranks (global BER/BLER); the return values are identical on all ranks.
    max_window: iterations per host read for keyed models (default MAX_WINDOW; 1 = the reference's
    read after every iteration).  The counter block is all-reduced on the group backend's device
    (an RCCL group: the model's GPU; gloo: the host), whatever `device` says.  A model with
    next_epoch() (channel.FusedAWGN) is advanced once per call, so a second run over the same
    model draws fresh codewords, as the reference's global RNG would.  return_counts adds the int64 [points, 4] counters
    [bit errors, block errors, bits, blocks]."""
    dist = None
    if process_group is not None:
        import torch.distributed as dist
    rank0 = dist is None or dist.get_rank(process_group) == 0
    verbose = verbose and rank0
    ebno_dbs = tc.from_numpy(np.asarray(ebno_dbs)).to(tc.float32)
    P = ebno_dbs.shape[0]
    model = _model_of(mc_fun)
    cdev = _counter_device(device, dist, process_group, model)
    keyed = bool(getattr(model, "keyed_streams", False))
    wmax = (MAX_WINDOW if max_window is None else max(1, int(max_window))) if keyed else 1
    # channel.FusedAWGN with this package's SC decoder: decode and count in one kernel, no bit rows
    fused = None if soft_estimates else getattr(model, "error_counts", None)
    # counters: [bit_errors, block_errors, nb_bits, nb_blocks] per point (sim.py:72-75), on the host
    cnt = np.zeros([P, 4], dtype=np.int64)
    status = tc.zeros(P)
    runtime = np.zeros(P)
    header_done = False
    try:
        for i in range(P):
            t0 = time.perf_counter()
            done, w, stop, it = 0, 0, False, -1
            while done < max_mc_iter and not stop:
                w = _next_window(w, done, max_mc_iter, cnt[i], target_bit_errs, target_block_errs, wmax)
                block = _run_window(mc_fun, model, fused, keyed, i, done, w, batch_size, ebno_dbs[i], soft_estimates)
                block = block.to(cdev)
                if dist is not None:
                    dist.all_reduce(block, op=dist.ReduceOp.SUM, group=process_group)
                host = block.cpu().numpy()  # one host sync per window (the reference: per iteration, sim.py:114)
                for j in range(w):
                    it = done + j
                    cnt[i] += host[j]
                    if verbose:
                        if not header_done:
                            _row(_HEADER, "\n")
                            print('-' * 135)
                            header_done = True
                        _row(_cells(ebno_dbs[i], cnt[i], time.perf_counter() - t0, f"iter: {it:.0f}/{max_mc_iter:.0f}"), "\r")
                    if target_bit_errs is not None and cnt[i, 0] >= target_bit_errs:
                        status[i] = 3
                        stop = True
                        break
                    if target_block_errs is not None and cnt[i, 1] >= target_block_errs:
                        status[i] = 4
                        stop = True
                        break
                    if it == max_mc_iter - 1:
                        status[i] = 1
                done += w
            runtime[i] = time.perf_counter() - t0
            if verbose:
                _row(_cells(ebno_dbs[i], cnt[i], runtime[i], _STATUS[int(status[i])]), "\n")
            if early_stop and cnt[i, 1] == 0:
                status[i] = 2
                if verbose:
                    print(f"\nSimu stopped as no error occurred @ EbNo = {ebno_dbs[i].numpy():.1f} dB.\n")
                break
    finally:
        # the next run draws fresh codewords (keyed models: a new epoch of the (point, iteration)
        # key) -- also after a run that raised or was interrupted, so a retry never redraws it
        next_epoch = getattr(model, "next_epoch", None)
        if callable(next_epoch):
            next_epoch()
    c = tc.from_numpy(cnt)
    ber = c[:, 0] / c[:, 2]
    bler = c[:, 1] / c[:, 3]
    ber = tc.where(tc.isnan(ber), tc.zeros_like(ber), ber)
    bler = tc.where(tc.isnan(bler), tc.zeros_like(bler), bler)
    if return_counts:
        return ber, bler, c
    return ber, bler


def _counter_device(device, dist, process_group, model):
    """Where the per-window counter block is reduced: an RCCL ("nccl") group reduces device
    tensors, so the block goes to the model's GPU (else the current one) whatever `device` says;
    gloo and other CPU backends reduce host tensors; without a group, `device` as given."""
    if dist is None:
        return tc.device(device)
    if dist.get_backend(process_group) == "nccl":
        mdev = getattr(model, "device", None)
        if mdev is not None and tc.device(mdev).type == "cuda":
            return tc.device(mdev)
        return tc.device("cuda", tc.cuda.current_device())
    return tc.device("cpu")


def _run_window(mc_fun, model, fused, keyed, point, it0, w, batch_size, ebno, soft_estimates):
    """Launch iterations it0 .. it0 + w - 1 of SNR point `point`; returns their int64 [w, 4]
    counters (on the model's device, not yet read).  Keyed models draw iteration ii of the point
    as stream (point, ii); other models draw in call order (w is 1 for them)."""
    rows = []
    block = None
    for j in range(w):
        kw = {"stream": (point, it0 + j)} if keyed else {}
        if fused is not None:
            if block is None:
                dev = getattr(model, "device", None)
                block = tc.zeros([w, 4], dtype=tc.int64, device=dev)
            be = fused(batch_size, ebno, counts=block[j], **kw)
            if be is not None:
                continue
            fused = None  # this model/decoder pair has no fused count: forward() + count
        b, b_hat = mc_fun(batch_size=batch_size, ebno_db=ebno, **kw)
        if soft_estimates:
            b_hat = hard_decisions(b_hat)
        inc = _increment(b, b_hat)
        if block is not None:
            block[j] = inc.to(block.device)
        else:
            rows.append(inc)
    if block is None:
        return tc.stack(rows)
    k = getattr(model, "k", None)
    if k is None:
        raise ValueError("a model with error_counts must expose k (information bits per codeword)")
    # bits and blocks of the fused iterations (rows filled by forward() already hold theirs)
    filled = block[:, 3] == 0
    block[:, 2] = tc.where(filled, tc.full_like(block[:, 2], batch_size * int(k)), block[:, 2])
    block[:, 3] = tc.where(filled, tc.full_like(block[:, 3], batch_size), block[:, 3])
    return block


def _increment(b, b_hat):
    """[bit errors, block errors, bits, blocks] of one iteration (sim.py:84-100)."""
    if b.is_cuda and b_hat.is_cuda and b.shape == b_hat.shape and b.shape[-1] > 0:
        # both counters in one HIP pass (pl_count_errors), no torch reductions
        from . import ops
        counts = tc.zeros(4, dtype=tc.int64, device=b.device)
        ops.count_errors(b, b_hat, counts=counts[:2])
        counts[2] = b.numel()
        counts[3] = b.numel() // b.shape[-1]
        return counts
    return tc.stack([count_errors(b, b_hat), count_block_errors(b, b_hat),
                     tc.tensor(b.numel(), device=b.device), tc.tensor(b.numel() // b.shape[-1], device=b.device)])


def _cells(ebno, host, rt, status_txt):
    ber = host[0] / host[2] if host[2] else 0.0
    bler = host[1] / host[3] if host[3] else 0.0
    return [str(np.round(ebno.cpu().numpy(), 3)), f"{ber:.4e}", f"{bler:.4e}", int(host[0]), int(host[2]),
            int(host[1]), int(host[3]), np.round(rt, 1), status_txt]


class PlotBER:
    """Stores simulated curves (my_sn/plotting.py:22-48); plotting itself is optional (matplotlib)."""

    def __init__(self, title="Bit/Block Error Rate"):
        self.title = title
        self.ber, self.snr, self.legend = [], [], []

    def simulate(self, mc_fun, ebno_dbs, batch_size, legend="", add_ber=True, add_bler=False, max_mc_iter=1,
                 soft_estimates=False, target_bit_errs=None, target_block_errs=None, verbose=True, device='cpu',
                 process_group=None):
        ber, bler = sim_ber(mc_fun, ebno_dbs, batch_size, soft_estimates=soft_estimates, max_mc_iter=max_mc_iter,
                            target_bit_errs=target_bit_errs, target_block_errs=target_block_errs, verbose=verbose,
                            device=device, process_group=process_group)
        if add_ber:
            self.ber += [ber]
            self.snr += [ebno_dbs]
            self.legend += [legend]
        if add_bler:
            self.ber += [bler]
            self.snr += [ebno_dbs]
            self.legend += [legend + " (BLER)"]
        return ber, bler
