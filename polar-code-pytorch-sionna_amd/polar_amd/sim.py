"""Monte-Carlo BER/BLER simulation (the caller side of the decoder), single- or multi-GPU.

Mirrors my_sn/sim.py:19-140 (sim_ber: error counters, target-error stop, early stop at the first
error-free SNR point, the same progress table) and my_sn/plotting.py:22-48 (PlotBER.simulate).
Counters stay on the device; with a torch.distributed process group (one rank per GPU, RCCL over
xGMI) the only exchange is one all_reduce(SUM) of an int64[4] counter vector per Monte-Carlo
iteration, and every stop decision is taken on the reduced counts so all ranks leave together.
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


def _row(cells, end):
    print("{: >9} |{: >11} |{: >11} |{: >12} |{: >12} |{: >13} |{: >12} |{: >12} |{: >10}".format(*cells), end=end)


def sim_ber(mc_fun, ebno_dbs, batch_size, max_mc_iter, soft_estimates=False, target_bit_errs=None,
            target_block_errs=None, early_stop=True, verbose=True, dtype=tc.complex64, device='cpu',
            process_group=None, return_counts=False):
    """Returns (ber, bler) float tensors per SNR point, like my_sn/sim.py:sim_ber.

    With process_group set, each rank simulates its own batch_size codewords per iteration and the
    counters are summed over ranks (global BER/BLER); the return values are identical on all ranks.
    """
    dist = None
    if process_group is not None:
        import torch.distributed as dist
    rank0 = dist is None or dist.get_rank(process_group) == 0
    verbose = verbose and rank0
    ebno_dbs = tc.from_numpy(np.asarray(ebno_dbs)).to(tc.float32)
    P = ebno_dbs.shape[0]
    cdev = tc.device(device)
    # counters: [bit_errors, block_errors, nb_bits, nb_blocks] per point (sim.py:72-75)
    cnt = tc.zeros([P, 4], dtype=tc.int64, device=cdev)
    status = tc.zeros(P)
    runtime = np.zeros(P)
    # channel.FusedAWGN with this package's SC decoder: decode and count in one kernel, no bit rows
    fused = None if soft_estimates else getattr(getattr(mc_fun, "__self__", mc_fun), "error_counts", None)
    for i in range(P):
        t0 = time.perf_counter()
        it = -1
        for ii in range(max_mc_iter):
            it += 1
            be = fused(batch_size, ebno_dbs[i]) if fused is not None else None
            if be is not None:
                k = getattr(mc_fun, "__self__", mc_fun).k
                inc = tc.cat([be, tc.tensor([batch_size * k, batch_size], dtype=tc.int64, device=be.device)])
            else:
                b, b_hat = mc_fun(batch_size=batch_size, ebno_db=ebno_dbs[i])
                if soft_estimates:
                    b_hat = hard_decisions(b_hat)
                inc = _increment(b, b_hat)
            inc = inc.to(cdev)
            if dist is not None:
                dist.all_reduce(inc, op=dist.ReduceOp.SUM, group=process_group)
            cnt[i] += inc
            host = cnt[i].cpu().numpy()  # one host sync per iteration, as sim.py:114
            if verbose:
                if i == 0 and it == 0:
                    _row(_HEADER, "\n")
                    print('-' * 135)
                _row(_cells(ebno_dbs[i], host, time.perf_counter() - t0, f"iter: {ii:.0f}/{max_mc_iter:.0f}"), "\r")
            if target_bit_errs is not None and host[0] >= target_bit_errs:
                status[i] = 3
                break
            if target_block_errs is not None and host[1] >= target_block_errs:
                status[i] = 4
                break
            if it == max_mc_iter - 1:
                status[i] = 1
        runtime[i] = time.perf_counter() - t0
        host = cnt[i].cpu().numpy()
        if verbose:
            _row(_cells(ebno_dbs[i], host, runtime[i], _STATUS[int(status[i])]), "\n")
        if early_stop and host[1] == 0:
            status[i] = 2
            if verbose:
                print(f"\nSimu stopped as no error occurred @ EbNo = {ebno_dbs[i].numpy():.1f} dB.\n")
            break
    c = cnt.cpu()
    ber = c[:, 0] / c[:, 2]
    bler = c[:, 1] / c[:, 3]
    ber = tc.where(tc.isnan(ber), tc.zeros_like(ber), ber)
    bler = tc.where(tc.isnan(bler), tc.zeros_like(bler), bler)
    if return_counts:
        return ber, bler, c
    return ber, bler


def _increment(b, b_hat):
    """[bit errors, block errors, bits, blocks] of one iteration (sim.py:84-100)."""
    if b.is_cuda and b_hat.is_cuda and b.shape == b_hat.shape and b.shape[-1] > 0:
        # both counters in one HIP pass (pl_count_errors), no torch reductions
        from . import ops
        be = ops.count_errors(b, b_hat)
        return tc.cat([be, tc.tensor([b.numel(), b.numel() // b.shape[-1]], dtype=tc.int64, device=b.device)])
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
