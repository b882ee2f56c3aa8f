"""BER/BLER simulation driver with the flags of x_run_sn_polar/main.py + config.py.

    python -m polar_amd.cli --k 32 --n 64 --algos [scl] --bs 100 --mc_iter 1
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m polar_amd.cli \\
        --k 512 --n 1024 --bs 65536 --mc_iter 10 --snr_end 4.5

Reference: main.py:32-76 (gen_code, seed 42 per code, SNR grid arange(0, snr_end, 0.5), SC always,
SCL when 'scl' in algos, PlotBER.simulate with target_block_errs=1000) and config.py:5-26.
--llr_device cpu reproduces the reference run bit for bit (LLRs generated on the CPU with the
reference's RNG call order, decoded on the GPU); the default generates LLRs on the GPU.  With
several ranks (torchrun, one per GPU) every rank simulates --bs codewords per iteration with its
own RNG stream (seed 42 + rank) and the error counters are summed with one RCCL all_reduce.
"""
import argparse
import math
import os
import random

import numpy as np
import torch as tc


def _list_arg(s):
    s = s.strip()
    if s.startswith("[") and s.endswith("]"):
        s = s[1:-1]
    return [x.strip().strip("'\"") for x in s.split(",") if x.strip()]


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--algos", type=_list_arg, default=["scl"])
    ap.add_argument("--kern", default="F2")
    ap.add_argument("--verbose", type=lambda s: s.lower() in ("1", "true", "yes"), default=False)
    ap.add_argument("--bs", type=int, default=3)
    ap.add_argument("--snr_end", type=float, default=5)
    ap.add_argument("--mc_iter", type=int, default=10)
    ap.add_argument("--list_size", type=int, default=8)
    ap.add_argument("--mode", default="max")
    ap.add_argument("--spec", default=False)
    ap.add_argument("--llr_device", choices=["cuda", "cpu"], default="cuda")
    ap.add_argument("--llr_producer", choices=["fused", "ops"], default="fused",
                    help="cuda LLRs: one fused HIP kernel (Philox; default) or the op-by-op torch port")
    ap.add_argument("--target_block_errs", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--plot", default=None, help="save the BLER plot here (matplotlib)")
    ap.add_argument("--frozen", choices=["reference", "recompute"], default="reference",
                    help="reference: the pinned sets froze.py produced; recompute: re-run froze.py's recipe")
    return ap.parse_args(argv)


def set_seed(seed):  # main.py:24-29
    np.random.seed(seed)
    random.seed(seed)
    tc.manual_seed(seed)


def gen_code(c, name, mode, device, generator=None):  # main.py:32-41
    from . import channel, frozen
    from .decoders import SC_Dec, SCL_Dec
    assert math.log(c.n, 2).is_integer()
    G, _, fp = frozen.get_Kern_frozen_bits(c.n, c.n - c.k, frozen.F2)
    if c.frozen == "reference":
        try:
            fp = frozen.reference_frozen_pos(c.k, c.n)
        except KeyError:
            pass
    if device.type == "cuda":
        enc = channel.GpuEncoder(fp, c.n)
    else:
        enc = channel.DenseEncoder(fp, c.n, G, device=device)
    dev_str = str(device) if device.type == "cuda" else "cpu"
    if mode == "sc":
        dec = SC_Dec(fp, c.n, device=dev_str)
    elif mode == "scl":
        dec = SCL_Dec(fp, c.n, c.list_size, device=dev_str)
    else:
        raise Exception('error...')
    if device.type == "cuda" and getattr(c, "llr_producer", "fused") == "fused":
        # one HIP launch for bits/encoder/mapper/channel/demapper; rank r draws stream rows
        # [r*bs, (r+1)*bs) of the seed's stream
        rank = int(os.environ.get("RANK", "0"))
        model = channel.FusedAWGN(c.n, c.k, fp, dec, device=device, seed=c.seed, row0=rank * c.bs)
    else:
        model = channel.System_AWGN_model(c.n, c.k, enc, dec, device=device, generator=generator)
    return [model, name]


def main(argv=None):
    from .sim import PlotBER
    c = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if tc.cuda.is_available():
        # one GPU per rank whichever backend carries the counters: the decoders run on the
        # current device when the LLRs are produced on the CPU (gloo path)
        tc.cuda.set_device(local % tc.cuda.device_count())
    if world > 1:
        import torch.distributed as dist
        if c.llr_device == "cuda":
            dist.init_process_group("nccl", device_id=tc.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        pg = dist.group.WORLD
    device = tc.device("cuda", local) if c.llr_device == "cuda" else tc.device("cpu")
    gen = tc.Generator(device=device).manual_seed(c.seed + rank) if device.type == "cuda" else None
    ebno_db = np.arange(0, c.snr_end, 0.5)
    codes = [gen_code(c, "SC", "sc", device, gen)]
    if "scl" in c.algos:
        codes.append(gen_code(c, f"SCL-{c.list_size}", "scl", device, gen))
    plot = PlotBER(f"Performance of Short Len Codes (k={c.k}, n={c.n})")
    results = {}
    for model, name in codes:
        if rank == 0:
            print("\nRunning: " + name)
        set_seed(c.seed + rank)
        if gen is not None:
            gen.manual_seed(c.seed + rank)
        counter_dev = device if device.type == "cuda" else "cpu"
        ber, bler = plot.simulate(model, ebno_dbs=ebno_db, batch_size=c.bs, target_block_errs=c.target_block_errs,
                                  legend=name, soft_estimates=False, max_mc_iter=c.mc_iter, add_bler=True,
                                  device=counter_dev, process_group=pg)
        results[name] = (ber.numpy(), bler.numpy())
    if rank == 0 and c.plot:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        plt.figure(figsize=(16, 12))
        for i, leg in enumerate(plot.legend):
            if "BLER" in leg:
                plt.semilogy(ebno_db, plot.ber[i], c='C%d' % i, label=leg, linewidth=2,
                             linestyle='--' if "SC" in leg and "SCL" not in leg else '-')
        plt.grid(which="both")
        plt.xlabel(r"$E_b/N_0$ (dB)")
        plt.ylabel("BLER")
        plt.legend()
        plt.savefig(c.plot)
    if pg is not None:
        import torch.distributed as dist
        dist.destroy_process_group()
    return results


if __name__ == "__main__":
    main()
