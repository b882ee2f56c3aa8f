"""Development aid: where an end-to-end Monte-Carlo iteration's time goes on the GPU --
LLR production (bits, encoder, QPSK, AWGN, demapper), SC decode, error counting.
  python tools/sim_time.py [--k 512 --n 1024 --bs 65536 --ebno 2.0 --producer torch|fused]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "polar-code-pytorch-sionna_amd"))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=512)
ap.add_argument("--n", type=int, default=1024)
ap.add_argument("--bs", type=int, default=65536)
ap.add_argument("--ebno", type=float, default=2.0)
ap.add_argument("--producer", default="torch")
a = ap.parse_args()

import polar_amd  # noqa: E402
from polar_amd import channel, ops, sim  # noqa: E402

dev = torch.device("cuda")
fp = polar_amd.reference_frozen_pos(a.k, a.n)
dec = polar_amd.SC_Dec(fp, a.n)
gen = torch.Generator(device=dev).manual_seed(42)
if a.producer == "fused":
    model = channel.FusedAWGN(a.n, a.k, fp, dec, device=dev, seed=42)
else:
    model = channel.System_AWGN_model(a.n, a.k, channel.GpuEncoder(fp, a.n), dec, device=dev, generator=gen)
eb = torch.tensor(a.ebno, dtype=torch.float32)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3, r


t_llr, (bits, _, llr) = timed(lambda: model.llrs(a.bs, eb))
t_dec, bh = timed(lambda: dec(llr))
t_cnt, _ = timed(lambda: ops.count_errors(bits, bh))
t_all, _ = timed(lambda: model(a.bs, eb))
print(f"({a.k},{a.n}) bs={a.bs} producer={a.producer}: LLR production {t_llr:.3f} ms, decode {t_dec:.3f} ms, "
      f"counting {t_cnt:.3f} ms, model() {t_all:.3f} ms -> {a.bs / t_all / 1e3:.1f} Mcw/s end to end, "
      f"BLER {float(sim.count_block_errors(bits, bh)) / a.bs:.4f}", flush=True)
if a.producer == "fused":
    counts = torch.zeros(2, dtype=torch.int64, device=dev)
    for sk, what in ((False, "pl_awgn_qpsk_llr_bits + pl_sc_decode_count"), (True, "pl_sc_sim_count")):
        model.sim_kernel = sk
        t_fc, _ = timed(lambda: model.error_counts(a.bs, eb, counts), reps=50)
        print(f"  sim_ber's fused path ({what}): {t_fc:.3f} ms per iteration -> "
              f"{a.bs / t_fc / 1e3:.1f} Mcw/s", flush=True)
