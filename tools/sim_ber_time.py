"""Wall time per Monte-Carlo iteration of sim_ber (the windowed loop) against the fused kernel
alone, one GPU: FusedAWGN + SC_Dec -> pl_sc_sim_count at (k, n), bs codewords per iteration.

  python tools/sim_ber_time.py [--k 512 --n 1024 --bs 65536 --iters 400 --ebno 3.0]

Prints, per configuration: ms per iteration of
  * the kernel loop: ops.sc_sim_count back to back, HIP events (no host reads);
  * sim_ber with the default window (one host read per window);
  * sim_ber with max_window=1 (a host read after every iteration, as my_sn/sim.py:107-123).
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "polar-code-pytorch-sionna_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=512)
ap.add_argument("--n", type=int, default=1024)
ap.add_argument("--bs", type=int, default=65536)
ap.add_argument("--iters", type=int, default=400)
ap.add_argument("--ebno", type=float, default=3.0)
a = ap.parse_args()

import polar_amd  # noqa: E402
from polar_amd import channel, ops, sim  # noqa: E402

dev = torch.device("cuda", 0)
fp = polar_amd.reference_frozen_pos(a.k, a.n)
dec = polar_amd.SC_Dec(fp, a.n)
model = channel.FusedAWGN(a.n, a.k, fp, dec, device=dev, seed=42)
no = float(channel.ebnodb2no(a.ebno, 2, a.k / a.n))
plan = dec.plan(dev)
counts = torch.zeros(2, dtype=torch.int64, device=dev)

# settle the clock
t = time.perf_counter()
while time.perf_counter() - t < 0.2:
    for i in range(20):
        ops.sc_sim_count(plan, a.bs, no, 1, i, 0, counts)
    torch.cuda.synchronize()

stream = torch.cuda.current_stream(dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(stream)
for i in range(a.iters):
    ops.sc_sim_count(plan, a.bs, no, 2, i, 0, counts)
e1.record(stream)
torch.cuda.synchronize()
kern = e0.elapsed_time(e1) / a.iters
print(f"({a.k},{a.n}) bs={a.bs}: kernel loop {kern:.4f} ms/iteration ({a.bs / kern / 1e3:.1f} Mcw/s)", flush=True)

for w in (None, 1):
    best = None
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, _, c = sim.sim_ber(model, np.array([a.ebno]), a.bs, max_mc_iter=a.iters, verbose=False, device="cuda",
                              return_counts=True, max_window=w)
        dt = (time.perf_counter() - t0) * 1e3 / a.iters
        assert int(c[0, 3]) == a.bs * a.iters
        best = dt if best is None else min(best, dt)
    label = f"max_window={w if w else sim.MAX_WINDOW}"
    print(f"  sim_ber {label}: {best:.4f} ms/iteration (best of 3; {best / kern:.3f} x kernel), "
          f"BLER {float(c[0, 1]) / float(c[0, 3]):.4f}", flush=True)
