"""Quick SC decode timing (development aid; bench.py is the contract)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "polar-code-pytorch-sionna_amd"))
import torch
import polar_amd
from polar_amd import _lib
FM = int(os.environ.get("SC_FMODE", "0"))  # 1: the exact-boxplus f (my_sn SC_Dec)
for (k, n, bs) in [(128, 256, 4096), (512, 1024, 65536), (32, 64, 65536), (1024, 2048, 32768)]:
    fp = polar_amd.reference_frozen_pos(k, n).numpy()
    plan = _lib.Plan(n, polar_amd.frozen_mask(fp, n), 1, FM)
    x = torch.randn((bs, n), device="cuda") * 2 + 1
    out = torch.empty((bs, k), device="cuda")
    for _ in range(3):
        polar_amd.ops.sc_decode(plan, x, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        polar_amd.ops.sc_decode(plan, x, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"SC f_mode={FM} kernel={plan.kernel()[0]} ({k},{n}) bs={bs}: {ms:.3f} ms  {bs / ms / 1e3:.2f} Mcw/s  {bs * k / ms / 1e6:.2f} Gbit/s info", flush=True)
