"""Development aid: time the my_sn SCL configurations (exact f, fast-SCL, CRC) on the GPU.

  python tools/mysn_time.py [--n 1024 --k 512 --L 8 --bs 8192]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "polar-code-pytorch-sionna_amd"))
import torch  # noqa: E402

import polar_amd  # noqa: E402
from polar_amd import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--k", type=int, default=512)
    ap.add_argument("--L", type=int, default=8)
    ap.add_argument("--bs", type=int, default=8192)
    a = ap.parse_args()
    fp = polar_amd.reference_frozen_pos(a.k, a.n).numpy()
    mask = polar_amd.frozen_mask(fp, a.n)
    g = torch.Generator(device="cuda").manual_seed(5)
    llr = (torch.randn((a.bs, a.n), device="cuda", generator=g) * 2.5 + 1.0).contiguous()
    sys.path.insert(0, ROOT)
    from bench import _time_launches  # the bench's launch sequence (configs_3 of the JSON line)
    for name, fm, flags in (("minsum", 0, 0), ("exact", 1, 0), ("minsum+fast", 0, _lib.PL_PLAN_FAST_SCL),
                            ("exact+fast (my_sn default)", 1, _lib.PL_PLAN_FAST_SCL)):
        plan = _lib.Plan(a.n, mask, a.L, fm, flags=flags)
        out = torch.empty((a.bs, a.k), device="cuda")
        ws = ops.scl_workspace(plan, a.bs, llr.device)
        fn = lambda: ops.scl_decode(plan, llr, out=out, workspace=ws)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        # cold: 3 launches right after the first (what this tool reported until round 4: the GPU
        # clock has not left its idle state yet, and the module path allocated the workspace per call)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            ops.scl_decode(plan, llr, out=out)
        e1.record()
        torch.cuda.synchronize()
        cold = e0.elapsed_time(e1) / 3
        # settled: bench.py's sequence (50 ms of untimed launches, 3 warm-up, 20 timed)
        ms = _time_launches(fn, 20, 3, 50.0, llr.device)
        print(f"{name:28s} kernel={plan.kernel()[0]:12s} {ms:8.3f} ms  {a.bs / ms / 1e3:7.4f} Mcw/s"
              f"  (cold, 3 launches, workspace per call: {cold:.3f} ms)", flush=True)

if __name__ == "__main__":
    main()
