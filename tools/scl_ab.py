"""Same-process A/B timing of the SCL kernels (subtree vs generic) at one shape.

    python tools/scl_ab.py [--n 1024 --k 512 --L 8 --bs 8192 --reps 5]
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--f-mode", type=int, default=0)
    ap.add_argument("--kernels", default="subtree,generic")
    a = ap.parse_args()
    fp = polar_amd.reference_frozen_pos(a.k, a.n).numpy()
    g = torch.Generator(device="cuda").manual_seed(5)
    llr = torch.randn((a.bs, a.n), device="cuda", generator=g) * 2.5 + 1.0
    out = torch.empty((a.bs, a.k), device="cuda")
    res = {}
    for kern in a.kernels.split(","):
        flags = _lib.PL_PLAN_GENERIC if kern == "generic" else 0
        plan = _lib.Plan(a.n, polar_amd.frozen_mask(fp, a.n), a.L, a.f_mode, flags=flags)
        ops.scl_decode(plan, llr, out=out)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            ops.scl_decode(plan, llr, out=out)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.reps
        res[kern] = out.clone()
        print(f"{kern:8s} {plan.kernel()[0]:12s} n={a.n} k={a.k} L={a.L} bs={a.bs}: {ms:8.3f} ms/launch "
              f"{a.bs / ms / 1e3:8.4f} Mcw/s", flush=True)
    keys = list(res)
    if len(keys) == 2:
        print("bit-identical:", bool(torch.equal(res[keys[0]], res[keys[1]])))


if __name__ == "__main__":
    main()
