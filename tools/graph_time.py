"""Development aid (GPU box): back-to-back launches of the specialised SC kernel, eager vs
replayed from a captured HIP graph, at small batches where the launch gap is a large share of the
time (BASELINE configs[1]: (128,256), bs = 4096).  Also the empty-launch floor of the same two
ways, through a trivial torch kernel.

  python tools/graph_time.py [--k 128 --n 256 --bs 4096 --launches 200]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "polar-code-pytorch-sionna_amd"))


def main():
    import torch

    import polar_amd
    from polar_amd import _lib, channel, ops
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--bs", type=int, default=4096)
    ap.add_argument("--launches", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    fp = polar_amd.reference_frozen_pos(a.k, a.n)
    plan = _lib.Plan(a.n, polar_amd.frozen_mask(fp, a.n), 1, 0, flags=_lib.PL_PLAN_CACHE_ONLY)
    print("kernel:", plan.kernel()[0], flush=True)
    gen = torch.Generator(device=dev).manual_seed(42)
    model = channel.System_AWGN_model(a.n, a.k, channel.GpuEncoder(fp, a.n), None, device=dev, generator=gen)
    _, _, llr = model.llrs(a.bs, torch.tensor(2.0))
    llr = llr.contiguous()
    out = torch.empty((a.bs, a.k), device=dev)
    want = ops.sc_decode(plan, llr).clone()

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up on the capture stream
        for _ in range(3):
            ops.sc_decode(plan, llr, out=out)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(a.launches):
            ops.sc_decode(plan, llr, out=out)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    print("graph replay bit-exact:", bool(torch.equal(out, want)), flush=True)

    x = torch.zeros(1, device=dev)
    ge = torch.cuda.CUDAGraph()
    with torch.cuda.graph(ge):
        for _ in range(a.launches):
            x.add_(1.0)

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda.synchronize()
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.launches  # us per launch

    def eager():
        for _ in range(a.launches):
            ops.sc_decode(plan, llr, out=out)

    def eager_empty():
        for _ in range(a.launches):
            x.add_(1.0)
    for _ in range(2000):  # settle the clock
        ops.sc_decode(plan, llr, out=out)
    res = {"eager": [], "graph": [], "empty eager": [], "empty graph": []}
    for _ in range(a.rounds):
        res["eager"].append(timed(eager))
        res["graph"].append(timed(g.replay))
        res["empty eager"].append(timed(eager_empty))
        res["empty graph"].append(timed(ge.replay))
    for k, v in res.items():
        v = sorted(v)
        print(f"{k:12s} median {v[len(v) // 2]:.3f} us per launch  min {v[0]:.3f}  ({a.launches} launches, "
              f"(k={a.k}, n={a.n}) bs={a.bs})", flush=True)


if __name__ == "__main__":
    main()
