"""bench.py -- SC decode throughput on MI355X (BASELINE.json metric), 1..8 GPUs, one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Workload (BASELINE.json configs[2], and per GPU of configs[4]): SC decoding of (k=512, n=1024) polar
codewords, bs=65536 per GPU, AWGN LLRs at Eb/N0 = 2 dB (synthetic, generated on device with the
port of System_AWGN_model, seed 42+rank).  A step = one decode launch over one resident batch; the
steps cycle through --buffers distinct batches (default 3 for SC: 3 x 384 MB of LLRs and bits,
more than the 256 MB Infinity Cache), so every launch streams its LLRs from HBM as a Monte-Carlo
loop over fresh codewords would, rather than re-reading a batch the cache still holds.
Weak scaling: each rank decodes its own 65536 codewords (no data-path collective); ranks only
all_reduce the block-error counters (BLER) and the timing.

Reported: value = codewords decoded by all ranks / max-over-ranks wall time (Mcodewords/s);
roofline = algorithmic HBM bytes per launch (bs*(4n+4k): fp32 LLRs in, fp32 bits out) / average
launch time from HIP events on the decode stream, against 8.0 TB/s; cpu_baseline = the C oracle
(same algorithm, OpenMP) on host cores, rank 0 at N=1 only, bounded to ~10 s.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "polar-code-pytorch-sionna_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "Mcodewords/s + info-bit Gbit/s, SC n=1024 bs=65536 @1/2/4/8 GPU; BLER match"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, chip-level parameters (spec)
REF_BLER_2DB = 0.9999  # reference x_run SC BLER at (512,1024), 2.0 dB


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 1000 SC / 20 SCL)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 200 SC / 3 SCL)")
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="untimed launches before the warmup steps so the GPU clock leaves its idle state")
    ap.add_argument("--k", type=int, default=512)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--bs", type=int, default=None, help="codewords per GPU (default 65536 SC / 8192 SCL)")
    ap.add_argument("--ebno", type=float, default=2.0)
    ap.add_argument("--buffers", type=int, default=None,
                    help="distinct resident batches the steps cycle through (default 3 SC, 1 SCL)")
    ap.add_argument("--decoder", choices=["sc", "scl"], default="sc")
    ap.add_argument("--list-size", type=int, default=8)
    ap.add_argument("--fast-scl", action="store_true", help="SCL: fast-SCL pruning (my_sn SCL_Dec's default)")
    ap.add_argument("--fmode", type=int, default=0, choices=[0, 1],
                    help="f of the decoder: 0 min-sum (x_run SC_Dec / SCL_Dec, the headline), 1 the exact boxplus f "
                         "(my_sn SC_Dec / SCL_Dec; profiling runs)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sim-iteration", action="store_true",
                    help="skip the (untimed-region) Monte-Carlo iteration measurement of the fused producer")
    ap.add_argument("--dist", action="store_true",
                    help="create the process group even at world size 1 (rehearses the RCCL path on one GPU)")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the (untimed-region) lines of BASELINE.json configs[1] and configs[3]")
    a = ap.parse_args()
    if a.bs is None:
        a.bs = 65536 if a.decoder == "sc" else 8192  # BASELINE.json configs[2] / configs[3]
    if a.steps is None:
        a.steps = 1000 if a.decoder == "sc" else 20
    if a.warmup is None:
        a.warmup = 200 if a.decoder == "sc" else 3
    if a.buffers is None:
        a.buffers = 3 if a.decoder == "sc" else 1  # SCL is issue-bound (0.5 % of HBM): one batch
    return a


def cpu_model():
    """The host CPU's model name (lscpu, else /proc/cpuinfo)."""
    import subprocess
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(llr_host, fp, k, n, decoder, L, budget_s):
    """The pinned C oracle (port of the reference algorithm) on the host cores, bounded sample:
    all cores (OpenMP) and one core, each the best of 3 timed repetitions on the same LLR rows
    (BASELINE.md section 3)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.build()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    if decoder == "sc":
        fn = lambda x, t: oracle.sc_decode(x, fp, nthreads=t)  # noqa: E731
        big, small = llr_host[: min(len(llr_host), 65536)], llr_host[: min(len(llr_host), 4096)]
    else:
        fn = lambda x, t: oracle.scl_decode(x, fp, L, nthreads=t, lazy=True)  # noqa: E731
        big, small = llr_host[: min(len(llr_host), 4 * threads)], llr_host[: min(len(llr_host), 4)]

    def best_of_3(sample, t, budget):
        fn(sample[: min(len(sample), 256)], t)  # warm the thread pool and the caches
        best, done_all, t_all = 0.0, 0, 0.0
        for _ in range(3):
            done, t0 = 0, time.perf_counter()
            while True:
                fn(sample, t)
                done += len(sample)
                if time.perf_counter() - t0 >= budget / 3:
                    break
            dt = time.perf_counter() - t0
            best = max(best, done / dt)
            done_all, t_all = done_all + done, t_all + dt
        return best, done_all, t_all

    rate, done, dt = best_of_3(big, threads, 0.7 * budget_s)
    rate1, done1, dt1 = best_of_3(small, 1, 0.3 * budget_s)
    ref_note = ("reference x_run SC_Dec measured in the build container (8 Xeon threads): 0.00603 Mcodewords/s "
                "at this shape, 1 thread 0.00151 Mcodewords/s at bs=8192 (BASELINE.md \u00a72)") if decoder == "sc" \
        else ("reference x_run SCL_Dec (L=8) measured in the build container (8 Xeon threads): "
              "6.15e-06 Mcodewords/s at n=1024 (BASELINE.md \u00a72)")
    return {"value": round(rate / 1e6, 6), "unit": "Mcodewords/s", "cores": threads, "kind": "port",
            "best_of": 3, "cpu_model": cpu_model(),
            "sample": f"best of 3 repetitions over {done} codewords ({len(big)}-codeword batches of the same AWGN LLRs, "
                      f"(k={k},n={n}) {decoder.upper()}, oracle/polar_oracle.c OpenMP, {threads} threads) in {dt:.1f} s",
            "single_thread": {"value": round(rate1 / 1e6, 6), "unit": "Mcodewords/s", "cores": 1, "best_of": 3,
                              "sample": f"{done1} codewords ({len(small)}-codeword batches) in {dt1:.1f} s"},
            "reference_cpu_note": ref_note}


def sim_iteration(plan, fp, k, n, bs, ebno, dev, reps=20):
    """One Monte-Carlo iteration of the harness on this GPU, measured
    after the timed region: the fused producer (pl_awgn_qpsk_llr: bits, encoder, QPSK, AWGN,
    logits), the SC decode and the error counter (pl_count_errors), each by HIP events; and the
    two fused paths of FusedAWGN.error_counts, timed as whole iterations: pl_awgn_qpsk_llr_bits +
    pl_sc_decode_count (packed bits, decode and count in one kernel, no bit rows) and
    pl_sc_sim_count (the whole iteration inside the SC kernel, sim_ber's default path)."""
    from polar_amd import _lib, channel, ops
    enc = _lib.Plan(n, plan_mask(fp, n), 1, flags=_lib.PL_PLAN_GENERIC, device=dev)
    no = float(channel.ebnodb2no(ebno, 2, k / n))
    out = torch.empty((bs, k), dtype=torch.float32, device=dev)
    u, llr = ops.awgn_qpsk_llr(enc, bs, no, 42, 0)
    counts = torch.zeros(2, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    t = {}
    for name, fn in (("producer_ms", lambda: ops.awgn_qpsk_llr(enc, bs, no, 42, 1)),
                     ("decode_ms", lambda: ops.sc_decode(plan, llr, out=out)),
                     ("count_ms", lambda: ops.count_errors(u, out, counts=counts))):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        t[name] = round(e0.elapsed_time(e1) / reps, 5)
    tot = sum(t.values())
    res = {"mcw_s": round(bs / tot / 1e3, 2), **t,
           "note": "fused producer + SC decode + error count per iteration, one GPU, HIP events"}
    if plan.kernel()[0] == "specialized":
        it = [2]

        def fused_iter():
            ub, lf = ops.awgn_qpsk_llr_bits(enc, bs, no, 42, it[0])
            it[0] += 1
            ops.sc_decode_count(plan, lf, ub, counts)
        fused_iter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fused_iter()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / reps
        res["decode_count_path"] = {"mcw_s": round(bs / ms / 1e3, 2), "iteration_ms": round(ms, 5),
                                    "note": "pl_awgn_qpsk_llr_bits + pl_sc_decode_count"}
        try:
            ops.sc_sim_count(plan, bs, no, 42, 0, 0, counts)
        except _lib.PolarLibError:
            return res
        ws_bytes = int(_lib.lib().pl_sc_count_workspace_size(plan.handle, bs))
        ws = torch.empty((ws_bytes,), dtype=torch.uint8, device=dev)
        import ctypes
        L = _lib.lib()

        def sim_iter(i):
            _lib.check(L.pl_sc_sim_count(plan.handle, 42, i, 0, bs, no, ctypes.c_void_p(counts.data_ptr()),
                                         ctypes.c_void_p(ws.data_ptr()), ws_bytes, None, None,
                                         _lib.current_stream_ptr(dev)), "pl_sc_sim_count")
        sim_iter(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(reps):
            sim_iter(2 + i)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / reps
        res["sim_kernel_path"] = {"mcw_s": round(bs / ms / 1e3, 2), "iteration_ms": round(ms, 5),
                                  "note": "pl_sc_sim_count: bits, encoder, QPSK, AWGN, logits, SC decode and "
                                          "error count in one kernel, nothing but the counters in HBM "
                                          "(sim_ber's path)"}
    return res


def _time_launches(fn, steps, warmup, settle_ms, dev):
    """Average ms per call of fn() over `steps` back-to-back calls on the current stream (HIP
    events on that stream), after ~settle_ms of untimed calls (DVFS) and `warmup` more."""
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < settle_ms:
        for _ in range(20):
            fn()
        torch.cuda.synchronize(dev)
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / steps


def launch_stats(fn, launches, dev):
    """Per-launch kernel times of `launches` more back-to-back calls, each bracketed by its own pair
    of HIP events on the launch stream (after the mean's timed region, so that one is unperturbed):
    min and median ms, next to the mean the timed region gives.  An event between two launches
    costs each ~2-3 us of gap the back-to-back mean does not see, so these are reported only for
    launches much longer than that (the headline, configs_3 and the my_sn lines, not configs_1)."""
    stream = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(launches + 1)]
    ev[0].record(stream)
    for i in range(launches):
        fn()
        ev[i + 1].record(stream)
    torch.cuda.synchronize(dev)
    t = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(launches))
    return {"min_ms": round(t[0], 5), "median_ms": round(t[len(t) // 2], 5), "launches": launches}


def clock_ghz(dev):
    """The shader clock of one CU now (pl_clock_probe, on the decode stream: it runs right after the
    launches queued before it), or None if the probe is unavailable."""
    try:
        from polar_amd import ops
        return round(ops.shader_clock_ghz(dev), 4)
    except Exception:
        return None


def config_line(decoder, k, n, bs, L, ebno, dev, rank, steps, warmup, fmode=0, fast=False):
    """One more BASELINE.json configuration on this GPU, measured after the headline's timed
    region: kernel ms per launch (HIP events over back-to-back launches on one resident batch),
    Mcodewords/s, info Gbit/s, BLER, and the HBM roofline of the launch (bs (4n + 4k) bytes).
    fmode 1: the exact boxplus f (my_sn SC_Dec / SCL_Dec); fast: fast-SCL pruning (my_sn SCL_Dec's
    default, PL_PLAN_FAST_SCL)."""
    import polar_amd
    from polar_amd import _lib, channel, ops
    fp = polar_amd.reference_frozen_pos(k, n)
    plan = _lib.Plan(n, polar_amd.frozen_mask(fp, n), L, fmode, flags=_lib.PL_PLAN_FAST_SCL if fast else 0, device=dev)
    gen = torch.Generator(device=dev).manual_seed(1042 + rank)
    model = channel.System_AWGN_model(n, k, channel.GpuEncoder(fp, n), None, device=dev, generator=gen)
    with torch.no_grad():
        bits, _, llr = model.llrs(bs, torch.tensor(ebno, dtype=torch.float32))
    llr = llr.contiguous()
    out = torch.empty((bs, k), dtype=torch.float32, device=dev)
    ws = ops.scl_workspace(plan, bs, dev) if L > 1 else None
    if L > 1:
        fn = lambda: ops.scl_decode(plan, llr, out=out, workspace=ws)  # noqa: E731
    else:
        fn = lambda: ops.sc_decode(plan, llr, out=out)  # noqa: E731
    ms = _time_launches(fn, steps, warmup, 50.0, dev)
    ls = launch_stats(fn, min(steps, 50), dev) if ms > 0.05 else None
    nerr = int(torch.any(out != bits, dim=-1).sum().item())
    nbytes = bs * (4 * n + 4 * k)
    ach = nbytes / (ms * 1e-3) / 1e9
    res = {"workload": f"{'SCL' if L > 1 else 'SC'} decode (k={k}, n={n}), bs={bs}" + (f", L={L}" if L > 1 else "")
           + (", exact boxplus f (my_sn)" if fmode == 1 else "") + (", fast-SCL" if fast else ""),
           "kernel": plan.kernel()[0], "kernel_ms": round(ms, 5), "steps": steps,
           **({"kernel_min_ms": ls["min_ms"], "kernel_median_ms": ls["median_ms"]} if ls else {}),
           "mcw_s": round(bs / ms / 1e3, 3), "info_gbit_s": round(bs * k / ms / 1e6, 4),
           "dtype": "f64" if L > 1 else "f32", "bler": round(nerr / bs, 6),
           "roofline_hbm": {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(ach / HBM_PEAK_GBS, 5), "algorithmic_bytes_per_launch": nbytes}}
    return res, fn, plan, llr, out


def graph_line(fn, steps, dev, chain_us=None):
    """The same launches replayed from one captured HIP graph (polar_amd.ops.LaunchGraph): ms per
    launch, and the graph's own launch floor (the same number of empty kernels replayed), which
    replaces the eager floor in the critical-path bound."""
    from polar_amd import ops
    g = ops.LaunchGraph(fn, steps, dev)
    x = torch.zeros(1, device=dev)
    ge = ops.LaunchGraph(lambda: x.add_(1.0), steps, dev)

    def per_launch(graph):
        for _ in range(3):
            graph.replay()
        torch.cuda.synchronize(dev)
        st = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(5):
            graph.replay()
        e1.record(st)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / (5 * graph.launches)
    ms, floor_ms = per_launch(g), per_launch(ge)
    out = {"kernel_ms": round(ms, 5), "launches_per_graph": steps, "launch_floor_us": round(floor_ms * 1e3, 3)}
    if chain_us is not None:
        bound = chain_us / 1e3 + floor_ms
        out.update({"bound_ms": round(bound, 5), "frac": round(bound / ms, 4)})
    return out


def library_src_hash():
    """The source hash the loaded libpolar_mi355x.so was built from (pl_version)."""
    from polar_amd import _lib
    return _lib.lib().pl_version().decode().split()[-1]


def record_fresh(rec, tag, plan=None):
    """Whether a profiles/ record describes the kernel this run executes: the content-addressed
    code object name of a specialised SC kernel (changes exactly when its source does), the
    pinned instruction stream (tests/golden/kernel_isa.json), the sources of the SCL subtree
    kernel, or else the whole library's source hash."""
    if rec.get("code_object") and plan is not None:
        return os.path.basename(plan.kernel()[1]) == rec["code_object"]
    pin = current_isa_sha(tag)
    if pin:
        return rec.get("isa_sha") == pin
    if rec.get("kernel_src_hash"):
        from polar_amd import build as _b
        return rec["kernel_src_hash"] == _b.kernel_source_hash(_b.SCL_TREE_SOURCES)
    return rec.get("src_hash") == library_src_hash()


def latency_bound(tag, kern_ms, plan=None):
    """Independent critical-path bound of a batch that fills less than one wave per SIMD
    (profiles/latency.json, tools/isa_walk.py chain): the longest register-dependence chain of one
    wave's instruction stream, each edge weighted by the single-wave dependent latency
    tools/micro/chain_latency.hip measured for its form, plus the back-to-back launch floor of an
    empty kernel with the same grid.  frac = bound / measured kernel time (1.0: the launch costs no
    more than its dependent chain).  Also the in-order single-wave estimate (issue in program
    order after the sources are ready).  null when the record was made from other sources."""
    path = os.path.join(ROOT, "profiles", "latency.json")
    try:
        rec = json.load(open(path))[tag]
    except Exception:
        return None
    out = {"bound": "latency", "source": "profiles/latency.json", "chain_cycles": rec["chain_cycles"],
           "clock_ghz": rec["clock_ghz"], "latency_table": rec["latency_table"]}
    if not record_fresh(rec, tag, plan) or not rec.get("clock_ghz"):
        out.update({"stale": True, "frac": None})
        return out
    floor = rec["launch_floor_us"].get("256")
    bound_ms = (rec["chain_us"] + floor) / 1e3
    est_ms = (rec["in_order_us"] + floor) / 1e3
    out.update({"stale": False, "launch_floor_us": floor, "chain_us": rec["chain_us"], "bound_ms": round(bound_ms, 5),
                "in_order_estimate_ms": round(est_ms, 5), "achieved_ms": round(kern_ms, 5),
                "frac": round(bound_ms / kern_ms, 4), "frac_in_order": round(est_ms / kern_ms, 4)})
    return out


def plan_mask(fp, n):
    import polar_amd
    return polar_amd.frozen_mask(fp, n)


def valu_from_profiles(tag):
    """The VALU-issue inputs of this shape's kernel (profiles/valu.json, tools/valu_roofline.py),
    or None."""
    path = os.path.join(ROOT, "profiles", "valu.json")
    if not os.path.exists(path):
        return None
    try:
        return json.load(open(path)).get(tag)
    except Exception:
        return None


def current_isa_sha(tag):
    """The pinned instruction-stream hash of the bench kernel (tests/golden/kernel_isa.json, which
    tests/test_kernel_resources.py holds equal to the built kernel)."""
    pin = {"sc_k512_n1024_bs65536": "sc_k512_n1024_minsum", "scl_k512_n1024_bs8192_L8": "scl_L8_n1024_minsum",
           "scl_exact_fast_k512_n1024_bs8192_L8": "scl_L8_n1024_exact_fast"}.get(tag)
    try:
        return json.load(open(os.path.join(ROOT, "tests", "golden", "kernel_isa.json")))[pin]["sha"]
    except Exception:
        return None


def valu_roofline(tag, kern_ms, plan=None):
    """VALU-issue roofline of the kernel from its measured instruction mix: per launch, the SQ
    class counters (rocprofv3) times each class's issue cost (ns per wave-instruction per SIMD,
    calibrated by tools/micro/valu_cycles.hip at a settled clock), summed and spread over the
    1024 SIMDs, against the launch time measured here.  The instructions the counters leave
    unclassified (bitwise, bitop3, moves, DPP moves, compares, selects, min/max) cost 1.0 ... 1.8
    ns: frac_lo / frac_hi bound the fraction, frac is their mean.  No busy-cycle counter exists
    on gfx950 (SQ_ACTIVE_INST_VALU / SQ_THREAD_CYCLES_VALU count instructions), so none is reported.
    null fields when the profile was taken on another instruction stream than the built kernel's."""
    v = valu_from_profiles(tag)
    if v and "static" in v:
        st = v["static"]
        fresh = record_fresh(st, tag, plan)
        out = {"bound": "valu_issue", "unit": "us of VALU issue per SIMD per launch", "kernel_ms": round(kern_ms, 5),
               "method": "per-mnemonic: the walked instruction stream (tools/isa_walk.py) x calibrated issue cost per "
                         "form (tools/micro/valu_cycles.hip); the residual against SQ_INSTS_VALU as a cost range",
               "valu_per_wave_walk": st["valu_per_wave_walk"], "valu_per_wave_sq": st["valu_per_wave_sq"],
               "counter_files": v.get("source"), "calibration": st["calibration"], "stale": not fresh}
        if not fresh:
            out.update({"frac": None, "frac_lo": None, "frac_hi": None})
            return out
        waves = v.get("waves_per_launch") or st.get("waves_per_launch")
        ns = st["issue_ns_per_wave"]
        simd_ns = kern_ms * 1e6 * 1024
        lo = (ns["mapped"] + ns["rest_lo"]) * waves / simd_ns
        hi = (ns["mapped"] + ns["rest_hi"]) * waves / simd_ns
        out.update({"frac": round((lo + hi) / 2, 4), "frac_lo": round(lo, 4), "frac_hi": round(hi, 4),
                    "achieved": round((lo + hi) / 2 * kern_ms * 1e3, 2), "peak": round(kern_ms * 1e3, 2),
                    "wait_share_per_wave": round(v["per_wave"]["WAIT_ANY"] / v["per_wave"]["WAVE_CYCLES"], 4)
                    if "per_wave" in v and "WAIT_ANY" in v["per_wave"] and v.get("isa_sha") in (None, st.get("isa_sha"))
                    else None})  # the SQ pass's wait share, when it profiled this instruction stream
        return out
    if not v or "issue_ns_simd_per_launch" not in v:
        return None
    out = {"bound": "valu_issue", "unit": "us of VALU issue per SIMD per launch", "kernel_ms": round(kern_ms, 5),
           "valu_instr_per_launch": v["valu_per_launch"], "counter_files": v.get("source"),
           "isa_sha": v.get("isa_sha")}
    if not record_fresh(v, tag, plan):
        out.update({"stale": True, "frac": None, "frac_lo": None, "frac_hi": None})
        return out
    ns = v["issue_ns_simd_per_launch"]
    simd_ns = kern_ms * 1e6 * 1024
    lo = (ns["classified"] + ns["other_lo"]) / simd_ns
    hi = (ns["classified"] + ns["other_hi"]) / simd_ns
    out.update({"stale": False, "frac": round((lo + hi) / 2, 4), "frac_lo": round(lo, 4), "frac_hi": round(hi, 4),
                # achieved = VALU issue time per SIMD and launch (mean of the bounds), peak = the launch time
                "achieved": round((lo + hi) / 2 * kern_ms * 1e3, 2), "peak": round(kern_ms * 1e3, 2),
                "issue_us_per_simd": [round((ns["classified"] + ns["other_lo"]) / 1024 / 1e3, 2),
                                      round((ns["classified"] + ns["other_hi"]) / 1024 / 1e3, 2)],
                "wait_share_per_wave": round(v["per_wave"].get("WAIT_ANY", 0) / max(v["per_wave"].get("WAVE_CYCLES", 1), 1), 4)
                if "WAIT_ANY" in v["per_wave"] and "WAVE_CYCLES" in v["per_wave"] else None})
    return out


def traffic_from_profiles(tag, plan=None):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/traffic.json), if one
    exists for this shape and was measured on the kernel this run executes (its pinned instruction
    stream or code object, when the record names one); else None."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    try:
        rec = json.load(open(path)).get(tag, {})
    except Exception:
        return None
    if (rec.get("isa_sha") or rec.get("code_object")) and not record_fresh(rec, tag, plan):
        return None
    return rec.get("hbm_bytes_per_launch")


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one rank per GPU; PL_BENCH_BACKEND=gloo with more ranks than GPUs is the rehearsal of the
    # multi-GPU path on a one-GPU box (ranks share the card, gloo carries the collectives)
    gpu = local % max(torch.cuda.device_count(), 1)
    backend = None
    if world > 1 or a.dist:
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        backend = os.environ.get("PL_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)

    import polar_amd
    from polar_amd import _lib, channel, ops

    k, n, bs = a.k, a.n, a.bs
    fp = polar_amd.reference_frozen_pos(k, n)
    mask = polar_amd.frozen_mask(fp, n)
    L = a.list_size if a.decoder == "scl" else 1
    plan = _lib.Plan(n, mask, L, a.fmode, flags=_lib.PL_PLAN_FAST_SCL if (a.fast_scl and L > 1) else 0, device=dev)
    gen = torch.Generator(device=dev).manual_seed(42 + rank)
    model = channel.System_AWGN_model(n, k, channel.GpuEncoder(fp, n), None, device=dev, generator=gen)
    R = max(1, a.buffers)
    bitss, llrs, outs = [], [], []
    with torch.no_grad():
        for _ in range(R):  # R consecutive draws of the rank's stream: distinct codewords
            b_, _, l_ = model.llrs(bs, torch.tensor(a.ebno, dtype=torch.float32))
            bitss.append(b_)
            llrs.append(l_.contiguous())
            outs.append(torch.empty((bs, k), dtype=torch.float32, device=dev))
    bits, llr, out = bitss[0], llrs[0], outs[0]
    ws = ops.scl_workspace(plan, bs, dev) if a.decoder == "scl" else None
    cur = [0]

    def step():
        i = cur[0]
        cur[0] = (i + 1) % R
        if a.decoder == "sc":
            ops.sc_decode(plan, llrs[i], out=outs[i])
        else:
            ops.scl_decode(plan, llrs[i], out=outs[i], workspace=ws)

    # DVFS: a cold MI355X runs the first few ms of work at a lower clock (measured: 0.127 ms/launch
    # with 3 warmup steps vs 0.119 ms after ~0.1 s of load), so settle the clock first.
    t_settle = time.perf_counter()
    while (time.perf_counter() - t_settle) * 1e3 < a.settle_ms:
        for _ in range(50):
            step()
        torch.cuda.synchronize(dev)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    clk_before = clock_ghz(dev)  # the shader clock just before the timed region (after the warmup)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)  # the decode kernels launch on this stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(a.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    # this rank's time for its K steps (taken before the closing barrier, so the barrier's own
    # latency is not part of a rank's time; the max over ranks below is the job's time)
    wall = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    kern_ms = e0.elapsed_time(e1) / a.steps
    clk_after = clock_ghz(dev)  # ... and right after its last launch
    kstats = launch_stats(step, min(a.steps, 200), dev)

    cdev = dev if backend == "nccl" else torch.device("cpu")  # RCCL reduces device tensors, gloo host ones
    nerr = sum(int(torch.any(o != b, dim=-1).sum().item()) for o, b in zip(outs, bitss))
    blk = torch.tensor([nerr, bs * R], dtype=torch.int64, device=cdev)
    tmax = torch.tensor([wall], dtype=torch.float64, device=cdev)
    if dist is not None:
        dist.all_reduce(blk, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    wall = float(tmax.item())
    total_cw = bs * world * a.steps
    value = total_cw / wall / 1e6
    bytes_per_launch = bs * (4 * n + 4 * k)
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    tag = (f"{a.decoder}{'_exact' if a.fmode == 1 else ''}{'_fast' if (a.fast_scl and L > 1) else ''}_k{k}_n{n}_bs{bs}"
           + (f"_L{L}" if L > 1 else ""))
    sim_it = None
    if a.decoder == "sc" and a.fmode == 0 and not a.no_sim_iteration:
        sim_it = sim_iteration(plan, fp, k, n, bs, a.ebno, dev)
    configs = None
    if a.decoder == "sc" and a.fmode == 0 and not a.no_configs and (k, n, bs) == (512, 1024, 65536):
        # BASELINE.json configs[1] (k=128, n=256, bs=4096, SC) and configs[3] (k=512, n=1024,
        # L=8, bs=8192, SCL) on this GPU, after the headline's timed region
        c1, f1, p1, _, _ = config_line("sc", 128, 256, 4096, 1, a.ebno, dev, rank, 2000, 200)
        c1["roofline_latency"] = latency_bound("sc_k128_n256", c1["kernel_ms"], p1)
        # the same launches replayed from a captured HIP graph (the launch gap of a small batch)
        rl = c1["roofline_latency"]
        c1["graph"] = graph_line(f1, 200, dev, rl.get("chain_us") if rl and not rl.get("stale") else None)
        c3, _, p3, _, _ = config_line("scl", 512, 1024, 8192, 8, a.ebno, dev, rank, 20, 3)
        # the HBM bytes the SCL launch moves (its lane-private virtual-node cache)
        c3["roofline_hbm"]["traffic"] = traffic_from_profiles("scl_k512_n1024_bs8192_L8", p3)
        rv = valu_roofline("scl_k512_n1024_bs8192_L8", c3["kernel_ms"], p3)
        if rv is not None:
            c3["roofline_valu"] = rv
        # my_sn SC_Dec (the library API's default decoder, exact boxplus f) at the headline shape
        cx, _, px, _, _ = config_line("sc", 512, 1024, 65536, 1, a.ebno, dev, rank, 50, 10, fmode=1)
        rv = valu_roofline("sc_exact_k512_n1024_bs65536", cx["kernel_ms"], px)
        if rv is not None:
            cx["roofline_valu"] = rv
        # my_sn SCL_Dec's default (exact boxplus f + fast-SCL; also Polar5GDecoder's list decoder)
        cs, _, ps_, _, _ = config_line("scl", 512, 1024, 8192, 8, a.ebno, dev, rank, 10, 2, fmode=1, fast=True)
        cs["roofline_hbm"]["traffic"] = traffic_from_profiles("scl_exact_fast_k512_n1024_bs8192_L8", ps_)
        rv = valu_roofline("scl_exact_fast_k512_n1024_bs8192_L8", cs["kernel_ms"], ps_)
        if rv is not None:
            cs["roofline_valu"] = rv
        configs = {"configs_1": c1, "configs_3": c3, "mysn_sc_exact": cx, "mysn_scl": cs}
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.fmode == 0:
        cpu = cpu_baseline(llr.cpu().numpy(), fp.numpy(), k, n, a.decoder, L, a.cpu_seconds)
    if rank == 0:
        line = {
            "metric": (METRIC if a.fmode == 0 else "Mcodewords/s, exact-boxplus SC (my_sn SC_Dec)") if a.decoder == "sc"
                      else f"Mcodewords/s, SCL L={L} n={n}",
            "value": round(value, 4),
            "unit": "Mcodewords/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(wall / a.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if a.decoder == "sc" else "f64",  # SCL: fp64 LLRs and metrics (polar_scl.py:190-192)
            "data": f"synthetic AWGN LLRs, Eb/N0={a.ebno} dB, QPSK, generated on device (seed 42+rank)",
            "config": {"workload": f"{a.decoder.upper()} decode (k={k}, n={n}), bs={bs} per GPU"
                                   + (f", L={L}" if L > 1 else ""),
                       "k": k, "n": n, "bs_per_gpu": bs, "global_batch": bs * world, "resident_batches": R,
                       "kernel": plan.kernel()[0],
                       "parallelism": f"dp{world}"},
            "info_gbit_s": round(total_cw * k / wall / 1e9, 4),
            "bler": round(float(blk[0].item()) / float(blk[1].item()), 6),
            "bler_reference_at_ebno": REF_BLER_2DB if (a.decoder == "sc" and k == 512 and n == 1024 and a.ebno == 2.0) else None,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic_from_profiles(tag, plan),
                         "kernel_ms": round(kern_ms, 5), "kernel_min_ms": kstats["min_ms"],
                         "kernel_median_ms": kstats["median_ms"], "algorithmic_bytes_per_launch": bytes_per_launch},
            "kernel_ms_stats": dict(kstats, mean_ms=round(kern_ms, 5),
                                    note="mean: the timed region's HIP events over back-to-back launches; min / median: one "
                                         "event pair per launch over that many more launches after it (each pair adds "
                                         "~2-3 us of launch gap to its launch)"),
            "clock_ghz": {"before": clk_before, "after": clk_after,
                          "method": "pl_clock_probe: one wave's s_memtime cycles over s_memrealtime's 100 MHz ticks, "
                                    "launched on the decode stream right before and right after the timed region"},
            "cpu_baseline": cpu,
            "dist_backend": backend,
        }
        rv = valu_roofline(tag, kern_ms, plan)
        if a.decoder == "scl" and rv is not None:
            # the list decoder is bound by VALU issue and leaf latency (0.6 % of HBM): its roofline is
            # the VALU one, the HBM figure stays next to it
            line["roofline_hbm"] = line["roofline"]
            line["roofline"] = rv
        elif rv is not None:
            line["roofline_valu"] = rv
        if sim_it is not None:
            line["sim_iteration"] = sim_it
        if configs is not None:
            line.update(configs)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
