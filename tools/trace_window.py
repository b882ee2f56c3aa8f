"""The timed steps of one bench.py run, picked out of its rocprofv3 kernel trace.

  python tools/trace_window.py KERNEL_TRACE_CSV BENCH_JSON [--kernel pl_sc_static_f32 --marker awgn_llr_kernel]

bench.py launches, in order: the clock-settling steps and the --warmup steps, a shader-clock probe
(`--marker`, clock_kernel), the --steps timed steps (all the decode kernel), a second probe, then
per-launch timings and the other measurements.  So the timed steps are the decode launches between
the first two marker launches (traces without the probe: the `steps` decode launches before the
first launch of the Monte-Carlo producer, awgn_llr_kernel).  Prints their average / min / max duration,
the roofline fraction that average implies (algorithmic bytes from the bench line), and the
bench line's own HIP-event figure next to it.
"""
import argparse
import csv
import json
import re


def kname(raw):
    return re.sub(r"^(void )?(\(anonymous namespace\)::)?", "", raw.strip()).split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench_json")
    ap.add_argument("--kernel", default="pl_sc_static_f32")
    ap.add_argument("--marker", default="clock_kernel")
    a = ap.parse_args()
    line = json.loads([ln for ln in open(a.bench_json) if ln.startswith("{")][-1])
    steps = int(line["steps"])
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if kname(r["Kernel_Name"]) == a.marker]
    if len(marks) >= 2:
        dec = [r for r in rows[:marks[1]] if kname(r["Kernel_Name"]) == a.kernel]
        timed = [r for r in rows[marks[0]:marks[1]] if kname(r["Kernel_Name"]) == a.kernel]
    else:
        first = next((i for i, r in enumerate(rows) if kname(r["Kernel_Name"]) == "awgn_llr_kernel"), len(rows))
        dec = [r for r in rows[:first] if kname(r["Kernel_Name"]) == a.kernel]
        timed = dec[-steps:]
    assert len(timed) == steps, (len(dec), steps)
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in timed]  # us
    avg = sum(dur) / len(dur)
    span = (int(timed[-1]["End_Timestamp"]) - int(timed[0]["Start_Timestamp"])) / 1e3
    alg = line["roofline"].get("algorithmic_bytes_per_launch") or line.get("roofline_hbm", {}).get(
        "algorithmic_bytes_per_launch")
    out = {
        "kernel": a.kernel, "timed_launches": steps, "launches_before_window": len(dec) - steps,
        "avg_us": round(avg, 3), "min_us": round(min(dur), 3), "max_us": round(max(dur), 3),
        "window_span_us": round(span, 3), "span_per_step_us": round(span / steps, 3),
        "frac_from_trace_avg": round(alg / (avg * 1e-6) / 8.0e12, 5) if alg else None,
        "bench_kernel_ms": line["roofline"].get("kernel_ms"), "bench_frac": line["roofline"].get("frac"),
        "bench_ms_per_step": line["ms_per_step"],
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
