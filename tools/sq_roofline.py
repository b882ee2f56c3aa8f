"""Per-launch SQ counters of the bench kernels from one rocprofv3 --pmc pass, into
profiles/valu.json (what bench.py's VALU roofline reads) and a summary table.

  python tools/sq_roofline.py TAG DEC=CSV [DEC=CSV ...]     e.g.  r03c sc=gpurun_out/x.csv scl=gpurun_out/y.csv

The pass (tools/prof_r03.sh): rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES
SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 bench.py --decoder DEC --steps 5 --warmup 1.
Counters are chip totals per dispatch; SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES / SQ_WAIT_ANY count
quad-cycles (MI355X_MICROARCH.md, per-instruction cycle constants).  Every dispatch of the kernel
in the pass is averaged (the instruction counts are the same for every launch of one shape).
"""
import csv
import collections
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"sc": "pl_sc_static_f32", "scl": "scl_tree_kernel<8, 4, 0, false>"}
KEYS = {"sc": "sc_k512_n1024_bs65536", "scl": "scl_k512_n1024_bs8192_L8"}


def kname(raw):
    return re.sub(r"^(void )?(\(anonymous namespace\)::)?", "", raw.strip()).split("(")[0]


def per_dispatch(path, kernel):
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if kname(r["Kernel_Name"]) != kernel:
            continue
        d[int(r["Dispatch_Id"])][r["Counter_Name"]] = d[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + \
            float(r["Counter_Value"])
    return d


def main(tag, pairs):
    vj_path = os.path.join(ROOT, "profiles", "valu.json")
    vj = json.load(open(vj_path)) if os.path.exists(vj_path) else {}
    lines = []
    for dec, path in pairs:
        rows = per_dispatch(path, KERNELS[dec])
        if not rows:
            raise SystemExit(f"{path}: no dispatch of {KERNELS[dec]}")
        keys = sorted({c for v in rows.values() for c in v})
        mean = {c: sum(v[c] for v in rows.values()) / len(rows) for c in keys}
        w = mean["SQ_WAVES"]
        vj[KEYS[dec]] = {
            "kernel": KERNELS[dec], "dispatches": len(rows),
            "sq_insts_valu_per_launch": mean["SQ_INSTS_VALU"],
            "sq_active_inst_valu_per_launch": mean.get("SQ_ACTIVE_INST_VALU"),
            "waves_per_launch": w,
            "per_wave": {c: round(v / w, 1) for c, v in mean.items() if c.startswith("SQ_") and c != "SQ_WAVES"},
            "grbm_gui_active_per_launch": mean.get("GRBM_GUI_ACTIVE"),
            "source": f"profiles/{tag}_sq_{dec}.csv (rocprofv3 --pmc, tools/prof_r03.sh)",
        }
        lines.append(f"{dec} {KERNELS[dec]}: {len(rows)} dispatches, waves {w:.0f}, per wave " +
                     ", ".join(f"{c} {v / w:.1f}" for c, v in mean.items() if c != "SQ_WAVES"))
    json.dump(vj, open(vj_path, "w"), indent=1)
    open(os.path.join(ROOT, "profiles", f"{tag}_sq_summary.txt"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], [a.split("=", 1) for a in sys.argv[2:]])
