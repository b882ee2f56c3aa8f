"""Kernel durations of the bench line's extra configurations, from the same rocprofv3 kernel trace
(tools/prof_r04.sh): every dispatch of the SC / SCL kernels grouped by kernel and grid size --
(512,1024) x 65536 is the headline (16384 one-wave work-groups), (128,256) x 4096 configs[1] (256
work-groups; its single-wave latency probe: 1 work-group), the SCL L=8 kernel configs[3].

  python tools/trace_configs.py KERNEL_TRACE_CSV > out.json
"""
import csv
import json
import re
import statistics
import sys


def kname(raw):
    return re.sub(r"^(void )?(\(anonymous namespace\)::)?", "", raw.strip()).split("(")[0]


def grid(r):
    for key in ("Grid_Size_X", "Grid_Size", "grid_size"):
        if key in r and r[key]:
            return int(r[key])
    return -1


def main(path):
    groups = {}
    for r in csv.DictReader(open(path)):
        k = kname(r["Kernel_Name"])
        if not (k.startswith("pl_sc_static") or "scl_tree_kernel" in k):
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        groups.setdefault(f"{k} grid={grid(r)}", []).append(d)
    out = {}
    for key, ds in sorted(groups.items()):
        tail = ds[len(ds) // 2:]  # the later half: clock settled
        out[key] = {"dispatches": len(ds), "median_us_later_half": round(statistics.median(tail), 3),
                    "min_us": round(min(ds), 3), "mean_us_later_half": round(sum(tail) / len(tail), 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
