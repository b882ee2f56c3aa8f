"""Summarise one round's rocprofv3 --pmc passes (tools/prof_round.sh TAG) into
profiles/TAG_pmc_summary.csv and refresh profiles/traffic.json (the `traffic` bench.py reports).

  python tools/pmc_summary.py TAG [sc|scl ...]   (reads gpurun_out/TAG_pmc_{sc,scl}_{FETCH,WRITE}_SIZE.csv)

FETCH_SIZE is doubled for the HBM byte count, per MI355X_MICROARCH.md (gfx950 reports half of a
coalesced streaming read); counters are KB (x1024).
"""
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"sc": "pl_sc_static_f32", "scl": "scl_tree_kernel<8, 4, 0, false>", "sclx": "scl_tree_kernel<8, 4, 1, true>"}
KEYS = {"sc": "sc_k512_n1024_bs65536", "scl": "scl_k512_n1024_bs8192_L8", "sclx": "scl_exact_fast_k512_n1024_bs8192_L8"}
PINS = {"sc": "sc_k512_n1024_minsum", "scl": "scl_L8_n1024_minsum", "sclx": "scl_L8_n1024_exact_fast"}
ALG = {"sc": 65536 * (4 * 1024 + 4 * 512), "scl": 8192 * (4 * 1024 + 4 * 512), "sclx": 8192 * (4 * 1024 + 4 * 512)}


def mean_kb(path, kname):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            name = re.sub(r"^void \(anonymous namespace\)::", "", row["Kernel_Name"]).split("(")[0]
            if name == kname:
                vals.append(float(row["Counter_Value"]))
    return len(vals), (sum(vals) / len(vals) if vals else float("nan"))


def main(tag):
    out = os.path.join(ROOT, "gpurun_out")
    rows = [("bench", "kernel", "counter", "dispatches", "mean_kb_per_dispatch")]
    tj_path = os.path.join(ROOT, "profiles", "traffic.json")
    tj = json.load(open(tj_path))
    decs = sys.argv[2:] or list(KERNELS)  # a round may profile one decoder only
    for dec in decs:
        kname = KERNELS[dec]
        kb = {}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            n, m = mean_kb(os.path.join(out, f"{tag}_pmc_{dec}_{c}.csv"), kname)
            rows.append((dec, kname.replace(",", ""), c, n, m))
            kb[c] = m
        e = tj.setdefault(KEYS[dec], {"kernel": kname, "algorithmic_bytes_per_launch": ALG[dec],
                                      "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (tools/prof_pass.sh), "
                                              "KB x1024, FETCH_SIZE doubled as for the SC kernel."})
        # the instruction stream the counters were taken on (bench.py reports the traffic only
        # while the built kernel still has it)
        e["isa_sha"] = json.load(open(os.path.join(ROOT, "tests", "golden", "kernel_isa.json")))[PINS[dec]]["sha"]
        e["fetch_size_kb_per_launch"] = kb["FETCH_SIZE"]
        e["write_size_kb_per_launch"] = kb["WRITE_SIZE"]
        e["hbm_bytes_per_launch"] = int(round((2 * kb["FETCH_SIZE"] + kb["WRITE_SIZE"]) * 1024))
        e["note"] = re.sub(r"profiles/r01\w_pmc_summary\.csv", f"profiles/{tag}_pmc_summary.csv", e["note"])
        e["note"] = re.sub(r"tools/prof_round\.sh r01\w", f"tools/prof_round.sh {tag}", e["note"])
        e["source"] = [f"profiles/{tag}_pmc_summary.csv"]
    with open(os.path.join(ROOT, "profiles", f"{tag}_pmc_summary.csv"), "w", newline="") as f:
        csv.writer(f).writerows(rows)
    with open(tj_path, "w") as f:
        json.dump(tj, f, indent=1)
        f.write("\n")
    for r in rows:
        print(*r, sep=",")


if __name__ == "__main__":
    main(sys.argv[1])
