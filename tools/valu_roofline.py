"""VALU-issue roofline inputs of the bench kernels, from rocprofv3 SQ passes (tools/prof_r04.sh or
tools/prof_r04_sq.sh) and the calibration kernels (tools/micro/valu_cycles.hip), into
profiles/valu.json -- what bench.py's roofline_valu reads.

  python tools/valu_roofline.py TAG DEC [DEC ...] --cal CAL_TXT      e.g.  r04k scl --cal profiles/r04f_valu_cycles.txt

For each decoder DEC the passes gpurun_out/TAG_sq_DEC_{A,B,C}.csv give per launch: SQ_INSTS_VALU
and its class counters (ADD/MUL/FMA/TRANS_F32, INT32, CVT, ADD/MUL/FMA_F64, INT64), the SALU /
LDS / SMEM counts and SQ_WAIT_ANY / SQ_WAVE_CYCLES.  The calibration (same-session microbenchmark,
8 waves per SIMD, settled clock) gives each form's issue cost in ns per wave-instruction per SIMD.
What the counters cannot split ("other": bitwise ops, bitop3, moves, DPP moves, compares, selects,
min/max -- measured 1.0 ... 1.8 ns) is carried as a range.  SQ_THREAD_CYCLES_VALU and
SQ_ACTIVE_INST_VALU are instruction counts on gfx950 (1 per instruction and lane / per
instruction; 2 for a transcendental -- the calibration kernels show it), so they give no busy
fraction independent of the instruction count and are not used for one.

Each entry records the kernel's pinned instruction-stream hash (tests/golden/kernel_isa.json):
bench.py reports the roofline only while the built kernel still has that stream.
"""
import argparse
import collections
import csv
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import sys  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "polar-code-pytorch-sionna_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
KERNELS = {"sc": "pl_sc_static_f32", "scl": "scl_tree_kernel<8, 4, 0, false>", "scx": "pl_sc_static_f32",
           "sclx": "scl_tree_kernel<8, 4, 1, true>"}
KEYS = {"sc": "sc_k512_n1024_bs65536", "scl": "scl_k512_n1024_bs8192_L8", "scx": "sc_exact_k512_n1024_bs65536",
        "sclx": "scl_exact_fast_k512_n1024_bs8192_L8"}
# scx: the built exact-f kernel's stream (tools/isa_walk.py); sclx: its pinned stream (kernel_isa.json)
PINS = {"sc": "sc_k512_n1024_minsum", "scl": "scl_L8_n1024_minsum", "scx": None, "sclx": "scl_L8_n1024_exact_fast"}
# counter class -> calibration form(s) whose cost it carries
CLASSES = {"SQ_INSTS_VALU_ADD_F32": "v_add_f32", "SQ_INSTS_VALU_MUL_F32": "v_mul_f32",
           "SQ_INSTS_VALU_FMA_F32": "v_fma_f32", "SQ_INSTS_VALU_TRANS_F32": "v_exp_f32",
           "SQ_INSTS_VALU_INT32": "v_add_u32", "SQ_INSTS_VALU_CVT": "v_cvt_f32_f64+f64_f32",
           "SQ_INSTS_VALU_ADD_F64": "v_add_f64", "SQ_INSTS_VALU_MUL_F64": "v_mul_f64",
           "SQ_INSTS_VALU_FMA_F64": "v_fma_f64", "SQ_INSTS_VALU_INT64": "v_fma_f64"}
OTHER = ("v_xor_b32", "v_mov_b32_dpp")  # cheapest and dearest measured form of the unsplit rest


def kname(raw):
    return re.sub(r"^(void )?(\(anonymous namespace\)::)?", "", raw.strip()).split("(")[0]


def per_launch(path, kernel):
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if kname(r["Kernel_Name"]) == kernel:
            d[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    if not d:
        raise SystemExit(f"{path}: no dispatch of {kernel}")
    keys = sorted({c for v in d.values() for c in v})
    return {c: sum(v[c] for v in d.values()) / len(d) for c in keys}, len(d)


def calibration(path):
    cal = {}
    for line in open(path):
        m = re.match(r"^(\S+)\s+([\d.]+) ns per wave-instruction per SIMD", line)
        if m:
            cal[m.group(1)] = float(m.group(2))
    return cal


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("decoders", nargs="+")
    ap.add_argument("--cal", required=True)
    a = ap.parse_args()
    cal = calibration(os.path.join(ROOT, a.cal) if not os.path.isabs(a.cal) else a.cal)
    pins = json.load(open(os.path.join(ROOT, "tests", "golden", "kernel_isa.json")))
    vj_path = os.path.join(ROOT, "profiles", "valu.json")
    vj = json.load(open(vj_path)) if os.path.exists(vj_path) else {}
    for dec in a.decoders:
        merged, n = {}, 0
        for p in "ABC":
            vals, n = per_launch(os.path.join(ROOT, "profiles", f"{a.tag}_sq_{dec}_{p}.csv"), KERNELS[dec])
            merged.update(vals)
        waves = merged["SQ_WAVES"]
        total = merged["SQ_INSTS_VALU"]
        classes = {c: merged.get(c, 0.0) for c in CLASSES}
        other = total - sum(classes.values())
        known_ns = sum(classes[c] * cal[CLASSES[c]] for c in classes)
        from polar_amd import build as _b
        import isa_walk
        keep = vj.get(KEYS[dec], {}).get("static")  # tools/isa_walk.py valu: kept across SQ refreshes
        if PINS[dec]:
            sha = pins[PINS[dec]]["sha"]
        elif dec == "scx":  # the exact-f SC kernel is not pinned: the built kernel's stream (tools/isa_walk.py)
            sha = isa_walk.isa_sha(isa_walk.kernel_asm(512, 1024, 1))
        else:
            sha = None
        vj[KEYS[dec]] = {
            "kernel": KERNELS[dec], "isa_sha": sha,
            # freshness keys bench.py checks: the exact-f SC code object's content-addressed name;
            # the sources of the SCL subtree kernel
            "code_object": isa_walk.code_object_name(512, 1024, 1) if dec == "scx" else None,
            "kernel_src_hash": _b.kernel_source_hash(_b.SCL_TREE_SOURCES) if dec in ("scl", "sclx") else None,
            "src_hash": _b.source_hash(), "dispatches": n, "waves_per_launch": waves,
            "valu_per_launch": total, "class_counts_per_launch": classes, "other_per_launch": other,
            "issue_ns_simd_per_launch": {"classified": known_ns, "other_lo": other * cal[OTHER[0]],
                                         "other_hi": other * cal[OTHER[1]]},
            "per_wave": {c.replace("SQ_", ""): round(v / waves, 1) for c, v in merged.items()
                         if c.startswith("SQ_") and c != "SQ_WAVES"},
            "calibration_ns": {CLASSES[c]: cal[CLASSES[c]] for c in CLASSES} | {f: cal[f] for f in OTHER},
            "source": [f"profiles/{a.tag}_sq_{dec}_{p}.csv" for p in "ABC"] + [a.cal],
        }
        if keep is not None:
            vj[KEYS[dec]]["static"] = keep
        print(dec, json.dumps(vj[KEYS[dec]]["issue_ns_simd_per_launch"]), "per wave VALU",
              round(total / waves, 1), "other", round(other / waves, 1))
    json.dump(vj, open(vj_path, "w"), indent=1)


if __name__ == "__main__":
    main()
