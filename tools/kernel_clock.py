"""Shader clock per kernel from a rocprofv3 run that collected GRBM_GUI_ACTIVE with --kernel-trace:
GRBM_GUI_ACTIVE counts busy cycles summed over the chip's 8 XCDs, so clock = cycles / 8 /
dispatch duration.  Writes profiles/clocks.json: the calibration kernels' clocks by form
(tools/micro/valu_cycles.hip) and the decode kernels' clocks by bench tag, which
tools/isa_walk.py uses to put the calibrated issue costs on the decode kernel's clock (the fp64
calibration kernels run at ~2.13 GHz, the min-sum SC kernel at ~2.42 GHz).

  python tools/kernel_clock.py TAG      (reads gpurun_out/TAG_valu_cycles_{pmc,trace}.csv and
                                         gpurun_out/TAG_sq_{sc,scx,scl}_B{,_trace}.csv)
"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
XCDS = 8
FORMS = {"k_add_f32": "v_add_f32", "k_fma_f32": "v_fma_f32", "k_xor_b32": "v_xor_b32", "k_dpp_add": "v_add_f32_dpp",
         "k_exp_f32": "v_exp_f32", "k_add_f64": "v_add_f64", "k_fma_f64": "v_fma_f64", "k_mul_f64": "v_mul_f64",
         "k_mul_f32": "v_mul_f32", "k_bitop3": "v_bitop3_b32", "k_add_u32": "v_add_u32", "k_min_f32": "v_min_f32",
         "k_cvt_f64": "v_cvt_f32_f64+f64_f32", "k_movdpp": "v_mov_b32_dpp", "k_min3": "v_min3_f32",
         "k_med3": "v_med3_f32", "k_pkadd": "v_pk_add_f32", "k_alignbit": "v_alignbit_b32", "k_lshl": "v_lshlrev_b32",
         "k_lshr": "v_lshrrev_b32", "k_bfe": "v_bfe_u32", "k_and": "v_and_b32", "k_mov": "v_mov_b32",
         "k_cvtub": "v_cvt_f32_ubyte0", "k_bcnt": "v_bcnt_u32_b32", "k_xordpp": "v_xor_b32_dpp",
         "k_anddpp": "v_and_b32_dpp", "k_minudpp": "v_min_u32_dpp", "k_addudpp": "v_add_u32_dpp",
         "k_cndmask": "v_cndmask_b32_vcc", "k_cndmask64": "v_cndmask_b32", "k_cmpeq": "v_cmp_eq_f32"}
TAGS = {"sc": "sc_k512_n1024_bs65536", "scx": "sc_exact_k512_n1024_bs65536", "scl": "scl_k512_n1024_bs8192_L8"}


def kname(raw):
    raw = re.sub(r"^(void )?(\(anonymous namespace\)::)?", "", raw.strip()).split("(")[0]
    return re.sub(r"^_Z\d+", "", raw)


def clocks(pmc, trace, keep):
    cyc, names = collections.defaultdict(float), {}
    for r in csv.DictReader(open(pmc)):
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            d = int(r["Dispatch_Id"])
            cyc[d] += float(r["Counter_Value"])
            names[d] = kname(r["Kernel_Name"])
    dur = {int(r["Dispatch_Id"]): int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(trace))}
    out = collections.defaultdict(list)
    for d, c in cyc.items():
        if d in dur and dur[d] > 0 and keep(names[d]):
            out[names[d]].append(c / XCDS / dur[d])
    return {k: round(sum(v) / len(v), 4) for k, v in out.items()}


def main(tag):
    g = os.path.join(ROOT, "gpurun_out")
    cal = clocks(os.path.join(g, f"{tag}_valu_cycles_pmc.csv"), os.path.join(g, f"{tag}_valu_cycles_trace.csv"),
                 lambda k: True)
    res = {"source": tag, "calibration_ghz": {}, "kernels_ghz": {}}
    for k, ghz in cal.items():
        for kn, form in FORMS.items():
            if k.startswith(kn) and (k == kn or not k[len(kn)].isalnum() or k[len(kn):].startswith("P")):
                res["calibration_ghz"][form] = ghz
    for dec, key in TAGS.items():
        pmc, tr = os.path.join(g, f"{tag}_sq_{dec}_B.csv"), os.path.join(g, f"{tag}_sq_{dec}_B_trace.csv")
        if os.path.exists(pmc) and os.path.exists(tr):
            c = clocks(pmc, tr, lambda k: k.startswith("pl_sc_static_f32") or "scl_tree_kernel" in k)
            if c:
                res["kernels_ghz"][key] = list(c.values())[0]
    json.dump(res, open(os.path.join(ROOT, "profiles", "clocks.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
