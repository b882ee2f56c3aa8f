"""Static analysis of the specialised SC kernel's instruction stream (gfx950 assembly from hipcc):
the common-path walk, its per-mnemonic histogram, a per-mnemonic VALU-issue roofline and a
single-wave dependent-chain bound.

  python tools/isa_walk.py hist  --k 512 --n 1024                 # walk + histogram vs the SQ counters
  python tools/isa_walk.py valu  --k 512 --n 1024 --cal CAL.txt   # per-mnemonic VALU issue (profiles/valu.json)
  python tools/isa_walk.py chain --k 128 --n 256 --lat LAT.txt    # one wave's critical path (profiles/latency.json)

The specialised kernel (csrc/sc_static.h) is a straight-line program of one code: its branches are
wave-uniform tests for rare cases (an exact-zero or tied LLR at a repetition / SPC node, a tail
wave's missing rows) whose common direction is known, so walking the assembly from the entry
with those directions gives the dynamic instruction stream of a full wave on typical input.  The
walk is checked against rocprofv3's SQ counters per wave (VALU, SALU, LDS, SMEM): at (512,1024)
it reproduces SALU, LDS and SMEM exactly and VALU to 0.7 % (the rest: rare fallbacks taken).
"""
import argparse
import json
import os
import re
import sys
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "polar-code-pytorch-sionna_amd"), os.path.join(ROOT, "tests")]


def kernel_asm(k, n, fmode=0):
    """gfx950 assembly of the specialised SC kernel of the reference code (k, n), compiled with the
    flags the plan's code object uses (tests/test_kernel_resources.py does the same)."""
    import polar_amd
    from polar_amd import _lib
    import test_kernel_resources as t
    fp = polar_amd.reference_frozen_pos(k, n).numpy()
    src, _ = _lib.sc_source(n, polar_amd.frozen_mask(fp, n), fmode)
    flags, _ = _lib._source_header(src)
    extra = [f for f in flags if f not in ("--genco", "--no-gpu-bundle-output", "-O3", "-std=c++17",
                                           "-ffp-contract=off") and not f.startswith("--offload-arch")]
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "sc.hip")
        open(path, "w").write(src)
        return t._compile_asm(path, extra, td)


def parse(asm, kernel="pl_sc_static_f32"):
    """[(kind, text)] of the kernel body: ('label', name) or ('ins', instruction text)."""
    lines = asm.split("\n")
    st = [i for i, l in enumerate(lines) if l.startswith(kernel + ":")][0]
    en = [i for i in range(st, len(lines)) if lines[i].strip().startswith(".Lfunc_end")][0]
    out = []
    for line in lines[st + 1:en]:
        t = line.split(";")[0].strip()
        if not t:
            continue
        if re.match(r"^\.L\w+:$", t):
            out.append(("label", t[:-1]))
        elif not t.startswith(".") and re.match(r"^(s|v|ds|global|buffer|scratch|flat)_", t):
            out.append(("ins", t))
    return out


def walk(ins):
    """The common path: rare-case tests skipped (s_cbranch_vccz taken, s_cbranch_vccnz not taken:
    the zero/tie fix-ups and the missing-row stores are guarded that way), the vector output path
    taken (s_cbranch_scc1), loops left at their exit.  Returns the instruction indices in order."""
    lab = {t: i for i, (k, t) in enumerate(ins) if k == "label"}
    pc, trace = 0, []
    while pc < len(ins) and len(trace) < 10 ** 6:
        k, t = ins[pc]
        if k == "label":
            pc += 1
            continue
        m = t.split()[0]
        trace.append(pc)
        if m == "s_endpgm":
            break
        if m == "s_branch":
            pc = lab[t.split()[1]]
            continue
        if m.startswith("s_cbranch"):
            tgt = lab[t.split()[1]]
            take = {"s_cbranch_scc1": True, "s_cbranch_execz": False, "s_cbranch_vccz": True,
                    "s_cbranch_vccnz": False}.get(m, tgt > pc)  # execnz: backward = loop (exit)
            pc = tgt if take else pc + 1
            continue
        pc += 1
    return trace


def unit(m):
    if m.startswith("v_"):
        return "valu"
    if m.startswith("ds_"):
        return "lds"
    if m.startswith("s_load") or m.startswith("s_buffer_load"):
        return "smem"
    if m.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if m in ("s_nop", "s_waitcnt", "s_endpgm", "s_barrier") or m.startswith(("s_cbranch", "s_branch", "s_set", "s_sleep")):
        return "ctl"
    return "salu"


def histogram(ins, trace):
    return Counter(ins[i][1].split()[0] for i in trace)


# mnemonic (suffix-stripped) -> calibration form of tools/micro/valu_cycles.hip
CAL_MAP = {
    "v_bitop3_b32": "v_bitop3_b32", "v_add_f32_dpp": "v_add_f32_dpp", "v_xor_b32": "v_xor_b32",
    "v_min3_f32": "v_min3_f32", "v_mov_b32_dpp": "v_mov_b32_dpp", "v_add_f32": "v_add_f32",
    "v_med3_f32": "v_med3_f32", "v_cmp_eq_f32": "v_cmp_eq_f32", "v_pk_add_f32": "v_pk_add_f32",
    "v_alignbit_b32": "v_alignbit_b32", "v_lshlrev_b32": "v_lshlrev_b32", "v_lshrrev_b32": "v_lshrrev_b32",
    "v_ashrrev_i32": "v_lshrrev_b32", "v_bfe_u32": "v_bfe_u32", "v_cvt_f32_ubyte0": "v_cvt_f32_ubyte0",
    "v_and_b32": "v_and_b32", "v_or_b32": "v_and_b32", "v_and_or_b32": "v_bitop3_b32", "v_or3_b32": "v_bitop3_b32",
    "v_cndmask_b32": "v_cndmask_b32", "v_min_u32_dpp": "v_min_u32_dpp", "v_min_u32": "v_min_f32",
    "v_bcnt_u32_b32": "v_bcnt_u32_b32", "v_add_u32_dpp": "v_add_u32_dpp", "v_add_u32": "v_add_u32",
    "v_sub_u32": "v_add_u32", "v_add_co_u32": "v_add_u32", "v_addc_co_u32": "v_add_u32", "v_xor_b32_dpp": "v_xor_b32_dpp",
    "v_and_b32_dpp": "v_and_b32_dpp", "v_mov_b32": "v_mov_b32", "v_cmp_eq_u32": "v_cmp_eq_f32",
    "v_cmp_ne_u32": "v_cmp_eq_f32", "v_cmp_le_u32": "v_cmp_eq_f32", "v_cmp_lt_i64": "v_add_f64",
    "v_cmp_le_i64": "v_add_f64", "v_cmp_ge_i64": "v_add_f64", "v_cmp_ne_u16": "v_cmp_eq_f32",
    "v_mov_b64": "v_add_f64", "v_lshrrev_b64": "v_add_f64", "v_lshl_add_u64": "v_add_f64",
    "v_readfirstlane_b32": "v_mov_b32", "v_readlane_b32": "v_mov_b32", "v_mul_u32_u24": "v_add_u32",
    "v_mad_u32_u24": "v_bitop3_b32", "v_lshl_or_b32": "v_bitop3_b32", "v_lshl_add_u32": "v_bitop3_b32",
    "v_add3_u32": "v_bitop3_b32", "v_not_b32": "v_xor_b32", "v_max_f32": "v_min_f32", "v_min_f32": "v_min_f32",
    "v_sub_f32": "v_add_f32", "v_mul_f32": "v_mul_f32", "v_cmp_gt_u32": "v_cmp_eq_f32", "v_cmp_lt_u32": "v_cmp_eq_f32",
}


def base_mnemonic(m):
    return re.sub(r"_e(32|64)$", "", m)


def calibration(path):
    cal = {}
    for line in open(path):
        mm = re.match(r"^(\S+)\s+([\d.]+) ns per wave-instruction per SIMD", line)
        if mm:
            cal[mm.group(1)] = float(mm.group(2))
    return cal


def valu_issue(hist, cal):
    """Per-wave VALU issue in ns (sum over mnemonics of count x calibrated cost) and the counts
    without a calibrated form (carried as a range)."""
    ns, unmapped, lo_c, hi_c = 0.0, Counter(), min(cal.values()), max(v for k, v in cal.items() if k != "v_exp_f32")
    for m, c in hist.items():
        if unit(m) != "valu":
            continue
        b = base_mnemonic(m)
        form = CAL_MAP.get(b)
        if form is None or form not in cal:
            unmapped[b] += c
        else:
            ns += c * cal[form]
    return ns, unmapped, lo_c, hi_c


# ---- one wave's dependent chain ------------------------------------------------------------
REG = re.compile(r"^-?\|?(v|s)\[(\d+):(\d+)\]\|?$|^-?\|?(v|s)(\d+)\|?$")
SPECIAL = {"vcc": ("vcc",), "vcc_lo": ("vcc",), "vcc_hi": ("vcc",), "exec": ("exec",), "exec_lo": ("exec",),
           "exec_hi": ("exec",), "m0": ("m0",), "scc": ("scc",)}


def regs(tok):
    """Register names a (comma-separated) operand token names."""
    tok = tok.strip()
    if tok in SPECIAL:
        return list(SPECIAL[tok])
    mm = REG.match(tok)
    if not mm:
        return []
    if mm.group(1):
        return [f"{mm.group(1)}{r}" for r in range(int(mm.group(2)), int(mm.group(3)) + 1)]
    return [f"{mm.group(4)}{mm.group(5)}"]


def operands(text):
    body = text.split(None, 1)[1] if " " in text or "\t" in text else ""
    toks = [t.strip() for t in body.split(",")] if body else []
    if toks:
        toks[-1] = toks[-1].split()[0]  # drop trailing modifiers (dpp controls, offsets, bitop3:...)
    return toks


def dst_src(text):
    """(destination registers, source registers) of one instruction, implicit VCC / SCC / M0 / EXEC
    included."""
    m = text.split()[0]
    toks = operands(text)
    rs = [regs(t) for t in toks]
    flat = lambda xs: [r for x in xs for r in x]  # noqa: E731
    if m.startswith(("global_store", "buffer_store", "scratch_store", "ds_write", "flat_store")):
        return [], flat(rs)
    if m.startswith("global_load_lds") or m.startswith("buffer_load_dword") and "lds" in text:
        return [], flat(rs) + ["m0"]
    if m.startswith(("s_cbranch_vcc")):
        return [], ["vcc"]
    if m.startswith("s_cbranch_scc"):
        return [], ["scc"]
    if m.startswith("s_cbranch_exec"):
        return [], ["exec"]
    if m in ("s_waitcnt", "s_nop", "s_branch", "s_endpgm", "s_barrier") or not toks:
        return [], []
    if m.startswith("v_cmp") and m.endswith("_e32"):
        return ["vcc"], flat(rs)
    if m.startswith("s_cmp") or m.startswith("s_bitcmp"):
        return ["scc"], flat(rs)
    d, srcs = rs[0], flat(rs[1:])
    if m.startswith(("v_addc_co", "v_subb_co", "v_subbrev_co")) and m.endswith("_e32"):
        return d + ["vcc"], srcs + ["vcc"]
    if m.startswith(("v_add_co", "v_sub_co", "v_subrev_co")) and m.endswith("_e32"):
        return d + ["vcc"], srcs
    if m.startswith("v_cndmask") and m.endswith("_e32"):
        return d, srcs + ["vcc"]
    if m.startswith(("v_addc_co", "v_subb_co")) and m.endswith("_e64"):
        return d + rs[1], flat(rs[2:])
    if m.startswith("s_") and not m.startswith(("s_mov", "s_load", "s_buffer")):
        return d + ["scc"], srcs
    return d, srcs


def latency_table(path):
    """cycles per dependent instruction by form (tools/micro/chain_latency.hip output)."""
    lat = {}
    for line in open(path):
        mm = re.match(r"^(\S.*?)\s+([\d.]+) s_memtime cycles per dependent instruction", line)
        if mm:
            lat[mm.group(1).strip()] = float(mm.group(2))
        mm = re.match(r"^empty kernel,\s+(\d+) blocks\s+([\d.]+) us per back-to-back launch", line)
        if mm:
            lat[f"launch_{mm.group(1)}"] = float(mm.group(2))
    return lat


def inst_latency(m, lat):
    """Cycles from issue to result of one instruction (the chain_latency forms; memory by kind)."""
    if m.startswith("ds_bpermute") or m.startswith("ds_permute") or m.startswith("ds_swizzle"):
        return lat["ds_bpermute_b32"]
    if m.startswith("ds_read"):
        return lat["ds_read_b32"]
    if m.startswith(("global_load", "buffer_load", "scratch_load")):
        return lat["global_load (L2)"]
    if m.startswith("s_load"):
        return lat.get("s_load", 200.0)
    if m.startswith("v_"):
        b = base_mnemonic(m)
        if "_dpp" in b:
            return lat["s_nop1+v_add_f32_dpp"] - 2.0  # the chain form includes its s_nop 1
        if b.startswith(("v_cmp", "v_cndmask")):
            return lat["v_cmp+v_cndmask"] / 2.0
        if b.endswith("_f64") or b.endswith("_u64") or b.endswith("_b64") or b.endswith("_i64"):
            return lat["v_fma_f64"]
        if b.startswith("v_pk_"):
            return lat["v_pk_add_f32"]
        for form in ("v_bitop3_b32", "v_min3_f32", "v_med3_f32", "v_alignbit_b32"):
            if b.startswith(form.split("_")[0] + "_" + form.split("_")[1]):
                return lat[form]
        return lat["v_add_f32"]
    return 2.0  # SALU


def chain(ins, trace, lat):
    """Longest latency-weighted dependency chain through the walked instruction stream (register
    data dependences only: a lower bound on one wave's time), and the in-order single-wave estimate
    (issue in program order, each instruction after its sources are ready and the previous one has
    issued; s_nop N costs N + 1 cycles, s_waitcnt waits for the counted memory operations)."""
    ready = {}
    depth = {}  # register -> chain length (cycles) of the value it holds
    longest = 0.0
    t = 0.0
    vm, lgkm = [], []  # completion times of outstanding memory operations (in issue order)
    for i in trace:
        text = ins[i][1]
        m = text.split()[0]
        d, s_ = dst_src(text)
        if m == "s_nop":
            t += int(text.split()[1], 0) + 1
            continue
        if m == "s_waitcnt":
            for part in text.split()[1:]:
                mm = re.match(r"(vmcnt|lgkmcnt)\((\d+)\)", part)
                if mm:
                    q = vm if mm.group(1) == "vmcnt" else lgkm
                    keep = int(mm.group(2))
                    while len(q) > keep:
                        t = max(t, q.pop(0))
            continue
        lt = inst_latency(m, lat)
        start = max([t] + [ready.get(r, 0.0) for r in s_])
        dep = max([0.0] + [depth.get(r, 0.0) for r in s_]) + lt
        done = start + lt
        for r in d:
            ready[r] = done
            depth[r] = dep
        longest = max(longest, dep)
        if unit(m) == "vmem" and not m.startswith(("global_store", "buffer_store", "scratch_store")):
            vm.append(done)
        elif unit(m) == "vmem":
            vm.append(start + 8.0)  # stores: counted by vmcnt too, complete early for the wave
        elif unit(m) in ("lds", "smem"):
            lgkm.append(done)
        t = start + (1.0 if unit(m) in ("salu", "ctl") else 4.0 if unit(m) == "valu" else 4.0)
    end = max([t] + vm + lgkm)
    return longest, end


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["hist", "valu", "chain"])
    ap.add_argument("--k", type=int, default=512)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--cal", default=None)
    ap.add_argument("--lat", default=None)
    ap.add_argument("--asm", default=None, help="read the assembly from this file instead of compiling")
    a = ap.parse_args()
    asm = open(a.asm).read() if a.asm else kernel_asm(a.k, a.n)
    ins = parse(asm)
    trace = walk(ins)
    hist = histogram(ins, trace)
    units = Counter()
    for m, c in hist.items():
        units[unit(m)] += c
    if a.cmd == "hist":
        print(json.dumps(dict(units)))
        for m, c in hist.most_common():
            print(f"{m:28s} {c}")
        return
    if a.cmd == "valu":
        cal = calibration(a.cal)
        ns, unmapped, lo_c, hi_c = valu_issue(hist, cal)
        print(json.dumps({"valu_per_wave_walk": units["valu"], "issue_ns_per_wave_mapped": round(ns, 1),
                          "unmapped": dict(unmapped), "unmapped_cost_range_ns": [lo_c, hi_c]}))
        return
    if a.cmd == "chain":
        lat = latency_table(a.lat)
        longest, est = chain(ins, trace, lat)
        print(json.dumps({"instructions": len(trace), "chain_cycles": round(longest, 1),
                          "in_order_cycles": round(est, 1), "launch_floor_us": {k: v for k, v in lat.items() if k.startswith("launch")}}))


if __name__ == "__main__":
    main()
