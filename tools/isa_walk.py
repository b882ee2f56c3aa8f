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
    taken (s_cbranch_scc1), loops left at their exit; in the exact-f functions the lane-divergent
    llr_max test's fast arm entered (s_cbranch_execnz after the s_xor_b64 of a saveexec) and its
    empty else arm skipped (after s_andn2_saveexec_b64).  Returns the instruction indices in order."""
    lab = {t: i for i, (k, t) in enumerate(ins) if k == "label"}
    pc, trace, prev, cmp43, masks43 = 0, [], "", False, set()
    while pc < len(ins) and len(trace) < 10 ** 6:
        k, t = ins[pc]
        if k == "label":
            pc += 1
            continue
        m = t.split()[0]
        trace.append(pc)
        if m.startswith("v_cmp"):  # the exact f's range test: llr_max against 43.0 (0x422c0000)
            cmp43 = m.startswith("v_cmp_ngt_f32") and any(
                ins[j][0] == "ins" and "0x422c0000" in ins[j][1] for j in range(max(0, pc - 6), pc))
            mm = re.match(r"v_cmp_ngt_f32_e64 (s\[\d+:\d+\])", t)
            if cmp43 and mm:  # the test hoisted into an SGPR pair (inlined f): each site ands it with exec
                masks43.add(mm.group(1))
        mm = re.match(r"s_and_b64 vcc, exec, (s\[\d+:\d+\])", t)
        if mm:
            cmp43 = mm.group(1) in masks43
        if m in ("s_endpgm", "s_setpc_b64"):
            break
        if m == "s_branch":
            pc = lab[t.split()[1]]
            prev = m
            continue
        if m.startswith("s_cbranch"):
            tgt = lab[t.split()[1]]
            if m in ("s_cbranch_vccz", "s_cbranch_vccnz") and cmp43:
                take = m == "s_cbranch_vccnz"  # the llr_max <= 43 test (exactf.h): true in every lane
            elif m == "s_cbranch_execnz":
                take = prev == "s_xor_b64" and tgt > pc
            elif m == "s_cbranch_execz":
                take = prev == "s_andn2_saveexec_b64"
            else:
                take = {"s_cbranch_scc1": True, "s_cbranch_execz": False, "s_cbranch_vccz": True,
                        "s_cbranch_vccnz": False}.get(m, tgt > pc)
            pc = tgt if take else pc + 1
            prev = m
            continue
        prev = m
        pc += 1
    return trace


def callees(ins, trace):
    """Counter of the functions the walked stream calls (s_swappc_b64 through a register pair set by
    s_getpc_b64 + s_add_u32 SYM@rel32@lo)."""
    pair, calls = {}, Counter()
    for i in trace:
        t = ins[i][1]
        mm = re.match(r"s_add_u32 s(\d+), s\d+, (\S+)@rel32@lo", t)
        if mm:
            pair[int(mm.group(1))] = mm.group(2)
        mm = re.match(r"s_swappc_b64 s\[30:31\], s\[(\d+):\d+\]", t)
        if mm:
            calls[pair.get(int(mm.group(1)), "?")] += 1
    return calls


def dynamic_histogram(asm, kernel):
    """Histogram of the walked kernel stream plus, per call, the walked stream of its callee."""
    ins = parse(asm, kernel)
    tr = walk(ins)
    h = histogram(ins, tr)
    for fn, c in callees(ins, tr).items():
        fi = parse(asm, fn)
        for m, v in histogram(fi, walk(fi)).items():
            h[m] += v * c
    return h, ins, tr


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
    """Mnemonic counts of the walked stream; a VOP2 select that directly follows another VOP2 select
    (the VALU before it) is counted as "v_cndmask_b32_e32:b2b": only that pairing issues slowly
    (tools/micro/cndmask_forms.hip)."""
    h, prev = Counter(), None
    for i in trace:
        m = ins[i][1].split()[0]
        if m.startswith("v_"):
            h[m + ":b2b" if m == prev == "v_cndmask_b32_e32" else m] += 1
            prev = m
        else:
            h[m] += 1
    return h


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
    "v_lshlrev_b16": "v_lshlrev_b32", "v_bitop3_b16": "v_bitop3_b32", "v_bfrev_b32": "v_bfe_u32",
    "v_cmp_gt_i64": "v_add_f64", "v_lshlrev_b64": "v_add_f64", "v_subrev_u32": "v_add_u32", "v_min3_u32": "v_min3_f32",
    "v_xor_b32_sdwa": "v_xor_b32_dpp", "v_lshlrev_b32_sdwa": "v_xor_b32_dpp",
    # fp64 and conversions (the exact-f kernels)
    "v_fma_f64": "v_fma_f64", "v_fmac_f64": "v_fma_f64", "v_mul_f64": "v_mul_f64", "v_add_f64": "v_add_f64",
    "v_ldexp_f64": "v_mul_f64", "v_cvt_f32_f64": "v_cvt_f32_f64+f64_f32", "v_cvt_f64_f32": "v_cvt_f32_f64+f64_f32",
    "v_cvt_f64_i32": "v_cvt_f32_f64+f64_f32", "v_cmp_ngt_f32": "v_cmp_eq_f32", "v_cmp_gt_f32": "v_cmp_eq_f32",
    "v_cmp_gt_i32": "v_cmp_eq_f32", "v_sub_f32_dpp": "v_add_f32_dpp", "v_subrev_f32_dpp": "v_add_f32_dpp",
    "v_max_f32": "v_min_f32", "v_med3_f32": "v_med3_f32", "v_cmp_nlt_f32": "v_cmp_eq_f32",
}
# VOP2 v_cndmask_b32_e32 (mask = VCC, implicit).  valu_cycles.hip times a run of them back to back
# at 9.4 ns per instruction (8 waves per SIMD), against 1.8 ns for the VOP3 form; in the kernels'
# patterns they cost what the VOP3 form costs (tools/micro/cndmask_forms.hip,
# profiles/r05f_cndmask_forms.txt: after a v_cmp 1.58 vs 1.57 ns per instruction, one per three adds
# 1.057 vs 1.056).  Two back to back after a v_cmp (the min/max swaps of the exact f: "cmp_sel2")
# add ~2.5 ns to the second; those (":b2b", 232 per wave in the exact-f SC kernel) are costed as the
# VOP3 form too, the difference below 0.5 % of that kernel's issue time.
E32_FORM = {"v_cndmask_b32_e32": "v_cndmask_b32", "v_cndmask_b32_e32:b2b": "v_cndmask_b32"}


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


def isa_sha(asm, kernel="pl_sc_static_f32"):
    """The instruction-stream hash tests/golden/kernel_isa.json pins (test_kernel_resources.isa_summary)."""
    import test_kernel_resources as t
    return t.isa_summary(asm, lambda nm: nm == kernel)[kernel]["sha"]


def code_object_name(k, n, fmode):
    """Cache file name of the specialised SC kernel of the reference (k, n) code (content-addressed:
    it changes exactly when the kernel's source does)."""
    import polar_amd
    from polar_amd import _lib
    fp = polar_amd.reference_frozen_pos(k, n).numpy()
    return _lib.sc_source(n, polar_amd.frozen_mask(fp, n), fmode)[1]


def record_valu(asm, tag, cal_path, sq_valu_per_wave=None, waves_per_launch=None, codewords_per_wave=None,
                normalise=False, code_object=None):
    """profiles/valu.json[tag]["static"]: the walked stream's VALU per wave by mnemonic, each with
    its calibrated issue cost (tools/micro/valu_cycles.hip), and the residual against the SQ
    counter (instructions the walk does not see: rare fallbacks) carried as a cost range."""
    cal = calibration(cal_path)
    # the calibration kernels and the decode kernel run at different clocks (DVFS: the fp64 forms at
    # ~2.13 GHz, the min-sum SC kernel at ~2.42): costs go to cycles at their own clock and back to
    # ns at the decode kernel's (profiles/clocks.json, tools/kernel_clock.py), when both are known
    # (off by default: the clocks come from profiled runs, whose kernels run ~10-15 % slower than the
    # clean calibration run; --clock-normalise applies them)
    clk_path = os.path.join(ROOT, "profiles", "clocks.json")
    clk = json.load(open(clk_path)) if (normalise and os.path.exists(clk_path)) else {}
    f_dec = clk.get("kernels_ghz", {}).get(tag)
    if f_dec:
        cal = {f: ns * clk["calibration_ghz"].get(f, f_dec) / f_dec for f, ns in cal.items()}
    h, ins, tr = dynamic_histogram(asm, "pl_sc_static_f32")
    by = {}
    mapped_ns, unmapped = 0.0, Counter()
    for m, c in sorted(h.items(), key=lambda x: -x[1]):
        if unit(m) != "valu":
            continue
        b = base_mnemonic(m)
        form = E32_FORM.get(m) if m in E32_FORM and E32_FORM[m] in cal else CAL_MAP.get(b)
        cost = cal.get(form) if form else None
        by[m] = [c, form, cost]
        if cost is None:
            unmapped[m] += c
        else:
            mapped_ns += c * cost
    walk_valu = sum(c for m, c in h.items() if unit(m) == "valu")
    plain = [v for k, v in cal.items() if k != "v_exp_f32" and not k.endswith("_vcc")]
    lo_c, hi_c = min(plain), max(plain)  # the rest: between the cheapest and the dearest plain form
    resid = (sq_valu_per_wave - walk_valu) if sq_valu_per_wave is not None else 0.0
    un = sum(unmapped.values())
    from polar_amd import build as _b
    rec = {"isa_sha": isa_sha(asm), "src_hash": _b.source_hash(), "code_object": code_object, "calibration": cal_path,
           "clock_normalised": bool(f_dec), "kernel_clock_ghz": f_dec, "valu_per_wave_walk": walk_valu,
           "valu_per_wave_sq": sq_valu_per_wave, "residual_per_wave": round(resid, 1),
           "issue_ns_per_wave": {"mapped": round(mapped_ns, 1),
                                 "rest_lo": round((un + max(resid, 0)) * lo_c, 1),
                                 "rest_hi": round((un + max(resid, 0)) * hi_c, 1)},
           "unmapped": dict(unmapped), "by_mnemonic": by,
           "units_per_wave": dict(Counter({unit(m): 0 for m in h}) + Counter({u: sum(c for m, c in h.items() if unit(m) == u) for u in ("valu", "salu", "lds", "vmem", "smem")})),
           "calls_per_wave": dict(callees(ins, tr)), "waves_per_launch": waves_per_launch,
           "codewords_per_wave": codewords_per_wave}
    path = os.path.join(ROOT, "profiles", "valu.json")
    vj = json.load(open(path)) if os.path.exists(path) else {}
    vj.setdefault(tag, {})["static"] = rec
    json.dump(vj, open(path, "w"), indent=1)
    return rec


def record_chain(asm, tag, lat_path, kernel_ms=None, code_object=None):
    """profiles/latency.json[tag]: the walked stream's longest register-dependence chain (cycles,
    chain_latency.hip's per-form latencies) and the in-order single-wave estimate, in us at the
    measured s_memtime clock, plus the back-to-back launch floor."""
    lat = latency_table(lat_path)
    clock = None
    for line in open(lat_path):
        mm = re.match(r"^s_memtime clock: ([\d.]+) GHz", line)
        if mm:
            clock = float(mm.group(1))
    ins = parse(asm)
    tr = walk(ins)
    longest, est = chain(ins, tr, lat)
    from polar_amd import build as _b
    rec = {"isa_sha": isa_sha(asm), "src_hash": _b.source_hash(), "code_object": code_object, "latency_table": lat_path,
           "instructions_per_wave": len(tr),
           "chain_cycles": round(longest, 1), "in_order_cycles": round(est, 1), "clock_ghz": clock,
           "chain_us": round(longest / clock / 1e3, 3) if clock else None,
           "in_order_us": round(est / clock / 1e3, 3) if clock else None,
           "launch_floor_us": {k[7:]: v for k, v in lat.items() if k.startswith("launch_")}}
    path = os.path.join(ROOT, "profiles", "latency.json")
    lj = json.load(open(path)) if os.path.exists(path) else {}
    lj[tag] = rec
    json.dump(lj, open(path, "w"), indent=1)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["hist", "valu", "chain"])
    ap.add_argument("--k", type=int, default=512)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--cal", default=None)
    ap.add_argument("--lat", default=None)
    ap.add_argument("--asm", default=None, help="read the assembly from this file instead of compiling")
    ap.add_argument("--fm", type=int, default=0, help="f mode of the plan (1: the exact boxplus f)")
    ap.add_argument("--tag", default=None, help="valu.json / latency.json key")
    ap.add_argument("--bs", type=int, default=65536)
    ap.add_argument("--cpw", type=int, default=None, help="codewords per wave (64 / lanes per codeword)")
    ap.add_argument("--clock-normalise", action="store_true", help="valu: costs onto the decode kernel's clock (profiles/clocks.json)")
    a = ap.parse_args()
    asm = open(a.asm).read() if a.asm else kernel_asm(a.k, a.n, a.fm)
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
        tag = a.tag or f"sc_k{a.k}_n{a.n}_bs{a.bs}"
        vj = json.load(open(os.path.join(ROOT, "profiles", "valu.json")))
        sq = vj.get(tag, {}).get("per_wave", {}).get("INSTS_VALU")
        if sq is not None and vj[tag].get("isa_sha") not in (None, isa_sha(asm)):
            sq = None  # the SQ pass counted another instruction stream
        waves = vj.get(tag, {}).get("waves_per_launch") or (a.bs // a.cpw if a.cpw else None)
        rec = record_valu(asm, tag, a.cal, sq, waves, a.cpw, a.clock_normalise,
                          None if a.asm else code_object_name(a.k, a.n, a.fm))
        print(json.dumps({k: rec[k] for k in ("valu_per_wave_walk", "valu_per_wave_sq", "issue_ns_per_wave", "unmapped")}))
        return
    if a.cmd == "chain":
        rec = record_chain(asm, a.tag or f"sc_k{a.k}_n{a.n}", a.lat,
                           code_object=None if a.asm else code_object_name(a.k, a.n, a.fm))
        print(json.dumps({k: v for k, v in rec.items() if k != "latency_table"}))


if __name__ == "__main__":
    main()
