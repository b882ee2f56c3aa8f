"""Register and scratch budgets of the two bench kernels, read from hipcc's gfx950 assembly (CPU).

The measured throughput of both decoders rests on occupancy facts that a source change can break
silently (DESIGN.md sections 3.1 and 3.2):
  * the specialised SC kernel of the BASELINE code (512,1024) runs 4 waves per SIMD: <= 128 VGPRs,
    no VGPR spills, no scratch;
  * the SCL subtree kernel at L = 8 (min-sum, no fast-SCL: the bench kernel) runs 2 waves per SIMD
    with no VGPR spills and no scratch (each round-2 change was checked against this; spills cost
    5-20 % whenever they appeared).
The sources are compiled exactly as build() / the code-object cache compile them, to assembly only.
"""
import os
import re
import subprocess
import tempfile

import pytest

from polar_amd import build as _build

HIPCC = os.path.join(_build.ROCM, "bin", "hipcc")
pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")


def _kernel_meta(asm, name_pred):
    """{kernel name: {field: int}} from the amdhsa metadata of an assembly file."""
    out = {}
    for block in asm.split("  - .agpr_count")[1:]:
        m = re.search(r"\.name:\s+(\S+)", block)
        if not m or not name_pred(m.group(1)):
            continue
        fields = {}
        for key in ("vgpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size"):
            f = re.search(r"\." + key + r":\s+(\d+)", block)
            fields[key] = int(f.group(1)) if f else None
        out[m.group(1)] = fields
    return out


def _compile_asm(src_path, extra, workdir):
    out = os.path.join(workdir, "k.s")
    cmd = [HIPCC, f"--offload-arch={_build.ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", *extra,
           "--cuda-device-only", "-S", src_path, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return open(out).read()


_SCL_ASM = {}


def _scl_l8_asm():
    if "asm" not in _SCL_ASM:
        src = os.path.join(_build.CSRC, "scl_tree_kernel.hip")
        with tempfile.TemporaryDirectory() as td:
            _SCL_ASM["asm"] = _compile_asm(src, ["-DPL_SCL_TREE_L=8"], td)
    return _SCL_ASM["asm"]


def test_scl_bench_kernel_no_vgpr_spills_private_memory_is_the_vcache():
    """No VGPR spills.  Private memory (scratch) IS used: the per-lane virtual-node cache (VCache,
    stage-6 and stage-7 entries, <= 1616 B with the frame) lives there by design; the bound below
    is what this test permits."""
    asm = _scl_l8_asm()
    # scl_tree_kernel<L = 8, V = 4, f_mode = 0 (min-sum), FAST = false>: the kernel bench.py --decoder scl runs
    meta = _kernel_meta(asm, lambda n: "scl_tree_kernelILi8ELi4ELi0ELb0E" in n)
    assert len(meta) == 1, list(meta)
    (m,) = meta.values()
    assert m["vgpr_spill_count"] == 0, m
    # private memory: only the per-lane virtual node-of-64 cache (VCache: the stage-6 entries, 512 B,
    # A/B r04g 0.925 vs 0.978 ms; the stage-7 entries, 1 KB, A/B r04q 0.868 vs 0.893 ms) and the
    # 16-byte frame -- no register spills
    assert m["private_segment_fixed_size"] <= 1616, m
    assert m["vgpr_count"] <= 256, m  # amdgpu_waves_per_eu(2)


# exact-f subtree kernels at L = 8: (V, fast) -> (VGPR spills, private bytes) allowed.  Round 6:
# vvisit_ex's per-path levels use compile-time register indices (2.03 -> 1.80 ms for my_sn's
# default, bit-identical, profiles/r06v_vex_ab_mysn.txt); at V = 4 the pass's two 16-entry register
# blocks then leave the allocator short, and the fast kernel spills values of the per-(pass, item)
# set-up -- reloaded once per item, not per path (39 VGPRs with the polynomial exact f, 13 with the
# table-driven one).  Budgets: what the kernels spill as built.
_SCL_EXACT_BUDGET = {(3, "0"): (0, 560), (3, "1"): (0, 576), (4, "0"): (0, 560), (4, "1"): (13, 608)}


def test_scl_exact_f_kernels_spill_budget():
    """The exact-f (FM = 1) subtree kernels at n = 512 / 1024 (V = 3, 4) -- my_sn SCL_Dec's default
    (with and without fast-SCL) and Polar5GDecoder's list decoder: 2 waves per SIMD (<= 256 VGPRs),
    no spills at V = 3, at most the measured spills at V = 4; private memory = the VCache (512 B per
    lane), the frames of the out-of-line calls and those spills."""
    asm = _scl_l8_asm()
    for (v, fast), (spills, priv) in _SCL_EXACT_BUDGET.items():
        meta = _kernel_meta(asm, lambda n: f"scl_tree_kernelILi8ELi{v}ELi1ELb{fast}E" in n)
        assert len(meta) == 1, (v, fast, list(meta))
        (m,) = meta.values()
        assert m["vgpr_spill_count"] <= spills, (v, fast, m)
        assert m["private_segment_fixed_size"] <= priv, (v, fast, m)
        assert m["vgpr_count"] <= 256, (v, fast, m)


@pytest.mark.parametrize("L", [16, 32])
def test_scl_wide_list_minsum_kernels_have_no_spills(L):
    """The min-sum subtree kernels of the wider lists (one or two codewords per wave): no VGPR
    spills (the round-4 stage-7 cache spilled 38 VGPRs at L = 16 and is on at L <= 8 only)."""
    src = os.path.join(_build.CSRC, "scl_tree_kernel.hip")
    with tempfile.TemporaryDirectory() as td:
        asm = _compile_asm(src, [f"-DPL_SCL_TREE_L={L}"], td)
    meta = _kernel_meta(asm, lambda n: f"scl_tree_kernelILi{L}E" in n and "ELi0ELb" in n)
    assert len(meta) == 10, list(meta)  # V = 0..4, fast-SCL off / on
    for name, m in meta.items():
        assert m["vgpr_spill_count"] == 0, (name, m)


def test_sc_bench_kernel_fits_four_waves_per_simd():
    import polar_amd
    from polar_amd import _lib
    fp = polar_amd.reference_frozen_pos(512, 1024).numpy()
    src, _ = _lib.sc_source(1024, polar_amd.frozen_mask(fp, 1024), _lib.PL_F_MINSUM)
    flags, _ = _lib._source_header(src)
    extra = [f for f in flags if f not in ("--genco", "--no-gpu-bundle-output", "-O3", "-std=c++17",
                                           "-ffp-contract=off") and not f.startswith("--offload-arch")]
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "sc.hip")
        with open(path, "w") as f:
            f.write(src)
        asm = _compile_asm(path, extra, td)
    meta = _kernel_meta(asm, lambda n: n in ("pl_sc_static_f32", "pl_sc_static_sim"))
    assert set(meta) == {"pl_sc_static_f32", "pl_sc_static_sim"}, list(meta)
    for name, m in meta.items():
        assert m["vgpr_count"] <= 128, (name, m)  # 4 waves per SIMD (512 VGPRs per lane)
        assert m["vgpr_spill_count"] == 0, (name, m)
        assert m["private_segment_fixed_size"] == 0, (name, m)


def test_sc_exact_f_bench_kernel_spill_budget():
    """the exact-f specialised SC kernel of the BASELINE code (my_sn SC_Dec at
    (512,1024), the mysn_sc_exact bench line) runs 3 waves per SIMD (<= 168 VGPRs) and spills at
    most the 6 VGPRs it spilled at the end of round 5 (9 scratch instructions per wave, 32 B of
    private memory): more spills must show up here before they show up in the timing."""
    import polar_amd
    from polar_amd import _lib
    fp = polar_amd.reference_frozen_pos(512, 1024).numpy()
    src, _ = _lib.sc_source(1024, polar_amd.frozen_mask(fp, 1024), _lib.PL_F_EXACT)
    flags, _ = _lib._source_header(src)
    extra = [f for f in flags if f not in ("--genco", "--no-gpu-bundle-output", "-O3", "-std=c++17",
                                           "-ffp-contract=off") and not f.startswith("--offload-arch")]
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "sc.hip")
        with open(path, "w") as f:
            f.write(src)
        asm = _compile_asm(path, extra, td)
    meta = _kernel_meta(asm, lambda n: n == "pl_sc_static_f32")
    (m,) = meta.values()
    assert m["vgpr_count"] <= 168, m  # 3 waves per SIMD
    assert m["vgpr_spill_count"] <= 6, m
    assert m["private_segment_fixed_size"] <= 32, m


# ---- instruction-stream pins -------------------------------------------
# Static instruction counts by class and a hash of the mnemonic sequence of the two bench
# kernels, as hipcc emits them for gfx950.  A change of either kernel's code shows up here (and
# must be re-pinned on purpose: python tools/pin_isa.py), so a bench number can always be tied to
# the instruction stream that produced it; pl_version() carries the source hash on the box.
PIN_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kernel_isa.json")


def isa_summary(asm, label_pred):
    """{label: {"valu", "salu", "vmem", "lds", "smem", "dpp", "total", "sha"}} for the functions
    of `asm` whose label satisfies label_pred (body = label .. its .Lfunc_end)."""
    import hashlib
    out = {}
    lines = asm.split("\n")
    i = 0
    while i < len(lines):
        m = re.match(r"^([A-Za-z_.$][\w.$]*):", lines[i])
        if m and label_pred(m.group(1)) and not m.group(1).startswith(".L"):
            name, ops = m.group(1), []
            i += 1
            while i < len(lines) and not lines[i].startswith(".Lfunc_end"):
                t = lines[i].strip().split()
                if t and re.match(r"^[vsdgb][a-z0-9_]+$", t[0]) and not t[0].startswith("s_nop"):
                    ops.append(t[0] + ("_dpp" if ("row_" in lines[i] or "quad_perm" in lines[i]) else ""))
                i += 1
            c = {"valu": sum(o.startswith("v_") for o in ops), "salu": sum(o.startswith("s_") and not
                 o.startswith(("s_load", "s_buffer_load", "s_store")) for o in ops),
                 "vmem": sum(o.startswith(("global_", "buffer_", "scratch_")) for o in ops),
                 "lds": sum(o.startswith("ds_") for o in ops),
                 "smem": sum(o.startswith(("s_load", "s_buffer_load")) for o in ops),
                 "dpp": sum(o.endswith("_dpp") for o in ops), "total": len(ops),
                 "sha": hashlib.sha256("\n".join(ops).encode()).hexdigest()[:16]}
            out[name] = c
        i += 1
    return out


def sc_bench_asm(td):
    import polar_amd
    from polar_amd import _lib
    fp = polar_amd.reference_frozen_pos(512, 1024).numpy()
    src, _ = _lib.sc_source(1024, polar_amd.frozen_mask(fp, 1024), _lib.PL_F_MINSUM)
    flags, _ = _lib._source_header(src)
    extra = [f for f in flags if f not in ("--genco", "--no-gpu-bundle-output", "-O3", "-std=c++17",
                                           "-ffp-contract=off") and not f.startswith("--offload-arch")]
    path = os.path.join(td, "sc.hip")
    with open(path, "w") as f:
        f.write(src)
    return _compile_asm(path, extra, td)


def current_pins():
    with tempfile.TemporaryDirectory() as td:
        sc = isa_summary(sc_bench_asm(td), lambda n: n == "pl_sc_static_f32")
    scl = isa_summary(_scl_l8_asm(), lambda n: "scl_tree_kernelILi8ELi4ELi0ELb0E" in n)
    # my_sn SCL_Dec's default (exact f + fast-SCL; Polar5GDecoder's list decoder), the mysn_scl line
    sclx = isa_summary(_scl_l8_asm(), lambda n: "scl_tree_kernelILi8ELi4ELi1ELb1E" in n)
    assert len(sc) == 1 and len(scl) == 1 and len(sclx) == 1, (list(sc), list(scl), list(sclx))
    return {"sc_k512_n1024_minsum": list(sc.values())[0], "scl_L8_n1024_minsum": list(scl.values())[0],
            "scl_L8_n1024_exact_fast": list(sclx.values())[0]}


def test_bench_kernel_instruction_streams_are_pinned():
    import json
    want = json.load(open(PIN_PATH))
    got = current_pins()
    for key in got:
        assert got[key] == want[key], (key, got[key], want[key], "re-pin with: python tools/pin_isa.py")


def test_scl_vcache_entries_fit_for_release_virtual_stages():
    """the per-lane VCache has kVcEntries = 32 (item, path) entries.  Every release
    configuration (pick_v's V for n = 32 ... 1024, L = 2 ... 32) needs at most that many; larger
    virtual nodes exist only in development builds, where node_fg runs them uncached."""
    R = 4
    for S in range(5, 11):
        v = min(S - 1 - R, 4)
        if v == 4 and S != 10:
            v = 3
        v = max(v, 0)
        if v == 0:
            continue
        h = 1 << (S - 1 - v)  # elements per half of the first virtual node (stage SS + 1)
        for L in (2, 4, 8, 16, 32):
            cpw = 32 // L
            assert (cpw * h + 63) // 64 * L <= 32, (S, v, L)
    src = open(os.path.join(_build.CSRC, "scl_tree_kernel.hip")).read()
    assert "constexpr int kVcEntries = 32;" in src
