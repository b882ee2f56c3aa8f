"""CPU-side checks of the C-ABI library: it loads and exports every symbol include/*.h declares.

No compute calls here (there is no GPU in the build container).
"""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "polar_mi355x.h")


def _declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pl_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_expected_api():
    names = _declared()
    for must in ("pl_plan_create", "pl_plan_destroy", "pl_sc_decode", "pl_scl_decode", "pl_last_error_string"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from polar_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail(f"{_lib.LIB_PATH} not built (run __graft_entry__.build())")
    L = _lib.lib()
    for name in _declared():
        assert hasattr(L, name), f"{name} declared in include/polar_mi355x.h but not exported"
    assert set(_lib.EXPORTED_SYMBOLS) == set(_declared())
    assert L.pl_version().decode().startswith("polar_mi355x")


def test_library_targets_gfx950():
    from polar_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_plan_create_rejects_bad_arguments_without_gpu():
    # argument validation happens before any HIP call, so it is testable on the CPU
    import numpy as np
    from polar_amd import _lib
    L = _lib.lib()
    h = ctypes.c_void_p()
    mask = np.zeros(6, dtype=np.uint8)
    assert L.pl_plan_create(ctypes.byref(h), 6, mask.ctypes.data_as(ctypes.c_void_p), 1, 0, 30.0, 0) == _lib.PL_EINVAL
    assert b"power of two" in L.pl_last_error_string()
    mask = np.zeros(8, dtype=np.uint8)
    assert L.pl_plan_create(ctypes.byref(h), 8, mask.ctypes.data_as(ctypes.c_void_p), 3, 0, 30.0, 0) == _lib.PL_EINVAL
    assert L.pl_plan_create(ctypes.byref(h), 8, mask.ctypes.data_as(ctypes.c_void_p), 1, 7, 30.0, 0) == _lib.PL_EINVAL


def test_no_cpu_fallback_without_gpu():
    import torch
    import polar_amd
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    dec = polar_amd.SC_Dec(torch.arange(32), 64)
    with pytest.raises(RuntimeError):
        dec(torch.zeros(2, 64))


def test_specialised_kernel_compiles_without_gpu(tmp_path):
    """pl_sc_specialize runs hiprtc only (no HIP device): the code object lands in the cache dir
    and carries both entry points for gfx950."""
    import numpy as np
    from polar_amd import _lib
    L = _lib.lib()
    mask = np.zeros(32, dtype=np.uint8)
    mask[[0, 1, 2, 4, 8, 16, 3, 5, 6, 9, 10, 12]] = 1
    buf = ctypes.create_string_buffer(4096)
    rc = L.pl_sc_specialize(32, mask.ctypes.data_as(ctypes.c_void_p), 0, str(tmp_path).encode(), buf, 4096)
    assert rc == 0, L.pl_last_error_string()
    path = buf.value.decode()
    assert path.startswith(str(tmp_path)) and os.path.exists(path)
    blob = open(path, "rb").read()
    assert b"pl_sc_static_f32" in blob and b"pl_sc_static_u8" in blob and b"gfx950" in blob
    # content-addressed: the same code maps to the same file, a different one to another
    buf2 = ctypes.create_string_buffer(4096)
    assert L.pl_sc_specialize(32, mask.ctypes.data_as(ctypes.c_void_p), 0, str(tmp_path).encode(), buf2, 4096) == 0
    assert buf2.value == buf.value
    mask[31] = 1
    assert L.pl_sc_specialize(32, mask.ctypes.data_as(ctypes.c_void_p), 0, str(tmp_path).encode(), buf2, 4096) == 0
    assert buf2.value != buf.value


def test_inprocess_hiprtc_n128_reference_codes(tmp_path):
    """In-process hiprtc in a process that has imported torch (so torch's bundled libhiprtc /
    amd_comgr are the ones mapped) on n = 128 reference codes, both f modes: the round-2 segfault
    ("In-process hiprtc") does not recur -- the full sweep over the 93 codes with n <= 256,
    with the GPU initialised, is profiles/r04l_hiprtc_inprocess_*.txt."""
    import numpy as np
    import torch  # noqa: F401  (load order as in a torch process)
    from polar_amd import _lib, build as b
    L = _lib.lib()
    codes = [c for c in b.reference_codes() if len(c[0]) == 128]
    codes = [c for c in codes if c[1] == 1][:1] + [c for c in codes if c[1] == 0][:2]
    assert len(codes) == 3
    buf = ctypes.create_string_buffer(4096)
    for m, fm in codes:
        m = np.ascontiguousarray(m, dtype=np.uint8)
        rc = L.pl_sc_specialize(128, m.ctypes.data_as(ctypes.c_void_p), fm, str(tmp_path).encode(), buf, 4096)
        assert rc == 0, L.pl_last_error_string()
        assert b"pl_sc_static_f32" in open(buf.value.decode(), "rb").read()


def test_reference_codes_are_prebuilt():
    """build() pre-compiles the specialised kernels of every pinned reference code."""
    from polar_amd import build as b
    if not os.path.isdir(b.KCACHE):
        pytest.fail("polar_amd/kcache missing (run __graft_entry__.build())")
    assert len([f for f in os.listdir(b.KCACHE) if f.endswith(".co")]) >= len(b.reference_codes())


def test_list_plan_rejects_llr_max_above_700():
    # the SCL metric penalty (softplus.h) is evaluated for |z| <= 700
    import numpy as np
    from polar_amd import _lib
    L = _lib.lib()
    h = ctypes.c_void_p()
    mask = np.zeros(8, dtype=np.uint8)
    assert L.pl_plan_create(ctypes.byref(h), 8, mask.ctypes.data_as(ctypes.c_void_p), 4, 0, 701.0, 0) == _lib.PL_EINVAL
    assert b"700" in L.pl_last_error_string()


def test_sc_source_and_cache_name():
    """pl_sc_source: the specialised kernel's source embeds the code's node table, and the cache
    name is content-addressed (same code -> same name, another code or f_mode -> another)."""
    import numpy as np
    import polar_amd
    from polar_amd import _lib
    m = polar_amd.frozen_mask(polar_amd.reference_frozen_pos(512, 1024).numpy(), 1024)
    src, name = _lib.sc_source(1024, m, 0)
    assert "struct PlCode" in src and "PL_SC_STATIC_KERNELS(PlCode)" in src and "N = 1024" in src
    assert "LOG_G = 4" in src and "#define PL_SC_MINW 3" in src  # n/64 = 16 lanes per codeword at min-sum n=1024
    assert re.fullmatch(r"sc_[0-9a-f]{16}\.co", name)
    assert _lib.sc_source(1024, m, 0)[1] == name
    assert _lib.sc_source(1024, m, 1)[1] != name
    m2 = m.copy()
    m2[np.nonzero(m2 == 0)[0][0]] = 1
    assert _lib.sc_source(1024, m2, 0)[1] != name


def test_exact_f_code_objects_per_llr_max_range():
    """Exact-f codes have one source per llr_max range (exactf.h PL_EXF_RANGE): <= 43 the fast
    forms with the lane-level f inlined (n <= 1024), > 43 (f_mode | PL_F_WIDE_RANGE) the full-range
    forms; the two are different cache objects; the flag is refused for min-sum codes."""
    import ctypes

    import polar_amd
    from polar_amd import _lib
    m = polar_amd.frozen_mask(polar_amd.reference_frozen_pos(512, 1024).numpy(), 1024)
    fast, nf = _lib.sc_source(1024, m, _lib.PL_F_EXACT)
    wide, nw = _lib.sc_source(1024, m, _lib.PL_F_EXACT | _lib.PL_F_WIDE_RANGE)
    assert "#define PL_EXF_RANGE 1" in fast and "#define PL_SC_FLANE_INLINE 1" in fast
    assert "#define PL_EXF_RANGE 2" in wide and "PL_SC_FLANE_INLINE 1" not in wide
    assert nf != nw
    m2 = polar_amd.frozen_mask(polar_amd.reference_frozen_pos(1024, 2048).numpy(), 2048)
    src2, _ = _lib.sc_source(2048, m2, _lib.PL_F_EXACT)
    assert "#define PL_EXF_RANGE 1" in src2 and "PL_SC_FLANE_INLINE 1" not in src2  # n = 2048: out of line
    size = ctypes.c_size_t()
    name = ctypes.create_string_buffer(64)
    rc = _lib.lib().pl_sc_source(1024, m.ctypes.data_as(ctypes.c_void_p), _lib.PL_F_MINSUM | _lib.PL_F_WIDE_RANGE,
                                 None, 0, ctypes.byref(size), name, 64)
    assert rc == _lib.PL_EINVAL


def test_prebuilt_kernels_cover_the_reference_codes():
    """build() pre-compiles (hipcc --genco) every code the reference, the bench and the GPU tests
    use, so nothing compiles on the GPU box."""
    from polar_amd import _lib, build
    have = set(os.listdir(build.KCACHE)) if os.path.isdir(build.KCACHE) else set()
    missing = [len(m) for m, fm in build.reference_codes() if _lib.sc_source(len(m), m, fm)[1] not in have]
    assert not missing, f"{len(missing)} specialised kernels not pre-built (run __graft_entry__.build())"


def test_list_plan_limits_rejected_at_creation_without_gpu():
    """SCL at n = 2048 needs list_size <= 16 (LDS-resident list state): L = 32 is refused by
    pl_plan_create itself (PL_ENOTSUP, before any device call), and by the module constructors."""
    import numpy as np
    import torch
    import polar_amd
    from polar_amd import _lib, mysn
    L = _lib.lib()
    h = ctypes.c_void_p()
    mask = np.zeros(2048, dtype=np.uint8)
    mask[:1024] = 1
    assert L.pl_plan_create(ctypes.byref(h), 2048, mask.ctypes.data_as(ctypes.c_void_p), 32, 0, 30.0, 0) == \
        _lib.PL_ENOTSUP
    assert b"list_size" in L.pl_last_error_string()
    fp = torch.arange(1024)
    for cls in (polar_amd.SCL_Dec, mysn.SCL_Dec):
        with pytest.raises(ValueError):
            cls(fp, 2048, list_size=32)
    cls(fp, 2048, list_size=16)  # supported: no plan is built before the first forward
    with pytest.raises(ValueError):
        polar_amd.SC_Dec(torch.arange(2048), 4096)


def test_generated_source_names_compiler_and_flags():
    """The specialised kernel's source starts with the hipcc flags and the compiler the library
    was built with (both part of the cache name); compile_code_object takes its flags from there."""
    import numpy as np
    from polar_amd import _lib
    m = np.zeros(64, dtype=np.uint8)
    m[:32] = 1
    src, name = _lib.sc_source(64, m, 0)
    flags, compiler = _lib._source_header(src)
    assert "--genco" in flags and "--offload-arch=gfx950" in flags
    assert compiler and compiler in _lib.hipcc_version(_lib.hipcc_path())
    assert name.startswith("sc_") and name.endswith(".co")


def test_specialised_source_compiles_for_edge_codes():
    """The specialised SC kernel source (every entry: f32, u8 and decode+count) compiles for the
    edge codes a plan may be asked for -- k = 0, k = 1, k = n - 1, k = n -- at several n, both f
    modes (hipcc -fsyntax-only; the GPU tests only compile the codes they decode)."""
    import shutil
    import subprocess
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    from polar_amd import _lib
    hipcc = _lib.hipcc_path()
    if hipcc is None or shutil.which(hipcc) is None and not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    jobs = []
    for n in (2, 64, 1024, 2048):
        for kind in ("k0", "k1", "kn-1", "kn"):
            m = np.zeros(n, np.uint8)
            if kind == "k0":
                m[:] = 1
            elif kind == "k1":
                m[:-1] = 1
            elif kind == "kn-1":
                m[0] = 1
            for fm in (0, 1):
                jobs.append((n, kind, fm, m))
    tmp = tempfile.mkdtemp()

    def one(job):
        n, kind, fm, m = job
        src, _ = _lib.sc_source(n, m, fm)
        f = os.path.join(tmp, f"c_{n}_{kind}_{fm}.hip")
        open(f, "w").write(src)
        r = subprocess.run([hipcc, "--offload-arch=gfx950", "--cuda-device-only", "-fsyntax-only", "-std=c++17", f],
                           capture_output=True, text=True)
        return job[:3], r.returncode, r.stderr[-600:]
    with ThreadPoolExecutor(8) as ex:
        bad = [(j, e) for j, rc, e in ex.map(one, jobs) if rc]
    assert not bad, bad[:2]


DEV_HOOKS = ("PL_SC_DEFINES", "PL_SC_SOURCE", "PL_SC_LOG_G", "PL_SCL_VIRTUAL", "PL_SCL_TREE_FAST")


def test_release_library_has_no_development_hooks():
    """The A/B hooks (environment variables that replace kernel sources, change layouts or switch on
    wrong-result diagnostic macros) are compiled only into libpolar_mi355x_dev.so (-DPL_DEV=1):
    the release library does not even contain their names, so no environment can reach them."""
    from polar_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    for name in DEV_HOOKS:
        assert name.encode() not in blob, name
    assert b"PL_SC_SPECIALIZE" in blob  # the documented switch (generic kernel, equally exact) stays


def test_release_source_ignores_hook_environment(monkeypatch):
    """The specialised kernel's source (hence its cache key and code object) is the same with the
    development variables set as without them."""
    from polar_amd import _lib
    import polar_amd
    m = polar_amd.frozen_mask(polar_amd.reference_frozen_pos(512, 1024), 1024)
    want = _lib.sc_source(1024, m, 0)
    monkeypatch.setenv("PL_SC_DEFINES", "PL_SC_DIAG_NO_TREE=1")
    monkeypatch.setenv("PL_SC_SOURCE", HEADER)
    monkeypatch.setenv("PL_SC_LOG_G", "3")
    assert _lib.sc_source(1024, m, 0) == want
    assert "#define PL_DEV" not in want[0] and "PL_SC_DIAG_NO_TREE 1" not in want[0]


def test_diagnostic_macros_refuse_release_builds(tmp_path):
    """A diagnostic (wrong-result) macro without PL_DEV is a compile error in every kernel source."""
    import subprocess
    from polar_amd import build as b
    hipcc = b._hipcc()
    for src, macro in (("sc_static.h", "PL_SC_DIAG_NO_TREE"), ("scl_tree_kernel.hip", "PL_SCL_DIAG_SKIP_V"),
                       ("sc_kernel.hip", "PL_SC_DIAG_NOSTORE"), ("channel_kernel.hip", "PL_AWGN_DIAG")):
        r = subprocess.run([hipcc, "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only", "-x", "hip",
                            f"-D{macro}=1", f"-I{b.OBJ}", os.path.join(b.CSRC, src)],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode != 0 and "development builds" in r.stderr, (src, r.stderr[-500:])


def test_bench_valu_roofline_from_committed_counters():
    """bench.py's VALU-issue roofline: from profiles/valu.json (per-class SQ counters x calibrated
    issue costs), current while the profiled instruction stream is the pinned one, reported null
    (stale) once the kernel changes."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    for tag, ms in (("sc_k512_n1024_bs65536", 0.0814), ("scl_k512_n1024_bs8192_L8", 0.93)):
        rv = bench.valu_roofline(tag, ms)
        assert rv is not None and rv["stale"] is False, tag
        assert 0.3 < rv["frac_lo"] <= rv["frac"] <= rv["frac_hi"] < 1.0
        assert "busy_frac" not in rv
        for f in rv["counter_files"]:
            assert os.path.exists(os.path.join(ROOT, f)), f
    orig = bench.current_isa_sha
    bench.current_isa_sha = lambda tag: "0" * 16
    try:
        rv = bench.valu_roofline("sc_k512_n1024_bs65536", 0.0814)
        assert rv["stale"] is True and rv["frac"] is None
    finally:
        bench.current_isa_sha = orig


def test_bench_records_keyed_to_their_kernels():
    """bench.py record_fresh: a record that names a specialised SC code object is current exactly
    while the plan loads that object; the SCL subtree records follow the hash of their own sources;
    the committed exact-f SC, SCL and my_sn SCL records are current for the built tree."""
    import importlib.util
    import json
    import types
    spec = importlib.util.spec_from_file_location("bench_mod2", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from polar_amd import _lib
    import polar_amd
    m = polar_amd.frozen_mask(polar_amd.reference_frozen_pos(512, 1024).numpy(), 1024)
    name = _lib.sc_source(1024, m, _lib.PL_F_EXACT)[1]
    plan = types.SimpleNamespace(kernel=lambda: ("specialized", "/somewhere/kcache/" + name))
    other = types.SimpleNamespace(kernel=lambda: ("specialized", "/somewhere/kcache/sc_0000000000000000.co"))
    rec = {"code_object": name}
    assert bench.record_fresh(rec, "sc_exact_k512_n1024_bs65536", plan)
    assert not bench.record_fresh(rec, "sc_exact_k512_n1024_bs65536", other)
    vj = json.load(open(os.path.join(ROOT, "profiles", "valu.json")))
    assert bench.record_fresh(vj["sc_exact_k512_n1024_bs65536"]["static"], "sc_exact_k512_n1024_bs65536", plan)
    for tag in ("scl_k512_n1024_bs8192_L8", "scl_exact_fast_k512_n1024_bs8192_L8"):
        assert bench.record_fresh(vj[tag], tag), tag
    assert not bench.record_fresh({"kernel_src_hash": "0" * 16}, "scl_exact_fast_k512_n1024_bs8192_L8")
