"""ctypes binding of libpolar_mi355x.so (the C ABI in include/polar_mi355x.h).

`import torch` happens before the CDLL load so that libamdhip64.so.7 resolves to the HIP runtime
torch already loaded (same SONAME), i.e. one runtime, one device context, torch's streams usable
as hipStream_t.  There is no CPU fallback: if the library or a GPU is missing, every decode call
raises.
"""
import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpolar_mi355x.so")

PL_OK, PL_EINVAL, PL_EHIP, PL_ENOTSUP = 0, -1, -2, -3
PL_F_MINSUM, PL_F_EXACT = 0, 1
PL_F_WIDE_RANGE = 0x100  # sc_source / pl_sc_specialize: the exact-f code object of plans with llr_max > 43
PL_OUT_F32, PL_OUT_U8 = 0, 1
PL_PLAN_GENERIC, PL_PLAN_CACHE_ONLY, PL_PLAN_FAST_SCL, PL_PLAN_JIT = 1, 2, 4, 8
PL_KERNEL_GENERIC, PL_KERNEL_SPECIALIZED, PL_KERNEL_SCL_SUBTREE = 0, 1, 2

_lock = threading.Lock()
_lib = None


class PolarLibError(RuntimeError):
    """A failed C-ABI call; .code = its return code (PL_EHIP, PL_ENOTSUP, ...)."""

    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


def _declare(L):
    P, i32, i64, u32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32
    L.pl_plan_create.argtypes = [ctypes.POINTER(P), i32, P, i32, i32, ctypes.c_float, u32]
    L.pl_plan_destroy.argtypes = [P]
    L.pl_plan_info.argtypes = [P, P, P, P]
    L.pl_plan_device.argtypes = [P, P]
    L.pl_sc_decode.argtypes = [P, P, i64, P, i32, P]
    L.pl_scl_workspace_size.argtypes = [P, i64]
    L.pl_scl_workspace_size.restype = ctypes.c_size_t
    L.pl_scl_decode.argtypes = [P, P, i64, P, i32, P, P, ctypes.c_size_t, P]
    L.pl_polar_encode.argtypes = [P, P, i64, P, P]
    L.pl_plan_kernel.argtypes = [P, P, ctypes.c_char_p, ctypes.c_size_t]
    L.pl_plan_set_crc.argtypes = [P, i32, u32]
    L.pl_sc_specialize.argtypes = [i32, P, i32, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
    L.pl_sc_source.argtypes = [i32, P, i32, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                               ctypes.c_char_p, ctypes.c_size_t]
    L.pl_crc_attach.argtypes = [P, i64, i32, P, i32, P, P]
    L.pl_crc_check.argtypes = [P, i64, i32, P, i32, P, P]
    L.pl_gather_rows.argtypes = [P, i64, i32, P, i32, P, P]
    L.pl_rate_recover.argtypes = [P, i64, i32, P, P, P, i32, P, P]
    L.pl_awgn_qpsk_llr.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64, i64, i64, ctypes.c_float, P, P, P]
    L.pl_count_errors.argtypes = [P, P, i64, i32, P, P]
    L.pl_awgn_qpsk_llr_bits.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64, i64, i64, ctypes.c_float, P, P, P]
    L.pl_sc_count_workspace_size.argtypes = [P, i64]
    L.pl_sc_count_workspace_size.restype = ctypes.c_size_t
    L.pl_sc_decode_count.argtypes = [P, P, i64, P, P, P, ctypes.c_size_t, P]
    L.pl_sc_sim_count.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64, i64, i64, ctypes.c_float, P, P,
                                  ctypes.c_size_t, P, P, P]
    L.pl_clock_probe.argtypes = [P, i32, P]
    L.pl_last_error_string.restype = ctypes.c_char_p
    L.pl_version.restype = ctypes.c_char_p
    for f in (L.pl_plan_create, L.pl_plan_destroy, L.pl_plan_info, L.pl_plan_device, L.pl_sc_decode, L.pl_scl_decode,
              L.pl_polar_encode, L.pl_plan_kernel, L.pl_sc_specialize, L.pl_sc_source, L.pl_plan_set_crc,
              L.pl_crc_attach, L.pl_crc_check,
              L.pl_gather_rows, L.pl_rate_recover, L.pl_awgn_qpsk_llr, L.pl_count_errors,
              L.pl_awgn_qpsk_llr_bits, L.pl_sc_decode_count, L.pl_sc_sim_count, L.pl_clock_probe):
        f.restype = ctypes.c_int
    return L


def use_dev_library():
    """Development tools only (tools/): load libpolar_mi355x_dev.so (python -m polar_amd.build
    --dev), the build with the A/B hooks (PL_SC_DEFINES, PL_SC_SOURCE, PL_SC_LOG_G,
    PL_SCL_VIRTUAL, PL_SCL_TREE_FAST and the diagnostic macros), instead of the release library.
    Must be called before the first library call of the process."""
    global LIB_PATH
    dev = os.path.join(_HERE, "libpolar_mi355x_dev.so")
    if _lib is not None and LIB_PATH != dev:
        raise PolarLibError("use_dev_library(): the release library is already loaded in this process")
    LIB_PATH = dev


def lib():
    """Load (once) and return the ctypes handle.  Raises if the library has not been built."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise PolarLibError(
                        f"{LIB_PATH} is missing: build it with `python -m polar_amd.build` "
                        "(hipcc, gfx950).  There is no CPU fallback.")
                _lib = _declare(ctypes.CDLL(LIB_PATH))
    return _lib


EXPORTED_SYMBOLS = ("pl_plan_create", "pl_plan_destroy", "pl_plan_info", "pl_plan_device", "pl_sc_decode",
                    "pl_scl_workspace_size", "pl_scl_decode", "pl_polar_encode",
                    "pl_plan_kernel", "pl_sc_specialize", "pl_sc_source", "pl_plan_set_crc", "pl_crc_attach",
                    "pl_crc_check", "pl_gather_rows",
                    "pl_rate_recover", "pl_awgn_qpsk_llr", "pl_count_errors", "pl_awgn_qpsk_llr_bits",
                    "pl_sc_count_workspace_size", "pl_sc_decode_count", "pl_sc_sim_count", "pl_clock_probe",
                    "pl_last_error_string", "pl_version")


def check(rc, what):
    if rc != PL_OK:
        msg = lib().pl_last_error_string().decode(errors="replace")
        if rc == PL_EINVAL:
            raise ValueError(f"{what}: {msg}")
        raise PolarLibError(f"{what} failed ({rc}): {msg}", rc)


def current_stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


# ---- code-specialised SC kernels, compiled out of process --------------------------------------
# The library can compile a specialised kernel itself (hiprtc, pl_sc_specialize), but in a
# process that has imported torch, hiprtc runs against torch's bundled amd_comgr (an older ROCm
# than /opt/rocm's hiprtc): measured here, that combination emits ~15 % more instructions for
# the (512,1024) kernel and segfaults on at least one reference code.  So the Python layer
# compiles with hipcc --genco in a child process (build.py ahead of time; Plan() for codes not
# pre-built) and hands the library only cached code objects (PL_PLAN_CACHE_ONLY).
#
# The generated source starts with two lines written by the library (jit.cpp static_source):
#   // pl-genco-flags: <hipcc flags>
#   // pl-compiler: <__clang_version__ of the compiler that built libpolar_mi355x.so>
# Both are part of the content-addressed cache name.  The flags are taken from there, and the
# object is only built when `hipcc --version` reports that same compiler, so a cached object's
# name always says which compiler and flags produced it.
_GENCO_TAG, _COMPILER_TAG = "// pl-genco-flags: ", "// pl-compiler: "
_hipcc_version = {}


def _source_header(src):
    flags = compiler = None
    for line in src.splitlines()[:8]:
        if line.startswith(_GENCO_TAG):
            flags = line[len(_GENCO_TAG):].split()
        elif line.startswith(_COMPILER_TAG):
            compiler = line[len(_COMPILER_TAG):].strip()
    return flags, compiler


def hipcc_version(hipcc):
    """`hipcc --version` text (cached per path)."""
    import subprocess
    if hipcc not in _hipcc_version:
        r = subprocess.run([hipcc, "--version"], capture_output=True, text=True, timeout=120)
        _hipcc_version[hipcc] = r.stdout if r.returncode == 0 else ""
    return _hipcc_version[hipcc]


def sc_source(n, frozen_mask_u8, f_mode):
    """(HIP source, cache file name) of the specialised SC kernel of a code (pl_sc_source)."""
    import numpy as np
    mask = np.ascontiguousarray(frozen_mask_u8, dtype=np.uint8)
    size, name = ctypes.c_size_t(), ctypes.create_string_buffer(256)
    ptr = mask.ctypes.data_as(ctypes.c_void_p)
    check(lib().pl_sc_source(int(n), ptr, int(f_mode), None, 0, ctypes.byref(size), name, 256), "pl_sc_source")
    buf = ctypes.create_string_buffer(size.value)
    check(lib().pl_sc_source(int(n), ptr, int(f_mode), buf, size.value, ctypes.byref(size), name, 256),
          "pl_sc_source")
    return buf.value.decode(), name.value.decode()


def kernel_cache_dirs():
    """The library's lookup order (jit.cpp cache_dirs): $PL_KERNEL_CACHE, <lib dir>/kcache,
    ~/.cache/polar_mi355x."""
    dirs = []
    if os.environ.get("PL_KERNEL_CACHE"):
        dirs.append(os.environ["PL_KERNEL_CACHE"])
    dirs.append(os.path.join(_HERE, "kcache"))
    if os.environ.get("HOME"):
        dirs.append(os.path.join(os.environ["HOME"], ".cache", "polar_mi355x"))
    return dirs


def hipcc_path():
    import shutil
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    return None


def compile_code_object(src, out_dir, name, timeout=600):
    """hipcc --genco of one specialised kernel into out_dir/name (atomic rename).  True on success;
    False when hipcc is missing, is not the compiler named in the source, or fails."""
    import shutil
    import subprocess
    import tempfile
    hipcc = hipcc_path()
    if hipcc is None:
        return False
    flags, compiler = _source_header(src)
    if not flags or not compiler:
        raise ValueError("specialised SC source without its build header (pl-genco-flags / pl-compiler)")
    if compiler not in hipcc_version(hipcc):
        import warnings
        warnings.warn(f"{hipcc} is not the compiler libpolar_mi355x.so was built with ({compiler}); rebuild the "
                      "library (python -m polar_amd.build) to compile specialised SC kernels")
        return False
    os.makedirs(out_dir, exist_ok=True)
    with tempfile.TemporaryDirectory(prefix="pl_sc_") as td:
        hip = os.path.join(td, "pl_sc_static.hip")
        with open(hip, "w") as f:
            f.write(src)
        tmp = os.path.join(td, name)
        r = subprocess.run([hipcc, *flags, hip, "-o", tmp], capture_output=True, text=True, timeout=timeout)
        if r.returncode != 0 or not os.path.exists(tmp):
            return False
        part = os.path.join(out_dir, f".{name}.{os.getpid()}.part")
        shutil.copyfile(tmp, part)
        os.replace(part, os.path.join(out_dir, name))
    return True


def ensure_sc_kernel(n, frozen_mask_u8, f_mode):
    """Make sure the specialised SC kernel of a code is in a kernel cache; compile it with hipcc
    in a child process if not.  Returns False when it could not be provided (the plan then runs
    the generic HIP kernel)."""
    src, name = sc_source(n, frozen_mask_u8, f_mode)
    dirs = kernel_cache_dirs()
    if any(os.path.exists(os.path.join(d, name)) for d in dirs):
        return True
    targets = ([dirs[0]] if os.environ.get("PL_KERNEL_CACHE") else []) + \
        [d for d in dirs if d.endswith("polar_mi355x")] + [os.path.join(_HERE, "kcache")]
    for d in targets:
        try:
            if compile_code_object(src, d, name):
                return True
        except (OSError, ValueError):
            pass
    return False


def device_index(device=None):
    """CUDA device index of `device` (None: the current device; None without a visible GPU)."""
    if device is None:
        return torch.cuda.current_device() if torch.cuda.is_available() else None
    if isinstance(device, int):
        return device
    d = torch.device(device)
    if d.type != "cuda":
        raise ValueError(f"plans live on a ROCm GPU, not on {d}")
    return d.index if d.index is not None else torch.cuda.current_device()


class Plan:
    """Owning wrapper of a pl_plan* (immutable, usable from any stream of its device).

    A plan is device-bound: pl_plan_create allocates its tables and loads its specialised kernel
    on the current device, so the plan is created inside `torch.cuda.device(device)` and the
    library rejects launches on another device's stream (PL_EINVAL).  Use PlanSet for one plan
    per device."""

    def __init__(self, n, frozen_mask_u8, list_size=1, f_mode=PL_F_MINSUM, llr_max=30.0, flags=0, device=None):
        """flags: 0 (SC plans get a kernel specialised to the frozen set), PL_PLAN_GENERIC,
        PL_PLAN_CACHE_ONLY or PL_PLAN_FAST_SCL (see include/polar_mi355x.h).  device: the GPU the
        plan lives on (default: the current device)."""
        import contextlib

        import numpy as np
        mask = np.ascontiguousarray(frozen_mask_u8, dtype=np.uint8)
        assert mask.shape == (n,)
        if int(list_size) == 1 and os.environ.get("PL_SC_SPECIALIZE") != "0" and \
                not (flags & (PL_PLAN_GENERIC | PL_PLAN_CACHE_ONLY)):
            # the library only loads cached code objects; compile out of process when missing.
            # Exact-f plans with llr_max > 43 (compared in fp32, as pl_plan_create does) run the
            # full-range code object (jit.cpp attach_static)
            wide = int(f_mode) == PL_F_EXACT and float(np.float32(llr_max)) > 43.0
            ensure_sc_kernel(n, mask, int(f_mode) | (PL_F_WIDE_RANGE if wide else 0))
            flags |= PL_PLAN_CACHE_ONLY
        idx = device_index(device)
        self._h = ctypes.c_void_p()
        with (torch.cuda.device(idx) if idx is not None else contextlib.nullcontext()):
            check(lib().pl_plan_create(ctypes.byref(self._h), int(n), mask.ctypes.data_as(ctypes.c_void_p),
                                       int(list_size), int(f_mode), float(llr_max), int(flags)), "pl_plan_create")
        n_, k_, l_, d_ = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        check(lib().pl_plan_info(self._h, ctypes.byref(n_), ctypes.byref(k_), ctypes.byref(l_)), "pl_plan_info")
        check(lib().pl_plan_device(self._h, ctypes.byref(d_)), "pl_plan_device")
        self.n, self.k, self.list_size = n_.value, k_.value, l_.value
        self.device = torch.device("cuda", d_.value)

    @property
    def handle(self):
        return self._h

    def set_crc(self, degree, poly_mask):
        """CRC-aided path selection for SCL plans (pl_plan_set_crc)."""
        check(lib().pl_plan_set_crc(self._h, int(degree), int(poly_mask)), "pl_plan_set_crc")

    def kernel(self):
        """(kind, code-object path or '') of the kernel this plan runs: kind is 'specialized' or
        'generic' for SC plans, 'scl_subtree' or 'generic' for SCL plans."""
        kind, buf = ctypes.c_int32(), ctypes.create_string_buffer(4096)
        check(lib().pl_plan_kernel(self._h, ctypes.byref(kind), buf, 4096), "pl_plan_kernel")
        names = {PL_KERNEL_GENERIC: "generic", PL_KERNEL_SPECIALIZED: "specialized",
                 PL_KERNEL_SCL_SUBTREE: "scl_subtree"}
        return names[kind.value], buf.value.decode()

    def __deepcopy__(self, memo):  # a copy would double-free the handle
        raise TypeError("polar_amd Plan objects are not copyable; build another Plan")

    def __reduce__(self):
        raise TypeError("polar_amd Plan objects are not picklable")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib is not None:
            _lib.pl_plan_destroy(h)
            self._h = None


class PlanSet:
    """The plans of one code, one per GPU, made on first use by `make(device_index)`.

    Decoder modules keep one of these instead of a single plan, so a module works on whichever
    device its input is on (and replicas of a module on several GPUs share it).  Copying or
    pickling a module gives it an empty set (plans are rebuilt on first use)."""

    def __init__(self):
        self._plans = {}
        self._lock = threading.Lock()

    def get(self, device, make):
        idx = device_index(device)
        p = self._plans.get(idx)
        if p is None:
            with self._lock:
                p = self._plans.get(idx)
                if p is None:
                    p = self._plans[idx] = make(idx)
        return p

    def __len__(self):
        return len(self._plans)

    def __deepcopy__(self, memo):
        return PlanSet()

    def __getstate__(self):
        return {}

    def __setstate__(self, state):
        self.__init__()
