"""Development aid: in-process hiprtc (pl_sc_specialize) in a process that has
imported torch and initialised the GPU, over the reference codes up to n = NMAX, with Python's
faulthandler on, and the comgr / hiprtc libraries the process mapped.

  python -X faulthandler tools/hiprtc_inprocess.py LIB NMAX [gpu|nogpu]
"""
import ctypes
import os
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "polar-code-pytorch-sionna_amd"))
from polar_amd import build  # noqa: E402

lib, nmax = sys.argv[1], int(sys.argv[2])
if len(sys.argv) < 4 or sys.argv[3] == "gpu":
    torch.zeros(1, device="cuda").add_(1)
    torch.cuda.synchronize()
L = ctypes.CDLL(os.path.abspath(lib))
L.pl_sc_specialize.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_char_p, ctypes.c_char_p,
                               ctypes.c_size_t]
L.pl_last_error_string.restype = ctypes.c_char_p
codes = sorted((c for c in build.reference_codes() if len(c[0]) <= nmax), key=lambda c: len(c[0]))
d = tempfile.mkdtemp()
buf = ctypes.create_string_buffer(4096)
print(len(codes), "codes, lib", lib, flush=True)
for i, (m, fm) in enumerate(codes):
    t = time.time()
    mb = bytes(bytearray(m))
    rc = L.pl_sc_specialize(len(m), mb, fm, d.encode(), buf, 4096)
    err = "" if rc == 0 else L.pl_last_error_string().decode(errors="replace")[:300]
    print(i, "n", len(m), "k", int(len(m) - m.sum()), "f", fm, "rc", rc, f"{time.time() - t:.2f}s", err, flush=True)
maps = {ln.split()[-1] for ln in open("/proc/self/maps") if "comgr" in ln or "hiprtc" in ln}
print("mapped:", sorted(maps))
print("done")
