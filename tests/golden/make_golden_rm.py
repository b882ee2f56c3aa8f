"""Golden fixtures for the Reed-Muller frozen-set helper generate_rm_code (my_sn/fec/polar/utils.py:73-101).

TEST INFRASTRUCTURE ONLY; runs in the build container (imports the reference read-only from
/root/reference) and writes tests/golden/rm_codes.npz: for every 0 <= r <= m <= 10 the
reference's [frozen_pos, info_pos, n, k, d_min].

Run-time shim (nothing in the reference is modified): `importlib_resources` is not installed, so a
module object exposing the standard library's importlib.resources.files / as_file is placed in
sys.modules (utils.py:4 imports it), as in make_golden_5g.py.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_rm.py
"""
import importlib.resources
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path += [REF]

_shim = types.ModuleType("importlib_resources")
_shim.files = importlib.resources.files
_shim.as_file = importlib.resources.as_file
sys.modules["importlib_resources"] = _shim

from my_sn.fec.polar.utils import generate_rm_code  # noqa: E402


def main():
    out = {}
    for m in range(11):
        for r in range(m + 1):
            frozen, info, n, k, d_min = generate_rm_code(r, m)
            out[f"r{r}_m{m}_frozen"] = np.asarray(frozen, dtype=np.int32)
            out[f"r{r}_m{m}_info"] = np.asarray(info, dtype=np.int32)
            out[f"r{r}_m{m}_meta"] = np.array([n, k, d_min], dtype=np.int64)
    np.savez_compressed(os.path.join(OUT, "rm_codes.npz"), **out)
    print(f"wrote {len(out) // 3} RM codes")


if __name__ == "__main__":
    main()
