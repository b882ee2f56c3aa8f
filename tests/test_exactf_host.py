"""The host mirror of csrc/exactf.h (tools/micro/exactf_rounding.cpp: the same tables, the same
operation sequence in fp64 with fma) against correctly rounded expl / logl: exp, log, e^(x+y) by
the product e^x e^y e^d, and the whole exact f.  The full record (5e7 arguments each, all zero) is
in DESIGN.md; this is a 2e5-argument guard that the mirror still builds and still agrees."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "micro", "exactf_rounding.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_exactf_host_mirror_is_correctly_rounded(tmp_path):
    exe = str(tmp_path / "exr")
    subprocess.run(["g++", "-O2", "-o", exe, SRC], check=True, capture_output=True, timeout=300)
    out = subprocess.run([exe, "200000"], check=True, capture_output=True, text=True, timeout=300).stdout
    counts = [int(v) for v in re.findall(r"(?:exp|normal\)|0\.01\)|product|differing) (\d+)", out)]
    assert len(counts) == 5, out
    assert counts == [0, 0, 0, 0, 0], out
