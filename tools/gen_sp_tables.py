"""Generate the log table of the SCL penalty's table-driven log (csrc/softplus.h, PL_SP_FORM 3,
between the GENERATED markers):  python tools/gen_sp_tables.py

y = 2^e m, m in [1, 2) (y >= 1 always: y = 1 + e^z); cell j = the top 7 bits of m's fraction;
c_j = 1/(cell midpoint) rounded to fp32 (c_0 = 1, so ln y near 1 keeps full relative accuracy);
ln y = e ln2 + (-ln c_j) + log1p(m c_j - 1), |m c_j - 1| <= 2^-8 (2^-7 in cell 0);
-ln c_j as hi (fp64) + lo (fp32).  mpmath at 120 bits.
"""
import os
import re
import struct

import mpmath

mpmath.mp.prec = 120
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "polar-code-pytorch-sionna_amd", "polar_amd", "csrc", "softplus.h")
BEGIN, END = "// ---- BEGIN GENERATED SP TABLE (tools/gen_sp_tables.py) ----", "// ---- END GENERATED SP TABLE ----"


def f32(x):
    return struct.unpack("<f", struct.pack("<f", float(x)))[0]


def render():
    out = [BEGIN, "// {c_j (fp32), lo(-ln c_j) (fp32), hi(-ln c_j) (fp64)} per cell j of m in [1, 2)",
           "__device__ const SpCell kSpLogTab[128] = {"]
    for j in range(128):
        if j == 0:
            c, hi, lo = 1.0, 0.0, 0.0
        else:
            mid = 1 + (mpmath.mpf(j) + mpmath.mpf("0.5")) / 128
            c = f32(1 / mid)
            L = -mpmath.log(mpmath.mpf(c))
            hi = float(L)
            lo = f32(L - mpmath.mpf(hi))
        out.append(f"    {{{float.hex(c)}f, {float.hex(lo)}f, {float.hex(hi)}}},".replace("0x0.0p+0f", "0.0f").replace("{0x0.0p+0", "{0.0"))
    out += ["};", END]
    return "\n".join(out)


def main():
    src = open(HDR).read()
    if BEGIN not in src:
        raise SystemExit(f"{HDR}: no GENERATED SP TABLE markers")
    src = re.sub(re.escape(BEGIN) + r".*?" + re.escape(END), lambda _: render(), src, flags=re.S)
    open(HDR, "w").write(src)
    print("table written:", HDR)


if __name__ == "__main__":
    main()
