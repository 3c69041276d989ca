"""Generate the table of tools/enf_exptab_variant.h (a measured, rejected variant): the 2^B entries {2^(j/2^B) hi, lo} (B = 5) of
exp64_tab / expm1_64_tab (round 6, VERDICT r05 item 7: a table-driven fp64 exp for the Center forms),
with mpmath at 60 digits: hi = the double nearest 2^(j/32), lo = the double nearest the remainder.

    python tools/gen_exptab.py            (print the table)
    python tools/gen_exptab.py --check    (the reduced range and the truncation of the series to r^7/5040)
"""
import os
import sys

import mpmath

mpmath.mp.dps = 60
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = 5


def table():
    rows = []
    for j in range(1 << B):
        v = mpmath.power(2, mpmath.mpf(j) / (1 << B))
        hi = float(v)
        lo = float(v - mpmath.mpf(hi))
        rows.append((hi, lo))
    return rows


def check():
    # r = w - k ln2/32 with k = rint(w 32/ln2): |r| <= ln2/64 (+ the rounding of w 32/ln2 and of the hi/lo split)
    rmax = mpmath.log(2) / 64 * (1 + mpmath.mpf(2) ** -40)
    # expm1(r) = r + r^2 (1/2 + r/6 + r^2/24 + r^3/120 + r^4/720 + r^5/5040): the next term r^8/40320, relative to
    # expm1(r) itself (the expm1 path at j = 0, n = 0) r^7/40320
    print("|r| max", float(rmax), "relative truncation r^7/40320", float(rmax ** 7 / 40320), "(2^-53 =", 2.0 ** -53, ")")


if "--check" in sys.argv:
    check()
    sys.exit(0)

out = [f"constexpr int kExpTabBits = {B};",
       f"constexpr int kExpTabN = {1 << B};",
       f"__constant__ const double kExpTab[2 * {1 << B}] = {{"]
for hi, lo in table():
    out.append(f"    {hi!r}, {lo!r},")
out += ["};"]
print("\n".join(out))
