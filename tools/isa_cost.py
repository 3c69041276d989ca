"""Issue-cost model of a gfx950 ISA loop body (design tool, not product).

Costs are the measured per-wave-instruction issue times of tools/microbench5..9 at 4 waves per SIMD
(profiles/r02_microbench_issue_costs.txt), in ns at the microbenchmarks' clock:
  fast  ~1.0 ns: v_fma/v_fmac/v_mul/v_add/v_sub f32 (VGPR/inline/literal operands, not three
                 distinct source VGPRs in one bank), v_and/v_or/v_xor/v_mov, v_add/sub_u32,
                 v_ashrrev, output modifiers (clamp, omod), source modifiers (abs, neg)
  slow  ~1.85 ns: any SGPR source operand, three source VGPRs in one bank (index mod 4), v_bfi,
                 v_cndmask, v_cmp, DPP, v_max/v_min/v_med3/v_max3 (f32 and int), v_lshlrev,
                 v_ldexp, v_cvt, v_or3, v_and_or, v_xad
  trans ~3.4 ns: v_log/v_exp/v_sqrt/v_rsq/v_rcp f32
Usage: python tools/isa_cost.py file.s LABEL   (LABEL: the loop header, e.g. .LBB9_50)
Prints the instruction classes, the three-same-bank FMAs and the modelled issue time per iteration.
"""
from __future__ import annotations

import re
import sys

FAST, SLOW, TRANS = 1.0, 1.85, 3.4
TRANS_OPS = ("v_log_f32", "v_exp_f32", "v_sqrt_f32", "v_rsq_f32", "v_rcp_f32")
SLOW_OPS = ("v_bfi", "v_cndmask", "v_cmp", "v_max", "v_min", "v_med3", "v_lshlrev", "v_ldexp", "v_cvt", "v_or3",
            "v_and_or", "v_xad", "v_mov_b32_dpp", "v_readfirstlane", "v_readlane", "v_writelane", "v_perm")


def vregs(ops):
    out = []
    for o in ops:
        o = o.strip().lstrip("-|").rstrip("|")
        m = re.match(r"v\[(\d+):(\d+)\]", o)
        if m:
            out.append(int(m.group(1)))
            continue
        m = re.match(r"v(\d+)$", o)
        if m:
            out.append(int(m.group(1)))
    return out


def classify(line):
    s = line.split(";")[0].strip()
    if not s or s.startswith(".") or s.endswith(":"):
        return None, s
    op = s.split()[0]
    if not op.startswith("v_"):
        return None, s
    if op.startswith(TRANS_OPS):
        return "trans", s
    if "_dpp" in op or " quad_perm" in s or "row_" in s:
        return "slow", s
    if op.startswith(SLOW_OPS):
        return "slow", s
    args = s[len(op):].split(",")
    if any(re.match(r"\s*s\[?\d", a) or a.strip() in ("vcc", "exec") for a in args[1:]):
        return "slow", s
    srcs = vregs(args[1:])
    if op.startswith("v_fmac"):
        srcs = srcs + vregs(args[:1])
    if len(set(srcs)) == 3 and len({r % 4 for r in srcs}) == 1:
        return "slow-bank", s
    return "fast", s


def main():
    path, label = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(label + ":"))
    body = []
    for l in lines[start + 1:]:
        body.append(l)
        if re.match(r"\s*s_cbranch_\w+\s+" + re.escape(label) + r"\b", l):
            break
    counts = {"fast": 0, "slow": 0, "slow-bank": 0, "trans": 0}
    banked = []
    for l in body:
        c, s = classify(l)
        if c:
            counts[c] += 1
            if c == "slow-bank":
                banked.append(s)
    t = counts["fast"] * FAST + (counts["slow"] + counts["slow-bank"]) * SLOW + counts["trans"] * TRANS
    print({k: v for k, v in counts.items()}, f"model {t:.1f} ns per iteration per SIMD (4 waves)")
    for s in banked[:8]:
        print("  bank conflict:", s)


if __name__ == "__main__":
    main()
