"""Per-kernel VGPR / spill counts from a hipcc -S listing (design tool): python tools/kernel_regs.py file.s [filter]"""
import re
import sys

txt = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.split(r"\n\s+- \.", txt.split("amdhsa.kernels:")[-1]):
    m = re.search(r"\.name:\s+(\S+)", blk)
    if not m or flt not in m.group(1):
        continue
    g = lambda k: (re.search(k + r":\s+(\d+)", blk) or [None, "?"])[1]
    print(f"{g('.vgpr_count'):>4} vgpr {g('.vgpr_spill_count'):>3} spill {g('.sgpr_count'):>3} sgpr  {m.group(1)}")
