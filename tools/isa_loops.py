"""Loops of one kernel in a hipcc -S listing and the opcode histogram of one of them (design tool).
python tools/isa_loops.py file.s KERNEL_SYMBOL [LABEL]"""
import collections
import re
import sys

L = open(sys.argv[1]).read().split("\n")
name = sys.argv[2]
start = [i for i, l in enumerate(L) if l.startswith(name + ":")][0]
end = start
while not L[end].startswith(".Lfunc_end"):
    end += 1
body = L[start:end]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        labels[m.group(1)] = i
if len(sys.argv) < 4:
    for i, l in enumerate(body):
        m = re.search(r"s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            print("loop", m.group(2), "lines", labels[m.group(2)], "-", i, "len", i - labels[m.group(2)])
    sys.exit(0)
a = labels[sys.argv[3]]
b = a + 1
while b < len(body) and not re.search(r"s_(cbranch_\w+|branch)\s+" + re.escape(sys.argv[3]) + r"\b", body[b]):
    b += 1
c = collections.Counter()
for l in body[a:b + 1]:
    s = l.split(";")[0].strip()
    if s and not s.startswith(".") and not s.endswith(":"):
        c[s.split()[0]] += 1
v = sum(n for k, n in c.items() if k.startswith("v_"))
print(f"{sys.argv[3]}: {b - a} lines, {v} VALU")
for k, n in c.most_common():
    print(f"{n:5d} {k}")
