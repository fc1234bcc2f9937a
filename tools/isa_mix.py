"""Instruction mix of the main loop of one kernel in a .s file (largest basic-block loop).
Usage: python tools/isa_mix.py file.s mangled_kernel_name_prefix [steps_per_iter]"""
import collections
import re
import sys

s = open(sys.argv[1]).read().split("\n")
name = sys.argv[2]
steps = float(sys.argv[3]) if len(sys.argv) > 3 else 6.0
start = [i for i, l in enumerate(s) if l.startswith(name + ":")][0]
end = [i for i in range(start, len(s)) if s[i].strip().startswith(".Lfunc_end")][0]
body = s[start:end]
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\S+:", l)}
loops = []
for i, l in enumerate(body):  # backward branch = loop
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", l)
    if m:
        tgt = m.group(1) or m.group(2)
        if tgt in labels and labels[tgt] < i:
            loops.append((labels[tgt], i))
loops.sort(key=lambda b: b[0] - b[1])
which = int(sys.argv[4]) if len(sys.argv) > 4 else 0
print("loops (start, end):", loops[:4])
best = loops[which]
loop = body[best[0]:best[1] + 1]
c = collections.Counter()
for l in loop:
    t = l.strip().split()
    if t and not t[0].startswith((";", ".")):
        c[t[0]] += 1
valu = sum(v for k, v in c.items() if k.startswith("v_"))
pk = sum(v for k, v in c.items() if k.startswith("v_pk"))
print(f"loop lines {best}: instrs {sum(c.values())}  VALU {valu} (packed {pk})  per step {valu/steps:.1f}")
for k, v in c.most_common(30):
    print(f"  {k:28s} {v}")
for l in body:
    if "vgpr_count" in l or "sgpr_count" in l or "NumVgprs" in l:
        print(l.strip())
