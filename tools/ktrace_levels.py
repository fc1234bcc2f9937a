"""Per-level Jacobi time from a rocprofv3 kernel trace (tools/ktrace_levels.py run_kernel_trace.csv):
groups k_jres / k_jlag / k_jpipe dispatches of the last bench step by kernel and grid width and
sums their durations."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
warps = [i for i, r in enumerate(rows) if "k_warp_depth" in r["Kernel_Name"]]
step = rows[warps[-2]:warps[-1]] if len(warps) > 1 else rows
acc = collections.OrderedDict()
for r in step:
    n = r["Kernel_Name"]
    if "k_jlag" not in n and "k_jpipe" not in n and "k_jres" not in n:
        continue
    key = (n.split("(")[0].replace("void pf::", "")[:34], r["Grid_Size_X"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    c, t = acc.get(key, (0, 0.0))
    acc[key] = (c + 1, t + d)
tot = 0.0
for (k, g), (c, t) in acc.items():
    tot += t
    print(f"{k:36s} gridx={g:>7s} n={c:3d} total={t:8.1f} us  avg={t / c:7.1f} us")
print(f"jacobi total {tot:.1f} us")
# the step's other kernels (warp, registration, targets, border/seed), median over the serial steps
steps = [rows[warps[i]:warps[i + 1]] for i in range(len(warps) - 1)] if len(warps) > 1 else [rows]
per = collections.defaultdict(list)
for st in steps[-5:]:
    acc2 = collections.defaultdict(float)
    for r in st:
        n = r["Kernel_Name"]
        if not n.split("(")[0].replace("void ", "").startswith("pf::") or "k_jlag" in n or \
                "k_jres" in n or "k_jpipe" in n:
            continue
        acc2[n.split("(")[0].replace("void pf::", "").replace("pf::", "")[:30]] += \
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    for k, v in acc2.items():
        per[k].append(v)
for k, v in per.items():
    if len(v) < 3:  # kernels of the bench's tail (smoothing, checks), not of the steps
        continue
    v = sorted(v)
    print(f"{k:36s} median of {len(v)} steps {v[len(v) // 2]:8.1f} us")
