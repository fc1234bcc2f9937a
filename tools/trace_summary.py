"""Summarise a rocprofv3 kernel-trace CSV: per (kernel, grid) average duration and count.
Usage: python tools/trace_summary.py gpurun_out/prof/run_kernel_trace.csv [filter]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else "pf::"
agg = collections.OrderedDict()
for r in rows:
    name = r["Kernel_Name"]
    if flt not in name:
        continue
    short = name.split("(")[0]
    grid = (r.get("Grid_Size_X") or r.get("Grid_Size"), r.get("Grid_Size_Y", ""))
    dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    key = (short, grid, r.get("VGPR_Count", r.get("Arch_VGPR_Count", "")))
    n, t = agg.get(key, (0, 0))
    agg[key] = (n + 1, t + dur)
tot = sum(t for n, t in agg.values())
for (k, g, v), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{t/1e6:9.3f} ms {100*t/tot:5.1f}%  n={n:5d} avg={t/n/1e3:9.2f} us  vgpr={v:>4} grid={g}  {k}")
