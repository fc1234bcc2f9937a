"""Kernel-by-kernel timeline of one bench step from a rocprofv3 kernel trace: the segment between
the k_warp_depth dispatches number K and K+1 counted from the end (default K = 3: with the
bench's final one-process check last, that is the last profiled serial step)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
K = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
warps = [i for i, r in enumerate(rows) if "k_warp_depth" in r["Kernel_Name"]]
a, b = warps[-K - 1], warps[-K]
seg = rows[a:b]
t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
print(f"step span {(t1 - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us, {len(seg)} kernels")
prev = None
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"  gap {gap:8.1f}  dur {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:64]}")
    prev = e
