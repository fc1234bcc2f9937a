"""Concurrency of the bench loop from a rocprofv3 kernel trace: over the dispatches between the
first and last warp of the timed loop, the wall window, the time covered by at least one kernel
(busy), the summed kernel durations (work) and their ratio (mean kernels in flight), plus the
summed duration per kernel family.
Usage: python tools/lanes_overlap.py run_kernel_trace.csv"""
import collections
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "pf::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
warps = [i for i, r in enumerate(rows) if "k_warp_depth" in r["Kernel_Name"]]
# the warm-up + timed loop is the longest run of warps spaced under 10 ms apart
best, start = (0, 0), 0
for j in range(1, len(warps) + 1):
    if j == len(warps) or int(rows[warps[j]]["Start_Timestamp"]) - \
            int(rows[warps[j - 1]]["Start_Timestamp"]) > 10_000_000:
        if j - start > best[1] - best[0]:
            best = (start, j)
        start = j
w0, w1 = warps[best[0]], warps[best[1] - 1]
win = rows[w0:w1]
t0 = int(win[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in win)
busy = work = 0
end = t0
fam = collections.Counter()
for r in win:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    work += e - s
    fam[r["Kernel_Name"].split("(")[0].replace("void pf::", "").split("<")[0]] += e - s
    if e > end:
        busy += e - max(s, end)
        end = e
n = max(best[1] - best[0] - 1, 1)
print(f"window: {n} warp-to-warp intervals, {(t1 - t0) / 1e6:.3f} ms wall, "
      f"{(t1 - t0) / 1e3 / n:.1f} us per step")
print(f"busy (>= 1 kernel) {busy / (t1 - t0) * 100:.1f} %, kernels in flight on average "
      f"{work / busy:.2f}, summed kernel time per step {work / 1e3 / n:.1f} us")
for k, v in fam.most_common(10):
    print(f"  {k:22s} {v / 1e3 / n:8.1f} us per step")
