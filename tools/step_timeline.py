"""Timeline of one bench step from a rocprofv3 kernel trace: every dispatch in start order with its
offset from the step start, duration, queue and the idle time before it, plus the step's busy and
idle totals (time covered by at least one kernel vs none).
Usage: python tools/step_timeline.py gpurun_out/prof/run_kernel_trace.csv [step_index_from_end=2]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if "pf::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
warps = [i for i, r in enumerate(rows) if "k_warp_depth" in r["Kernel_Name"]]
lo, hi = warps[-back - 1], warps[-back]
step = rows[lo:hi]
t0 = int(step[0]["Start_Timestamp"])
end = t0
busy = idle = 0
for r in step:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = max(0, s - end)
    idle += gap
    if e > end:
        busy += e - max(s, end)
        end = e
    q = r.get("Queue_Id") or r.get("Stream_Id") or ""
    name = r["Kernel_Name"].split("(")[0].replace("void pf::", "")[:40]
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap / 1e3:6.1f}  q{q:>3s} "
          f"grid {r['Grid_Size_X']:>8s}  {name}")
print(f"step span {(end - t0) / 1e3:.1f} us  busy {busy / 1e3:.1f} us  idle {idle / 1e3:.1f} us  "
      f"({len(step)} dispatches)")
