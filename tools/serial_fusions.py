"""Per-fusion Jacobi accounting from a rocprofv3 kernel trace: for every k_jres dispatch (one per
fusion), the kernels of that fusion's Jacobi stage (k_jres + the following k_jlag passes), their
summed durations and the wall span from the k_jres start to the last pass's end; then the
per-level split (kernel, grid) of the median fusion among the last LAST (default 5) fusions
before the final one (in bench.py: the profiled serial steps; the last fusion is the bench's
one-process bit-exactness check)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
LAST = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
fus = []
for r in rows:
    n = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    key = (n.split("(")[0].replace("void pf::", "").replace("pf::", "")[:34], r["Grid_Size_X"])
    if "k_jres" in n:
        fus.append({"start": s, "end": e, "busy": e - s, "n": 1, "parts": collections.OrderedDict([(key, e - s)])})
    elif "k_jlag" in n and fus:
        f = fus[-1]
        f["busy"] += e - s
        f["n"] += 1
        f["end"] = max(f["end"], e)
        f["parts"][key] = f["parts"].get(key, 0) + (e - s)
for i, f in enumerate(fus):
    print(f"fusion {i:3d}: jacobi kernels {f['n']:3d} busy {f['busy'] / 1e3:8.1f} us  "
          f"span {(f['end'] - f['start']) / 1e3:8.1f} us")
sel = fus[-1 - LAST:-1] if len(fus) > LAST else fus
med = sorted(sel, key=lambda f: f["busy"])[len(sel) // 2]
print(f"median of the {len(sel)} fusions before the last: busy {med['busy'] / 1e3:.1f} us")
for (k, g), t in med["parts"].items():
    print(f"  {k:36s} gridx={g:>7s} {t / 1e3:8.1f} us")
