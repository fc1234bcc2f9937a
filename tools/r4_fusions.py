"""Per-fusion Jacobi accounting from a rocprofv3 kernel trace: for every k_jres dispatch (one per
fusion), the kernels of that fusion's Jacobi stage (k_jres + the following k_jlag passes), their
summed durations and the wall span from the k_jres start to the last pass's end."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
fus = []
for r in rows:
    n = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if "k_jres" in n:
        fus.append({"start": s, "end": e, "busy": e - s, "n": 1, "jres": e - s})
    elif ("k_jlag" in n or "k_border" in n) and fus:
        f = fus[-1]
        if "k_jlag" in n:
            f["busy"] += e - s
            f["n"] += 1
        f["end"] = max(f["end"], e)
for i, f in enumerate(fus):
    print(f"fusion {i:3d}: jres {f['jres'] / 1e3:7.1f} us  jacobi kernels {f['n']:3d} busy "
          f"{f['busy'] / 1e3:8.1f} us  span {(f['end'] - f['start']) / 1e3:8.1f} us")
