"""Aggregate rocprofv3 --pmc counter CSVs per (kernel, grid): sums and per-dispatch averages.
Usage: python tools/pmc_summary.py gpurun_out/pmc_*/run_counter_collection.csv"""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for path in sys.argv[1:]:
    for f in glob.glob(path):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "pf::" not in name:
                continue
            key = (name.split("(")[0], r.get("Grid_Size", r.get("Grid_Size_X", "")))
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[key].add(r["Dispatch_Id"])
for key, d in sorted(agg.items()):
    n = len(cnt[key])
    print(f"{key[0]} grid={key[1]} dispatches={n}")
    for c, v in sorted(d.items()):
        print(f"    {c:28s} {v / n:16.1f} per dispatch")
