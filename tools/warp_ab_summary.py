"""Summarise tools/warp_cut_ab.sh: per cut, k_warp_depth's mean kernel time and PMC bytes."""
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/warp_ab"
for cut in sorted({os.path.basename(p)[6:-4] for p in glob.glob(os.path.join(d, "probe_*.txt"))}):
    print(cut, open(os.path.join(d, f"probe_{cut}.txt")).read().strip().splitlines()[-2:])
    for f in glob.glob(os.path.join(d, f"kt_{cut}", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "warp_depth" in r["Name"]:
                print("  kernel", r["Name"][:40], "calls", r["Calls"], "avg_ms",
                      float(r["AverageNs"]) / 1e6)
    for kind in ("f", "w"):
        tot, n = 0.0, 0
        for f in glob.glob(os.path.join(d, f"pmc_{cut}", kind, "**", "*counter_collection.csv"),
                           recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_warp_depth" in r["Kernel_Name"]:
                    tot += float(r["Counter_Value"])
                    n += 1
        if n:
            print("  ", "FETCH_SIZE" if kind == "f" else "WRITE_SIZE", "per launch MB",
                  tot / n * 1024 / 1e6, "(raw, FETCH not doubled)")
