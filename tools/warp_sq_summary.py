"""Per-launch SQ counters of k_warp_depth from profiles/r03/warp/warp_sq_summary.txt; recipe: tools/gpu_round.sh pmc-style passes (new vs old library)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/warp_sq"
for tag in ("new", "old"):
    vals = collections.defaultdict(float)
    cnt = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, f"[ab]_{tag}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_warp_depth" not in r["Kernel_Name"]:
                continue
            vals[r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
    if not vals:
        continue
    print(tag, open(os.path.join(d, f"probe_{tag}.txt")).read().strip().splitlines()[-1][:80])
    for k in sorted(vals):
        print(f"  {k:24s} {vals[k] / len(cnt[k]):16.1f}")
