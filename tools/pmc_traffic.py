"""HBM traffic per launch from the rocprofv3 --pmc passes of tools/pmc_round.sh.

Usage: python tools/pmc_traffic.py gpurun_out [out.json]

Groups dispatches by kernel family (k_jlag = every Jacobi pass of every level, the unit bench.py's
roofline aggregates over; k_warp_depth; k_targets_map; ...) and prints, per launch:
  fetch_size_B  FETCH_SIZE (KB -> B) as rocprofv3 reports it
  rdreq_B       32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B + 64*(other RDREQ)  (request sizes)
  write_B       WRITE_SIZE (KB -> B)
  traffic_B     hbm read + write per launch, read = max(2*fetch_size_B, rdreq_B): on gfx950
                FETCH_SIZE tallies 128-B requests at 64 B (MI355X_MICROARCH.md, HBM), so the raw
                counter is doubled; the request-size sum is the cross-check.
Writes the JSON next to the text (default <dir>/pmc_traffic.json).
"""
import collections
import csv
import glob
import json
import os
import sys


def family(name):
    name = name.replace("(anonymous namespace)::", "")
    short = name.split("(")[0].replace("void ", "").strip()
    return short.split("<")[0]


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(d, "pmc_traffic.json")
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in glob.glob(os.path.join(d, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "pf::" not in r["Kernel_Name"]:
                continue
            fam = family(r["Kernel_Name"])
            c = r["Counter_Name"]
            vals[fam][c] += float(r["Counter_Value"])
            disp[fam][c].add((f, r["Dispatch_Id"]))
    res = {}
    for fam, cs in sorted(vals.items()):
        per = {c: v / max(1, len(disp[fam][c])) for c, v in cs.items()}
        n = max(len(s) for s in disp[fam].values())
        fetch = per.get("FETCH_SIZE", 0.0) * 1024
        write = per.get("WRITE_SIZE", 0.0) * 1024
        rd = per.get("TCC_EA0_RDREQ_sum", 0.0)
        r32 = per.get("TCC_EA0_RDREQ_32B_sum", 0.0)
        r64 = per.get("TCC_EA0_RDREQ_64B_sum", 0.0)
        r128 = per.get("TCC_EA0_RDREQ_128B_sum", 0.0)
        other = max(0.0, rd - r32 - r64 - r128)
        rdreq = 32 * r32 + 64 * r64 + 128 * r128 + 64 * other
        read = max(2 * fetch, rdreq)
        res[fam] = {"dispatches": n, "fetch_size_B": fetch, "rdreq_B": rdreq, "write_B": write,
                    "read_B": read, "traffic_B": read + write, "counters_per_launch": per}
        print(f"{fam:22s} n={n:4d}  FETCH_SIZE {fetch/1e6:10.2f} MB  rdreq {rdreq/1e6:10.2f} MB"
              f"  WRITE {write/1e6:10.2f} MB  -> traffic {(read + write)/1e6:10.2f} MB/launch")
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
