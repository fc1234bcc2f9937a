#!/bin/bash
# vectorised k_border4: parity (fusion tests) then a serial trace of the step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_rowshard.py -k "fuse or merge or internals or c3 or row" \
  > gpurun_out/r3/border_parity.log 2>&1 || { tail -40 gpurun_out/r3/border_parity.log; exit 1; }
tail -2 gpurun_out/r3/border_parity.log
TAG=_b bash tools/r3_serial.sh || exit 1
python3 - $(find gpurun_out/serial_b/prof -name "run_kernel_trace.csv" | head -1) <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
w = [i for i, r in enumerate(rows) if "k_warp_depth" in r["Kernel_Name"]]
step = rows[w[-2]:w[-1]]
acc = collections.OrderedDict()
for r in step:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:36]
    acc[n] = acc.get(n, 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
for k, v in acc.items():
    if v > 3: print(f"{k:38s} {v:8.1f} us")
PY
