#!/bin/bash
# Barrier-free resident kernel: parity, then timing (serial steps) and the bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_jres.py > gpurun_out/r3/jres_tests.log 2>&1 || { tail -40 gpurun_out/r3/jres_tests.log; exit 1; }
tail -2 gpurun_out/r3/jres_tests.log
VARIANTS="noside:PF_NOSIDE=1 noside_dbg1:PF_NOSIDE=1,PF_JRES_DBG=1" TAG=_lf bash tools/jres_probe.sh || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3/b_lf_$r.log 2>&1 || exit 1
  tail -1 gpurun_out/r3/b_lf_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", round(d["value"]), "pano/s", round(d["ms_per_step"], 3), "ms", round(d["stages"]["jacobi"]["ms_per_step"],3))'
done
