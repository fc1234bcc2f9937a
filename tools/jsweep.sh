#!/bin/bash
# Jacobi engine tuning sweep on the GPU box: one bench process per setting "Tmax:step_overhead:lone_cycles".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${SWEEP:-10:3}; do
  IFS=: read -r T O C1 <<< "$cfg"
  PF_JT=$T PF_JOVH=${O:-3} PF_JC1=${C1:-6} timeout -k 10 300 python bench.py --steps 5 --warmup 2 \
    --no-cpu-baseline > gpurun_out/sweep_$cfg.log 2>&1; rc=$?
  python - "$cfg" gpurun_out/sweep_$cfg.log <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    j = d["stages"]["jacobi"]
    print(sys.argv[1], "value=%.1f" % d["value"], "jacobi_ms=%.3f" % j["ms_per_step"],
          "GBps=%.0f" % j["GBps"], "targets_ms=%.3f" % d["stages"]["targets"]["ms_per_step"],
          "warp_ms=%.3f" % d["stages"]["warp"]["ms_per_step"],
          "warp_GBps=%.0f" % d["stages"]["warp"]["GBps"])
except Exception as e:
    print(sys.argv[1], "FAILED", e)
PY
  [ $rc -eq 0 ] || exit $rc
done
