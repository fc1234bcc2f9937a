#!/bin/bash
# Jacobi tuning sweep on the GPU box: one short bench per environment setting; prints the Jacobi
# stage time and the pass plans.  Settings are ';'-separated lists of VAR=VALUE (space-separated).
#   SWEEP='PF_JT512=10 PF_JN512=6;PF_JPIPE=1' bash tools/jenv_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/jenv
IFS=';' read -ra CFGS <<< "${SWEEP:-}"
CFGS=("" "${CFGS[@]}")
i=0
for cfg in "${CFGS[@]}"; do
  i=$((i + 1))
  log=gpurun_out/jenv/run$i.log
  env $cfg PF_JPLAN=1 timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $log 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "[$cfg] rc=$rc"; tail -3 $log; exit $rc; }
  python3 - "$cfg" $log <<'PY'
import json, sys
lines = open(sys.argv[2]).read().splitlines()
d = json.loads(lines[-1])
plans = sorted(set(l.split(" C2:")[0].split("plan ")[1].split(" band")[0] + ":" + l.split(":", 1)[1].strip()[:60]
                   for l in lines if "jacobi plan" in l))
print("[%s] value=%.0f jacobi_ms=%.3f" % (sys.argv[1] or "default", d["value"], d["stages"]["jacobi"]["ms_per_step"]))
for p in plans:
    print("    ", p)
PY
done
