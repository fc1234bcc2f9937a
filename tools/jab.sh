#!/bin/bash
# A/B runs of the Jacobi engine on the GPU box: each line of $JAB (";"-separated) is
# "LIBNAME [ENV=VAL ...]" (LIBNAME = default or a lib/variants/libpanofuse_<name>.so); one short
# bench per line, printing the step, Jacobi and per-level pass plan.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PKG=$(ls -d wacv2023-*_amd)
mkdir -p gpurun_out
IFS=';' read -ra RUNS <<< "$JAB"
i=0
for run in "${RUNS[@]}"; do
  read -ra w <<< "$run"
  lib=${w[0]}; envs=("${w[@]:1}")
  so=$PKG/lib/libpanofuse.so; [ "$lib" != default ] && so=$PKG/lib/variants/libpanofuse_$lib.so
  i=$((i+1)); log=gpurun_out/jab_$i.log
  timeout -k 5 120 env PANOFUSE_LIB=$so PF_JPLAN=1 "${envs[@]}" python3 bench.py --steps 5 --warmup 2 \
    --no-cpu-baseline > $log 2>&1 || { echo "$run failed rc=$?"; tail -5 $log; exit 1; }
  python3 - "$run" $log <<'PY'
import json, sys
lines = open(sys.argv[2]).read().strip().split("\n")
d = json.loads(lines[-1])
st = d["stages"]
plans = sorted(set(l.split(":")[0].split(" band")[0].replace("jacobi plan ", "") + ":" +
                   " ".join(sorted(set(l.split(":", 1)[1].split()))) for l in lines if l.startswith("jacobi plan")))
print(f"{sys.argv[1]:40s} {d['ms_per_step']:.3f} ms/step jacobi {st['jacobi']['ms_per_step']:.3f}  | " + " | ".join(plans))
PY
done
