#!/bin/bash
# A/B of the step schedule on one GPU: the pipelined step, the side
# stream for the finer target planes (PF_NOSIDE) and the serial step; alternating, twice each.
# Usage (GPU box): bash tools/sched_ab.sh > gpurun_out/sched_ab.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {
  local tag=$1; shift
  local line extra=""
  [ "$tag" = serial ] && extra="--pipeline 0"
  line=$(env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
         --prof-steps 1 $extra 2>/dev/null | tail -1) || { echo "$tag FAILED"; exit 1; }
  python -c "import json,sys; d=json.loads(sys.argv[2]); print(f\"{sys.argv[1]:28s} {d['ms_per_step']:.3f} ms/step {d['value']:.0f} panoramas/s\")" "$tag" "$line"
}
for rep in 1 2; do
  run pipelined PF_NOSIDE=
  run pipelined_noside PF_NOSIDE=1
  run serial PF_NOSIDE=
done
