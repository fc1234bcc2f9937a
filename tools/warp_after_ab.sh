#!/bin/bash
# A/B: pipelined C3 step with the next batch's warp starting after the previous fusion only
# (PF_WARP_AFTER=-1), after level 0 of the current fusion (0) or after level 1 (1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/warp_after
mkdir -p $O
for r in 1 2 3; do
  for m in -1 0 1; do
    PF_WARP_AFTER=$m timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/b_${m}_$r.log 2>&1 || exit 1
    tail -1 $O/b_${m}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("after '$m' round '$r'", round(d["value"]), "pano/s", round(d["ms_per_step"], 3), "ms")'
  done
done
