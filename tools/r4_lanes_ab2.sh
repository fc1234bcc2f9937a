#!/bin/bash
# A/B: one pipelined lane (--pipeline 1), two plain lanes (--pipeline 2), two pipelined lanes
# (--pipeline 2 with PF_LANE_WARP=1), alternating rounds on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/lanes2
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in p1:1:0 p2:2:0 p2w:2:1 p3w:3:1; do
    IFS=: read name p w <<< "$v"
    PF_LANE_WARP=$w timeout -k 10 300 python3 bench.py --pipeline $p --steps 20 --warmup 3 --no-cpu-baseline \
      --no-extra-configs --prof-steps 1 > $O/$name.$r.log 2>&1 || { echo "$name rc=$?"; tail -5 $O/$name.$r.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/$name.$r.log') if l.startswith('{')][-1]); print('$name round $r: %.0f panoramas/s  %.3f ms/step  bit_exact %s' % (d['value'], d['ms_per_step'], d['bit_exact_vs_one_process']))"
  done
done
