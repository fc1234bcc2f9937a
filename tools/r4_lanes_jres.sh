#!/bin/bash
# Lanes x resident level-0 kernel: plain lanes (PF_LANE_WARP=0) at 2 and 4 lanes, with the resident
# level-0 kernel (default) and without it (PF_JRES=0: streaming passes for level 0 too).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/lanesj
mkdir -p $O
export TMPDIR=/tmp
for v in p2:2:1 p4:4:1 p2s:2:0 p4s:4:0 p4w:4:1w; do
  IFS=: read name p j <<< "$v"
  lw=0; [ "$j" = "1w" ] && { lw=1; j=1; }
  PF_LANE_WARP=$lw PF_JRES=$j timeout -k 10 300 python3 bench.py --pipeline $p --steps 20 --warmup 3 \
    --no-cpu-baseline --no-extra-configs --prof-steps 1 > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $O/$name.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/$name.log') if l.startswith('{')][-1]); print('$name (lanes $p, jres $j, lane warp $lw): %.0f panoramas/s  %.3f ms/step  bit_exact %s' % (d['value'], d['ms_per_step'], d['bit_exact_vs_one_process']))"
done
