#!/bin/bash
# A/B of the bench step schedule: --pipeline 1 (warp of batch k+1 beside the fusion of batch k)
# against N fusion lanes (--pipeline N), alternating rounds on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/lanes
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for p in ${PIPES:-1 2 3 4}; do
    timeout -k 10 300 python3 bench.py --pipeline $p --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
      --no-extra-configs --prof-steps 1 > $O/p$p.$r.log 2>&1 || { echo "p$p rc=$?"; tail -5 $O/p$p.$r.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/p$p.$r.log') if l.startswith('{')][-1]); print('pipeline $p round $r: %.0f panoramas/s  %.3f ms/step  bit_exact %s' % (d['value'], d['ms_per_step'], d['bit_exact_vs_one_process']))"
  done
done
