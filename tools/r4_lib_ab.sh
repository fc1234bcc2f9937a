#!/bin/bash
# A/B of library variants (lib/variants/libpanofuse_<name>.so via PANOFUSE_LIB) on the bench:
# serial steps (the Jacobi stage time) and the default two-lane line, alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-registrations_amd
O=gpurun_out/libab
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in default ${LIBS:-}; do
    if [ "$v" = default ]; then L=$(pwd)/$P/lib/libpanofuse.so; else L=$(pwd)/$P/lib/variants/libpanofuse_$v.so; fi
    for pipe in 0 2; do
      PANOFUSE_LIB=$L timeout -k 10 300 python3 bench.py --pipeline $pipe --steps 20 --warmup 3 --no-cpu-baseline \
        --no-extra-configs --prof-steps 5 > $O/$v.p$pipe.$r.log 2>&1 || { echo "$v p$pipe rc=$?"; tail -5 $O/$v.p$pipe.$r.log; exit 1; }
      python3 -c "import json; d=json.loads([l for l in open('$O/$v.p$pipe.$r.log') if l.startswith('{')][-1]); print('%-8s pipeline $pipe round $r: %.0f panoramas/s  jacobi %.3f ms  bit_exact %s' % ('$v', d['value'], d['stages']['jacobi']['ms_per_step'], d['bit_exact_vs_one_process']))"
    done
  done
done
