#!/bin/bash
# Registration stage A/B (serial bench, median of 5 profiled steps): default library against
# lib/variants/libpanofuse_<name>.so for each name in $LIBS, alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-registrations_amd
O=gpurun_out/regab
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in default ${LIBS:-head}; do
    if [ "$v" = default ]; then L=$(pwd)/$P/lib/libpanofuse.so; else L=$(pwd)/$P/lib/variants/libpanofuse_$v.so; fi
    PANOFUSE_LIB=$L timeout -k 10 300 python3 bench.py --pipeline 0 --steps 3 --warmup 1 --no-cpu-baseline \
      --prof-steps 5 > $O/$v.$r.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/$v.$r.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/$v.$r.log') if l.startswith('{')][-1]); print('%-8s round $r: register %.3f ms  c2 %.3f ms  c5 %.0f/s  bit_exact %s' % ('$v', d['stages']['register']['ms_per_step'], d['c2_batch1_ms'], d['c5_one_gpu']['value'], d['bit_exact_vs_one_process']))"
  done
done
