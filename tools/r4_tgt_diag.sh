#!/bin/bash
# Targets-kernel probes (PF_TGT_DIAG variants in lib/variants/; wrong outputs, timing only): the
# serial bench's targets stage for the default library and each variant, alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-registrations_amd
O=gpurun_out/tdiag
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in default ${LIBS:-t1 t2 t3}; do
    if [ "$v" = default ]; then L=$(pwd)/$P/lib/libpanofuse.so; else L=$(pwd)/$P/lib/variants/libpanofuse_$v.so; fi
    PANOFUSE_LIB=$L timeout -k 10 300 python3 bench.py --pipeline 0 --steps 3 --warmup 1 --no-cpu-baseline \
      --no-extra-configs --prof-steps 5 > $O/$v.$r.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/$v.$r.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/$v.$r.log') if l.startswith('{')][-1]); print('%-8s round $r: targets %.3f ms' % ('$v', d['stages']['targets']['ms_per_step']))"
  done
done
