#!/bin/bash
# Sweep depth 8 at 4 waves per SIMD (L ring in LDS, 118 VGPRs: lib variant lreg5) against the
# default T = 10 with the L ring in registers (166 VGPRs, 3 waves per SIMD); PF_JT caps T.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-registrations_amd
O=gpurun_out/t8
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in "base::" "t8reg:PF_JT=8:" "t8lds:PF_JT=8:lreg5" "t10lds::lreg5"; do
    IFS=: read name env lib <<< "$v"
    L=$(pwd)/$P/lib/libpanofuse.so; [ -n "$lib" ] && L=$(pwd)/$P/lib/variants/libpanofuse_$lib.so
    for pipe in 0 2; do
      ( [ -n "$env" ] && export $env; PANOFUSE_LIB=$L timeout -k 10 300 python3 bench.py --pipeline $pipe --steps 20 --warmup 3 \
        --no-cpu-baseline --no-extra-configs --prof-steps 5 > $O/$name.p$pipe.$r.log 2>&1 ) || { echo "$name rc=$?"; tail -5 $O/$name.p$pipe.$r.log; exit 1; }
      python3 -c "import json; d=json.loads([l for l in open('$O/$name.p$pipe.$r.log') if l.startswith('{')][-1]); print('%-7s pipeline $pipe round $r: %.0f panoramas/s  jacobi %.3f ms  bit_exact %s' % ('$name', d['value'], d['stages']['jacobi']['ms_per_step'], d['bit_exact_vs_one_process']))"
    done
  done
done
