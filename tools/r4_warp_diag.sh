#!/bin/bash
# Warp-kernel diagnostic probes: tools/warp_probe.py against the default library and the
# PF_WARP_DIAG variants in lib/variants/ (bits: 1 no stores, 2 no loads, 4 no LDS box reads,
# 8 no barriers; wrong outputs, timing only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-registrations_amd
mkdir -p gpurun_out/wdiag
for v in default ${LIBS:-d1 d2 d3 d4 d7 d8 d11}; do
  if [ "$v" = default ]; then L=$(pwd)/$P/lib/libpanofuse.so; else L=$(pwd)/$P/lib/variants/libpanofuse_$v.so; fi
  PANOFUSE_LIB=$L timeout -k 10 120 python tools/warp_probe.py > gpurun_out/wdiag/$v.log 2>&1 || { echo "$v rc=$?"; tail -3 gpurun_out/wdiag/$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/wdiag/$v.log') if l.startswith('{')][-1]); print('$v', 'warp %.3f noresp %.3f fill %.3f' % (d['warp_ms'], d['warp_noresp_ms'], d['fill_tiles_ms']))"
done
