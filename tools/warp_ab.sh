#!/bin/bash
# Rebuild with each FLAGS variant (";"-separated list in VARIANTS) and run tools/warp_probe.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PKG=wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-registrations_amd
IFS=';' read -ra VS <<< "${VARIANTS:- }"
for v in "${VS[@]}"; do
  touch $PKG/csrc/*.hip
  make -s -C $PKG HIPFLAGS_EXTRA="$v" > gpurun_out/warp_ab_build.log 2>&1 || { echo "build failed: $v"; exit 1; }
  timeout -k 10 300 python tools/warp_probe.py > gpurun_out/warp_ab.log 2>&1 || { echo "probe failed: $v"; tail -5 gpurun_out/warp_ab.log; exit 1; }
  echo "[$v] $(tail -1 gpurun_out/warp_ab.log)"
done
