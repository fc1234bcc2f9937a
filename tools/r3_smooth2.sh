#!/bin/bash
# Round 3: smoothing unroll variants (tools/smooth_probe.py), each under PANOFUSE_LIB.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PKG=wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-registrations_amd
mkdir -p gpurun_out/smooth
for v in ${VARIANTS:-su1 su4 su8}; do
  PANOFUSE_LIB=$PWD/$PKG/lib/variants/libpanofuse_$v.so timeout -k 10 120 python tools/smooth_probe.py > gpurun_out/smooth/$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/smooth/$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/smooth/$v.log)"
done
