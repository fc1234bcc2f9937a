#!/bin/bash
# Round 3: warp patch-size / block-size variants (tools/warp_variants.sh), probe each twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/wv2
PKG=wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-registrations_amd
for r in 1 2; do
for v in ${VARIANTS:-base p64w256 p64w512 p64w1024 p64w512c8k p32w512}; do
  if [ $v = base ]; then unset PANOFUSE_LIB; else export PANOFUSE_LIB=$PWD/$PKG/lib/variants/libpanofuse_$v.so; fi
  timeout -k 10 120 python tools/warp_probe.py > gpurun_out/wv2/$v.$r.log 2>&1 || { echo "probe $v failed"; tail -3 gpurun_out/wv2/$v.$r.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/wv2/$v.$r.log | cut -c1-160)"
done
done
