#!/bin/bash
# Warp-only library variants (run here): recompile pf_warp.hip with extra flags, link against the
# other objects of the default build.  Usage: tools/warp_variants.sh NAME "FLAGS" [...]
set -e
cd "$(dirname "$0")/.."
PKG=$(ls -d wacv2023-*_amd)
mkdir -p $PKG/lib/variants
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  d=/tmp/pfwarp_$name; rm -rf $d; mkdir -p $d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
    -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero $flags \
    -c $PKG/csrc/pf_warp.hip -o $d/pf_warp.o
  objs=$(ls $PKG/build/*.o | grep -v pf_warp.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $PKG/lib/variants/libpanofuse_$name.so $objs $d/pf_warp.o
  echo "built $name: $flags"
done
