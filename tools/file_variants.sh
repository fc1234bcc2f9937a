#!/bin/bash
# One-file library variants (run here, on the CPU): recompile csrc/FILE.hip with extra flags and
# link it with the other objects of the default build into lib/variants/libpanofuse_NAME.so.
# Usage: tools/file_variants.sh FILE NAME "FLAGS" [NAME "FLAGS" ...]   (builds run in parallel)
set -e
cd "$(dirname "$0")/.."
PKG=$(ls -d wacv2023-*_amd)
f=$1; shift
mkdir -p $PKG/lib/variants
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  (
    d=/tmp/pfvar_${f}_$name; rm -rf $d; mkdir -p $d
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
      -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero $flags \
      -c $PKG/csrc/$f.hip -o $d/$f.o
    objs=$(ls $PKG/build/*.o | grep -v "/$f.o")
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $PKG/lib/variants/libpanofuse_$name.so $objs $d/$f.o
    echo "built $name: $flags"
  ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
