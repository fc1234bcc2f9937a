#!/bin/bash
# Build library variants with extra compile flags into lib/variants/ (run here, on the CPU).
# Usage: tools/variants.sh NAME "FLAGS" [NAME "FLAGS" ...]
set -e
cd "$(dirname "$0")/.."
PKG=$(ls -d wacv2023-*_amd)
mkdir -p $PKG/lib/variants
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  rm -rf /tmp/pfvar_$name && mkdir -p /tmp/pfvar_$name
  for f in $PKG/csrc/*.hip; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
      -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero $flags \
      -c $f -o /tmp/pfvar_$name/$(basename $f .hip).o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $PKG/lib/variants/libpanofuse_$name.so /tmp/pfvar_$name/*.o
  echo "built $name: $flags"
done
