#!/bin/bash
# tools/build_variant.sh NAME "EXTRA HIPCC FLAGS": an A/B variant of libpanofuse.so built with extra
# compile-time flags (e.g. -DPF_JLAG_PF=3) into variants/NAME/lib/libpanofuse.so.  A run picks it
# with PANOFUSE_LIB=variants/NAME/lib/libpanofuse.so (tools/gpu_round.sh: VARIANTS="NAME:PANOFUSE_LIB=...").
set -e
cd "$(dirname "$0")/.."
PKG=$(ls -d *_amd)
make -s -C "$PKG" -j"${JOBS:-8}" BDIR="../variants/$1/build" LDIR="../variants/$1/lib" \
  HIPFLAGS_EXTRA="$2" "../variants/$1/lib/libpanofuse.so"
echo "variants/$1/lib/libpanofuse.so"
