#!/bin/bash
# tools/build_variant.sh NAME "EXTRA HIPCC FLAGS" [OBJ ...]: an A/B variant of libpanofuse.so built
# with extra compile-time flags (e.g. -DPF_JLAG_PF=3) into variants/NAME/lib/libpanofuse.so.  With
# OBJ names (e.g. pf_warp) only those objects are compiled with the flags; the others are the
# default build's.  A run picks the variant with PANOFUSE_LIB=variants/NAME/lib/libpanofuse.so
# (tools/gpu_round.sh: VARIANTS="NAME:PANOFUSE_LIB=...").
set -e
cd "$(dirname "$0")/.."
PKG=$(ls -d *_amd)
name=$1; flags=$2; shift 2
mkdir -p "variants/$name/build"
if [ $# -gt 0 ]; then
  make -s -C "$PKG" -j"${JOBS:-8}" lib/libpanofuse.so
  cp "$PKG"/build/*.o "variants/$name/build/"
  for o in "$@"; do rm -f "variants/$name/build/$o.o"; done
  touch "variants/$name/build/"*.o
fi
make -s -C "$PKG" -j"${JOBS:-8}" BDIR="../variants/$name/build" LDIR="../variants/$name/lib" \
  HIPFLAGS_EXTRA="$flags" "../variants/$name/lib/libpanofuse.so"
echo "variants/$name/lib/libpanofuse.so"
