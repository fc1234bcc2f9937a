#!/bin/bash
# Build library variants with extra compile flags into lib/variants/ (run here, on the CPU): each
# variant is the package Makefile run in a scratch copy with HIPFLAGS_EXTRA set.
# Usage: tools/variants.sh NAME "FLAGS" [NAME "FLAGS" ...]
# With ONLY="csrc/x.hip ..." the scratch copy starts from the current build/ objects and only
# those sources are recompiled with the flags (the flags must not affect the other files).
set -e
cd "$(dirname "$0")/.."
PKG=$(ls -d wacv2023-*_amd)
mkdir -p $PKG/lib/variants
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  W=/tmp/pfvar_$name
  rm -rf $W && mkdir -p $W/pkg $W/include
  cp -r $PKG/csrc $PKG/Makefile $W/pkg/ && cp include/*.h $W/include/
  if [ -n "${ONLY:-}" ]; then
    cp -rp $PKG/build $W/pkg/
    sleep 1
    for f in $ONLY; do touch $W/pkg/$f; done
  fi
  make -s -j8 -C $W/pkg lib/libpanofuse.so HIPFLAGS_EXTRA="$flags" > $W/build.log 2>&1 || { tail -20 $W/build.log; exit 1; }
  cp $W/pkg/lib/libpanofuse.so $PKG/lib/variants/libpanofuse_$name.so
  echo "built $name: $flags"
done
