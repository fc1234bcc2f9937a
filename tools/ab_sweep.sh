#!/bin/bash
# Rebuild the library with extra compile flags, then run a Jacobi tuning sweep.
# Usage: FLAGS="-DPF_JLAG_STAGEWISE=0" SWEEP="8:0:0 ..." tools/ab_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PKG=wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-registrations_amd
touch $PKG/csrc/*.hip
make -s -C $PKG HIPFLAGS_EXTRA="$FLAGS" > gpurun_out/ab_build.log 2>&1 || { echo build failed; exit 1; }
echo "flags: $FLAGS"
bash tools/jsweep.sh
