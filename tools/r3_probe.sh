#!/bin/bash
# Round-3 probe bundle on the GPU box: warp SQ counters (new vs round-2 library) and per-level
# Jacobi times for the current library and the PF_JLAG_PF=5 variant (serial steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/warp_sq.sh || exit 1
TAG=_pf2 BENCH_ARGS="--pipeline 0" bash tools/jprobe.sh > gpurun_out/jprobe_pf2.txt 2>&1 || exit 1
if [ -f tools/ubench/bin/pf5_libpanofuse.so ]; then
  PANOFUSE_LIB=$PWD/tools/ubench/bin/pf5_libpanofuse.so TAG=_pf5 BENCH_ARGS="--pipeline 0" \
    bash tools/jprobe.sh > gpurun_out/jprobe_pf5.txt 2>&1 || exit 1
fi
