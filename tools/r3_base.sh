#!/bin/bash
# Round-3 baseline on the GPU box: the warp's HBM ceiling (tools/ubench/stream_mix) and the
# per-level Jacobi pass times of serial steps at HEAD (tools/jprobe.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3
timeout -k 10 120 tools/ubench/bin/stream_mix > gpurun_out/r3/stream_mix.txt 2>&1 || exit $?
cat gpurun_out/r3/stream_mix.txt
TAG=_base BENCH_ARGS="--pipeline 0" bash tools/jprobe.sh > gpurun_out/r3/jprobe_base.txt 2>&1 || exit $?
cat gpurun_out/r3/jprobe_base.txt
