#!/bin/bash
# Jacobi parity (level internals, bit-exact vs oracle) then per-level pass times (serial steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py -k "level or jacobi or internals or merge" \
  > gpurun_out/jparity.log 2>&1 || { tail -30 gpurun_out/jparity.log; exit 1; }
tail -3 gpurun_out/jparity.log
TAG=${TAG:-_r3} BENCH_ARGS="--pipeline 0" bash tools/jprobe.sh
