#!/bin/bash
# Resident level kernel: parity (vs the streaming engine and the oracle), then per-level times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_jres.py > gpurun_out/r3/jres_tests.log 2>&1 || { tail -40 gpurun_out/r3/jres_tests.log; exit 1; }
tail -3 gpurun_out/r3/jres_tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py -k "fuse or merge or internals or c3" \
  > gpurun_out/r3/jres_parity.log 2>&1 || { tail -40 gpurun_out/r3/jres_parity.log; exit 1; }
tail -3 gpurun_out/r3/jres_parity.log
TAG=_jres BENCH_ARGS="--pipeline 0" bash tools/jprobe.sh > gpurun_out/r3/jprobe_jres.txt 2>&1
cat gpurun_out/r3/jprobe_jres.txt
