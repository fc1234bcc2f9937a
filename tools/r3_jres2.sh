#!/bin/bash
# Resident kernel: parity, then the A/B bench (tools/jres_ab.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_jres.py > gpurun_out/r3/jres_tests.log 2>&1 || { tail -40 gpurun_out/r3/jres_tests.log; exit 1; }
tail -2 gpurun_out/r3/jres_tests.log
PANOFUSE_LIB=$PWD/tools/ubench/bin/w16/libpanofuse.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_jres.py > gpurun_out/r3/jres_tests16.log 2>&1 || { tail -40 gpurun_out/r3/jres_tests16.log; exit 1; }
tail -2 gpurun_out/r3/jres_tests16.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_lm.py -k "register or lm" > gpurun_out/r3/reg_tests.log 2>&1 || { tail -40 gpurun_out/r3/reg_tests.log; exit 1; }
tail -2 gpurun_out/r3/reg_tests.log
bash tools/jres_ab.sh
