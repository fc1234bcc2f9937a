#!/bin/bash
# Warp kernel round-3 check: parity tests, then the SQ/probe comparison new vs old library
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "warp" > gpurun_out/r3/warp_tests.log 2>&1 || { tail -30 gpurun_out/r3/warp_tests.log; exit 1; }
tail -2 gpurun_out/r3/warp_tests.log
bash tools/warp_sq.sh || exit 1
python3 tools/warp_sq_summary.py gpurun_out/warp_sq
