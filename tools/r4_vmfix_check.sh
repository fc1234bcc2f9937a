#!/bin/bash
# The warp's loop-header vmcnt fix (PF_WARP_VMFIX): warp parity tests on the new default library,
# then tools/warp_probe.py timings alternating default / lib/variants/libpanofuse_novmfix.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_configs.py > gpurun_out/vmfix_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/vmfix_tests.log; exit 1; }
tail -2 gpurun_out/vmfix_tests.log
for r in 1 2; do LIBS="novmfix" bash tools/r4_warp_diag.sh || exit 1; done
