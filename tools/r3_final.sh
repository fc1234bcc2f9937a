#!/bin/bash
# Round-3 evidence at HEAD: every -m gpu test, smoke, the default bench line, a pipelined
# rocprofv3 kernel trace, the serial-step trace (per-level Jacobi), and the PMC traffic passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
STEPS="tests smoke bench prof" bash tools/gpu_round.sh || exit 1
TAG=_final bash tools/r3_serial.sh > /dev/null || exit 1
tail -1 gpurun_out/serial_final/levels.txt
bash tools/pmc_round.sh > gpurun_out/pmc_round.log 2>&1 || { tail -5 gpurun_out/pmc_round.log; exit 1; }
grep -E "k_warp_depth|k_jres|k_jlag|k_targets|k_register" gpurun_out/pmc_traffic.txt | head -12
