#!/bin/bash
# Round-4 check at HEAD: every -m gpu test (up to 5 failures reported), then the default bench
# line.  Each GPU step has its own time limit; a crash / abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -m gpu --maxfail 5 --timeout 180 \
  --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 3000 $OUT/bench.log
exit $rc
