#!/bin/bash
# Full GPU pass: every -m gpu test, smoke(), then the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/r3/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/r3/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # 1 = test failures (read the log); else stop
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r3/bench.log 2>&1 || exit 1
tail -1 gpurun_out/r3/bench.log | head -c 600
