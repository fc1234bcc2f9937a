#!/bin/bash
# GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.  Every GPU step has its own
# time limit; a crash/abort/timeout (exit >= 2 other than pytest's test-failure code 1) ends the
# script before any further GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
STEPS="${STEPS:-tests smoke bench prof}"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
      echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log; ok $rc || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1; rc=$?
      echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1; rc=$?
      echo "bench rc=$rc"; tail -2 $OUT/bench.log; [ $rc -eq 0 ] || exit $rc ;;
    c5)
      timeout -k 10 300 python bench.py --mode c5 --steps 3 --warmup 1 > $OUT/bench_c5.log 2>&1; rc=$?
      echo "c5 rc=$rc"; tail -2 $OUT/bench_c5.log; [ $rc -eq 0 ] || exit $rc ;;
    pmc)
      bash tools/pmc_round.sh; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1; rc=$?
      echo "prof rc=$rc"; tail -2 $OUT/prof.log; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
echo "all done"
