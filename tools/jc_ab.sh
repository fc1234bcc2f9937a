#!/bin/bash
# Packed C=4 Jacobi A/B: parity tests with C=4 forced, then bench at the cost model's choice,
# C=2 forced and C=4 forced (plans printed), and a kernel trace of the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/jc; rm -rf $OUT; mkdir -p $OUT
PF_JC=4 timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_c4.log 2>&1; rc=$?
tail -2 $OUT/pytest_c4.log; [ $rc -eq 0 ] || exit $rc
for v in auto 2 4; do
  if [ $v = auto ]; then unset PF_JC; else export PF_JC=$v; fi
  PF_JPLAN=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > $OUT/b_$v.log 2>&1 || { tail -3 $OUT/b_$v.log; exit 1; }
  grep "jacobi plan" $OUT/b_$v.log | sort | uniq | cut -c1-150
  python3 -c "import json; d=json.loads(open('$OUT/b_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],3), 'jacobi', round(d['stages']['jacobi']['ms_per_step'],3))"
done
unset PF_JC
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
python3 tools/trace_summary.py $OUT/prof/run_kernel_trace.csv | head -14
