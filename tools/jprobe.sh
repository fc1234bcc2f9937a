#!/bin/bash
# Jacobi probe on the GPU box: the pass plan of every level (PF_JPLAN) and per-level kernel time
# from a rocprofv3 kernel trace of a short bench run.  Extra env (PF_J*) passes through.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/jprobe${TAG:-}
rm -rf $OUT
mkdir -p $OUT
PF_JPLAN=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 || exit $?
grep "jacobi plan" $OUT/bench.log | sort | uniq -c
tail -1 $OUT/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("value", d["value"], "ms", d["ms_per_step"], {k: round(v["ms_per_step"], 3) for k, v in d["stages"].items()})'
python3 tools/ktrace_levels.py $(find $OUT/prof -name "run_kernel_trace.csv" | head -1)
