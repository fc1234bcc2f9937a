#!/bin/bash
# Serial-step kernel traces of several library builds (LIBS: "default" or variant names under
# lib/variants/libpanofuse_NAME.so): per-kernel averages and the per-level Jacobi split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-registrations_amd
for v in ${LIBS:-default}; do
  O=gpurun_out/trace_$v
  rm -rf $O; mkdir -p $O
  if [ "$v" = default ]; then L=$(pwd)/$P/lib/libpanofuse.so; else L=$(pwd)/$P/lib/variants/libpanofuse_$v.so; fi
  PANOFUSE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run \
    --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline \
    --no-extra-configs --pipeline ${PIPE:-0} ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo "$v rc=$?"; tail -3 $O/bench.log; exit 1; }
  T=$(find $O/prof -name "run_kernel_trace.csv" | head -1)
  python3 tools/ktrace_levels.py $T > $O/levels.txt
  python3 tools/trace_summary.py $T > $O/summary.txt
  python3 tools/r4_gaps.py $T > $O/gaps.txt
  echo "== $v"; cat $O/levels.txt; head -12 $O/summary.txt; head -30 $O/gaps.txt
done
