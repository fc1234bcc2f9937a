#!/bin/bash
# Serial-step (no pipelining) kernel trace + stats of the C3 bench: the committed basis of the
# Jacobi stage's VALU fraction (per-level times via tools/ktrace_levels.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/serial${TAG:-}
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --pipeline 0 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c 1-400
python3 tools/ktrace_levels.py $(find $O/prof -name "run_kernel_trace.csv" | head -1) > $O/levels.txt
cat $O/levels.txt
