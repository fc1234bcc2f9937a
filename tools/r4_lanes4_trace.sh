#!/bin/bash
# Why four lanes are slow: kernel traces of 2 and 4 pipelined lanes, per-family kernel time per
# step (tools/lanes_overlap.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/l4trace
rm -rf $O; mkdir -p $O
for p in 4 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p$p -o run --output-format csv -- \
    python3 bench.py --pipeline $p --steps 20 --warmup 3 --no-cpu-baseline --no-extra-configs \
    --prof-steps 1 > $O/p$p.log 2>&1 || { echo "p$p rc=$?"; tail -5 $O/p$p.log; exit 1; }
  T=$(find $O/p$p -name "*kernel_trace.csv" | head -1)
  echo "== lanes $p"; python3 tools/lanes_overlap.py $T | tee $O/p$p.overlap.txt
done
