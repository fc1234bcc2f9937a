#!/bin/bash
# Round-4 evidence at HEAD (everything lands under gpurun_out/r4ev/, copied into profiles/r04/):
#   1. serial-step rocprofv3 kernel trace + stats (per-level Jacobi split, tools/ktrace_levels.py)
#   2. the default (pipelined) bench under rocprofv3 --kernel-trace --stats
#   3. HBM-traffic PMC passes (tools/pmc_round.sh -> pmc_traffic.json)
# Every GPU step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4ev
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs --pipeline 0 \
  > $O/serial_bench.log 2>&1 || { echo "serial rc=$?"; tail -5 $O/serial_bench.log; exit 1; }
T=$(find $O/serial -name "run_kernel_trace.csv" | head -1)
python3 tools/r4_fusions.py $T > $O/serial_fusions.txt
python3 tools/trace_summary.py $T > $O/serial_summary.txt
echo "serial done"; tail -4 $O/serial_fusions.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pipelined -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs \
  > $O/pipelined_bench.log 2>&1 || { echo "pipelined rc=$?"; tail -5 $O/pipelined_bench.log; exit 1; }
echo "pipelined done"
bash tools/pmc_round.sh > $O/pmc_round.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc_round.log; exit 1; }
cp gpurun_out/pmc_traffic.txt gpurun_out/pmc_traffic.json $O/
grep -E "k_warp_depth|k_jres|k_jlag|k_targets|k_register" $O/pmc_traffic.txt
echo "all done"
