#!/bin/bash
# SQ issue counters of the resident level kernel (and the streaming passes beside it), serial
# steps with the side-stream gathers off.  Two PMC passes, each within the per-block limits.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/jres_sq${TAG:-}
mkdir -p $O
export PF_NOSIDE=1
timeout -k 5 -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE \
  -d $O/a -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --pipeline 0 \
  > $O/a.log 2>&1 || exit 1
timeout -k 5 -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
  SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA \
  -d $O/b -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --pipeline 0 \
  > $O/b.log 2>&1 || exit 1
python3 tools/pmc_summary.py "$O/a/*/run_counter_collection.csv" "$O/b/*/run_counter_collection.csv" "$O/a/run_counter_collection.csv" "$O/b/run_counter_collection.csv" > $O/summary.txt
grep -A 18 "k_jres\|k_jlag<2, 10, 0, false, true> grid=4" $O/summary.txt | head -80
