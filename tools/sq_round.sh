#!/bin/bash
# SQ (issue/stall) PMC pass + clock over one short bench run, and the Jacobi pass plans.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 5 120 env PF_JPLAN=1 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline \
  > gpurun_out/jplan.log 2>&1 || exit $?
grep "jacobi plan" gpurun_out/jplan.log | sort | uniq
timeout -k 5 -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE \
  -d gpurun_out/pmc_sq -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sq.log 2>&1 || exit $?
python3 tools/pmc_summary.py 'gpurun_out/pmc_sq/*counter_collection.csv' > gpurun_out/pmc_sq.txt
head -60 gpurun_out/pmc_sq.txt
