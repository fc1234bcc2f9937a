#!/bin/bash
# SQ issue counters of the Jacobi kernels in serial fusions (one rocprofv3 --pmc pass per group).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PMC_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-extra-configs --prof-steps 1 --pipeline 0"
bash tools/pmc.sh jsq_a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_INSTS_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE || { echo "pass a rc=$?"; tail -3 gpurun_out/pmc_jsq_a.log; exit 1; }
bash tools/pmc.sh jsq_b SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES \
  SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_LDS || { echo "pass b rc=$?"; tail -3 gpurun_out/pmc_jsq_b.log; exit 1; }
python3 tools/pmc_summary.py "gpurun_out/pmc_jsq_a/*counter_collection.csv" "gpurun_out/pmc_jsq_b/*counter_collection.csv" \
  > gpurun_out/jsq_summary.txt
grep -A18 "k_jlag\|k_jres" gpurun_out/jsq_summary.txt | head -80
