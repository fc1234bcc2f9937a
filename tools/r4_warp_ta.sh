#!/bin/bash
# k_warp_depth (tools/warp_probe.py): the per-CU vector-memory address path (TA) and data path (TD):
# busy and stall cycles, two counters of each block per rocprofv3 --pmc pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/wta
rm -rf $O; mkdir -p $O
i=0
for set in "TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TCP_STALL_CYCLES_sum TD_SPI_STALL_sum" \
           "TA_BUFFER_COALESCED_READ_CYCLES_sum TA_BUFFER_COALESCED_WRITE_CYCLES_sum"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/p$i -o run --output-format csv -- python3 tools/warp_probe.py \
    > $O/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 $O/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py "$O/p*/*counter_collection.csv" | grep -A14 "k_warp_depth" | tee $O/summary.txt
