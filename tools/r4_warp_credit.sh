#!/bin/bash
# k_warp_depth (tools/warp_probe.py): L2 hit rate and the L2->fabric credit stalls of its reads and
# writes (memory back-pressure), one rocprofv3 --pmc pass each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/wcredit
rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum \
  -d $O/a -o run --output-format csv -- python3 tools/warp_probe.py > $O/a.log 2>&1 || { echo "a rc=$?"; tail -3 $O/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum GRBM_GUI_ACTIVE \
  -d $O/b -o run --output-format csv -- python3 tools/warp_probe.py > $O/b.log 2>&1 || { echo "b rc=$?"; tail -3 $O/b.log; exit 1; }
python3 tools/pmc_summary.py "$O/a/*counter_collection.csv" "$O/b/*counter_collection.csv" | grep -A10 "k_warp_depth" | tee $O/summary.txt
