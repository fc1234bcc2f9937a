#!/bin/bash
# Warp-kernel session on the GPU box: tools/warp_probe.py timings, then HBM-traffic and SQ PMC
# passes over the probe (one rocprofv3 --pmc pass per counter group, each under its own timer).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/warp
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 180 python3 tools/warp_probe.py > $OUT/probe.log 2>&1 || { tail -5 $OUT/probe.log; exit 1; }
tail -1 $OUT/probe.log
pass() {
  local name=$1; shift
  timeout -k 5 -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/pmc_$name -o run --output-format csv -- \
    python3 tools/warp_probe.py > $OUT/pmc_$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass rdreq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
pass sq SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE
python3 tools/pmc_traffic.py $OUT > $OUT/traffic.txt && cat $OUT/traffic.txt
python3 tools/pmc_summary.py "$OUT/pmc_sq/*counter_collection.csv" > $OUT/sq.txt; grep -A12 warp_depth $OUT/sq.txt | head -30
