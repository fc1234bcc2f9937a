#!/bin/bash
# HBM-traffic PMC passes over one short bench run, one rocprofv3 --pmc pass per counter group
# (gfx950: FETCH_SIZE and WRITE_SIZE cannot share a pass).  Each pass has its own kill timer;
# a failed pass ends the script.  Summaries: tools/pmc_traffic.py -> gpurun_out/pmc_traffic.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="${PMC_ARGS:---steps 1 --warmup 1 --no-cpu-baseline --no-extra-configs --prof-steps 1}"
pass() {
  local name=$1; shift
  timeout -k 5 -s KILL 240 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$name -o run --output-format csv -- \
    python3 bench.py $ARGS > gpurun_out/pmc_$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass rdreq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
# the RGB warp (outside the bench's step; bench.py's roofline_warp_rgb): the same three passes
# over tools/rgb_probe.py
rgbpass() {
  local name=$1; shift
  timeout -k 5 -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pmc_rgb_$name -o run --output-format csv -- \
    python3 tools/rgb_probe.py --reps 2 > gpurun_out/pmc_rgb_$name.log 2>&1
  local rc=$?
  echo "pmc rgb $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
rgbpass fetch FETCH_SIZE
rgbpass write WRITE_SIZE
rgbpass rdreq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
python3 tools/pmc_traffic.py gpurun_out > gpurun_out/pmc_traffic.txt && cat gpurun_out/pmc_traffic.txt
