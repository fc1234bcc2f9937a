#!/bin/bash
# A/B of the depth warp's region cuts (PF_WARP_CUT) on the GPU box: kernel time (warp_probe.py),
# a kernel trace, and PMC read/write bytes per k_warp_depth launch.  Output under gpurun_out/warp_ab/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/warp_ab
mkdir -p $o
for cut in ${CUTS:-strip pixel}; do for ord in ${ORDERS:-0}; do export PF_WARP_ORDER=$ord; tag=${cut}_o$ord
  PF_WARP_CUT=$cut PF_WARP_STATS=1 timeout -k 10 120 python3 tools/warp_probe.py > $o/probe_$tag.txt 2>&1 || exit 1
  PF_WARP_CUT=$cut timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o/kt_$tag -o run --output-format csv -- \
    python3 tools/warp_probe.py > $o/kt_$tag.log 2>&1 || exit 1
  PF_WARP_CUT=$cut timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $o/pmc_$tag/f -o run --output-format csv -- \
    python3 tools/warp_probe.py > $o/pmcf_$tag.log 2>&1 || exit 1
  PF_WARP_CUT=$cut timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $o/pmc_$tag/w -o run --output-format csv -- \
    python3 tools/warp_probe.py > $o/pmcw_$tag.log 2>&1 || exit 1
done; done
