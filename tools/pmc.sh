#!/bin/bash
# One rocprofv3 PMC pass over a short bench run (counters given as arguments).
# Usage: tools/pmc.sh NAME COUNTER... ; output under gpurun_out/pmc_NAME/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
name=$1; shift
# PMC_SCRIPT (default bench.py) and PMC_ARGS select the profiled python program
timeout -k 10 600 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$name -o run --output-format csv -- \
  python3 ${PMC_SCRIPT:-bench.py} ${PMC_ARGS:---steps 2 --warmup 1 --no-cpu-baseline} \
  > gpurun_out/pmc_$name.log 2>&1
