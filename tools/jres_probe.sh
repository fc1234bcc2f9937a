#!/bin/bash
# Resident level kernel timing probes (serial steps): default, then the profiling-only variants
# PF_JRES_DBG=1 (no hand-offs) / 2 (no LDS edges, no barriers) / 3 (neither), and forced blockings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/jresp${TAG:-}
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/$name -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipeline 0 > $OUT/$name.log 2>&1 || return 1
  python3 - "$name" $(find $OUT/$name -name "run_kernel_trace.csv" | head -1) <<'PY'
import csv, sys
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in csv.DictReader(open(sys.argv[2])) if "k_jres" in r["Kernel_Name"]]
d = d[-4:]
print(f"{sys.argv[1]:12s} k_jres us: " + " ".join(f"{x:.1f}" for x in d))
PY
}
run default PF_JPLAN=1 || exit 1
grep "resident" $OUT/default.log | sort | uniq -c
for v in ${VARIANTS:-dbg1:PF_JRES_DBG=1 dbg2:PF_JRES_DBG=2 dbg3:PF_JRES_DBG=3 nb3:PF_JRES_NB=3 nb5:PF_JRES_NB=5 nb6:PF_JRES_NB=6}; do
  run ${v%%:*} $(echo ${v#*:} | tr "," " ") || exit 1
done
