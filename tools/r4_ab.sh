#!/bin/bash
# A/B of environment knobs on the default bench line: for each round, each variant in $VARIANTS
# ("NAME:ENV=VAL,ENV=VAL" or "NAME:" for none) runs bench.py once; prints value and stages.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    name=${v%%:*}; envs=${v#*:}
    ( for kv in ${envs//,/ }; do [ -n "$kv" ] && export "$kv"; done
      timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra-configs ${BENCH_ARGS:-} \
        > $OUT/$name.$r.log 2>&1 ); rc=$?
    [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 $OUT/$name.$r.log; exit $rc; }
    python - $OUT/$name.$r.log $name <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
st = d["stages"]
print(f"{sys.argv[2]:>10}  value {d['value']:.0f}  ms/step {d['ms_per_step']:.3f}  " +
      "  ".join(f"{k} {v['ms_per_step']:.3f}" for k, v in st.items() if v["ms_per_step"] and k != "metrics"))
PY
  done
done
