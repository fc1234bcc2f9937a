#!/bin/bash
# Quick GPU check: selected -m gpu test files ($TESTS), then $NB default bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4q
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -v -m gpu --maxfail 5 --timeout 180 \
    --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -8 $OUT/pytest.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
for i in $(seq 1 ${NB:-1}); do
  timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $OUT/bench.$i.log 2>&1; rc=$?
  echo "bench $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/bench.$i.log; exit $rc; }
  python - $OUT/bench.$i.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
st = d["stages"]
print(f"value {d['value']:.0f}  ms/step {d['ms_per_step']:.3f}  " +
      "  ".join(f"{k} {v['ms_per_step']:.3f}" for k, v in st.items() if v["ms_per_step"]))
PY
done
