#!/bin/bash
# On the GPU box: short bench of every lib/variants/*.so (and the default build), one line each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PKG=$(ls -d wacv2023-*_amd)
mkdir -p gpurun_out
for so in $PKG/lib/libpanofuse.so $PKG/lib/variants/*.so; do
  timeout -k 5 120 env PANOFUSE_LIB=$so python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/var_$(basename $so .so).log 2>&1 || { echo "$so failed rc=$?"; tail -5 gpurun_out/var_$(basename $so .so).log; exit 1; }
  python3 - "$so" gpurun_out/var_$(basename $so .so).log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().split("\n")[-1])
st = d["stages"]
print(f"{sys.argv[1].split('/')[-1]:34s} {d['value']:8.0f} panos/s  {d['ms_per_step']:.3f} ms/step  "
      + "  ".join(f"{k} {v['ms_per_step']:.3f}" for k, v in st.items() if v['ms_per_step'] > 0))
PY
done
