#!/bin/bash
# Round 3: target-gather variants A/B through the bench (stage times from the library's events).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PKG=wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-registrations_amd
mkdir -p gpurun_out/tgt
for r in 1 2; do
  for v in ${VARIANTS:-base tgtnt tgtnb4 tgtnb16}; do
    if [ $v = base ]; then unset PANOFUSE_LIB; else export PANOFUSE_LIB=$PWD/$PKG/lib/variants/libpanofuse_$v.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/tgt/$v.$r.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/tgt/$v.$r.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],3), 'targets', round(d['stages']['targets']['ms_per_step'],3), 'jacobi', round(d['stages']['jacobi']['ms_per_step'],3), d['bit_exact_vs_one_process'])" gpurun_out/tgt/$v.$r.log $v
  done
done
