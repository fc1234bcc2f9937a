#!/bin/bash
# Round 3: wave-owned warp boxes (PF_WARP_WAVEBOX variants) -- timing probe of each variant, then
# the warp parity tests and a short bench on the wb2k variant (PANOFUSE_LIB).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PKG=wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-registrations_amd
VARIANTS="base wb wb2k wb2k32" bash tools/r3_warp2.sh || exit 1
export PANOFUSE_LIB=$PWD/$PKG/lib/variants/libpanofuse_${WB:-wb2k}.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/wv2/wb_pytest.log 2>&1 || { tail -30 gpurun_out/wv2/wb_pytest.log; exit 1; }
tail -1 gpurun_out/wv2/wb_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/wv2/wb_bench.log 2>&1 || { tail -5 gpurun_out/wv2/wb_bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/wv2/wb_bench.log').read().strip().splitlines()[-1]); print('wb bench', round(d['value']), round(d['ms_per_step'],3), d['stages']['warp']['ms_per_step'])"
