#!/bin/bash
# A/B of the resident level-0 kernel in the real step: bench (pipelined, default) with the
# streaming engine (PF_JRES=0), the 8-wave resident kernel (default) and the 16-wave build
# (tools/ubench/bin/w16), alternating; then the kernels' own times with the side-stream target
# gathers off (PF_NOSIDE=1) and on.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/jres_ab${TAG:-}
mkdir -p $OUT
W16=$PWD/tools/ubench/bin/w16/libpanofuse.so
for r in 1 2 3; do
  for m in stream w8 w16; do
    case $m in
      stream) envs="PF_JRES=0" ;;
      w8) envs="PF_JRES=1" ;;
      w16) envs="PANOFUSE_LIB=$W16" ;;
    esac
    env $envs timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b_${m}_$r.log 2>&1 || exit 1
    tail -1 $OUT/b_${m}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$m' round '$r'", round(d["value"]), "pano/s", round(d["ms_per_step"], 3), "ms", {k: round(v["ms_per_step"], 3) for k, v in d["stages"].items()})'
  done
done
VARIANTS="noside:PF_NOSIDE=1 noside_dbg1:PF_NOSIDE=1,PF_JRES_DBG=1 w16:PANOFUSE_LIB=$W16 w16_noside:PANOFUSE_LIB=$W16,PF_NOSIDE=1 w16_dbg1:PANOFUSE_LIB=$W16,PF_NOSIDE=1,PF_JRES_DBG=1" TAG=_ab bash tools/jres_probe.sh
