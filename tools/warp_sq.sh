#!/bin/bash
# SQ issue / LDS counters of k_warp_depth for the current library and, if present, the round-2
# library ($OLD_LIB, default tools/ubench/bin/old_libpanofuse.so, built from git): output under
# gpurun_out/warp_sq/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/warp_sq
mkdir -p $o
for tag in new old; do
  lib=""
  if [ $tag = old ]; then
    lib=${OLD_LIB:-$PWD/tools/ubench/bin/old_libpanofuse.so}
    [ -f "$lib" ] || continue
  fi
  PANOFUSE_LIB=$lib timeout -k 10 120 python3 tools/warp_probe.py > $o/probe_$tag.txt 2>&1 || exit 1
  PANOFUSE_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    -d $o/a_$tag -o run --output-format csv -- python3 tools/warp_probe.py > $o/a_$tag.log 2>&1 || exit 1
  PANOFUSE_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES \
    -d $o/b_$tag -o run --output-format csv -- python3 tools/warp_probe.py > $o/b_$tag.log 2>&1 || exit 1
done
