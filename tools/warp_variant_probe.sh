cd "${GRAFT_REPO_ROOT:-/root/repo}"
PKG=wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-registrations_amd
for v in ${VARIANTS:-base nb8 nb32 cap4k cap2k base}; do
  if [ $v = base ]; then unset PANOFUSE_LIB; else export PANOFUSE_LIB=$PWD/$PKG/lib/variants/libpanofuse_$v.so; fi
  timeout -k 10 120 python tools/warp_probe.py > gpurun_out/wv_$v.log 2>&1 || { echo "probe $v failed"; tail -3 gpurun_out/wv_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/wv_$v.log)"
done
