set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_warp_maps.py > gpurun_out/pitch_tests.log 2>&1 && tail -2 gpurun_out/pitch_tests.log && \
LIBS="nopitch" bash tools/r4_warp_diag.sh && LIBS="nopitch" bash tools/r4_warp_diag.sh
