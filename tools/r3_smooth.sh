#!/bin/bash
# Round 3: list-driven SolveDepthBySmoothing -- parity (oracle, facade) then the bench's timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/smooth
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_smoothing.py tests/test_facade.py tests/test_gpu_parity.py > gpurun_out/smooth/pytest.log 2>&1 \
  || { tail -30 gpurun_out/smooth/pytest.log; exit 1; }
tail -2 gpurun_out/smooth/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/smooth/bench.log 2>&1 || { tail -5 gpurun_out/smooth/bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/smooth/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['smoothing_ablation'], d['stages']['warp'])"
