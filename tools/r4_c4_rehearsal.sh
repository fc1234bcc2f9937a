#!/bin/bash
# C4's 8-rank path on the one-GPU box: bench.py --gpus 8 launches its own 8 ranks (gloo, every rank
# on cuda:0), batch 64 per rank = 512 panoramas per step, then the C5 row-sharded mode over 8 ranks.
# The ranks share one GPU, so the rate is not a scaling number: this checks the launcher, the seed
# partition, the max-over-ranks timing and bit_exact_vs_one_process at C4's shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/c4r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py --gpus 8 --same-device --backend gloo --steps 3 --warmup 1 \
  --no-cpu-baseline --no-extra-configs --prof-steps 1 > $O/c4_8rank.log 2>&1 || { echo "c4 rc=$?"; tail -20 $O/c4_8rank.log; exit 1; }
tail -c 1500 $O/c4_8rank.log; echo
timeout -k 10 600 python3 bench.py --gpus 8 --same-device --backend gloo --mode c5 --steps 2 --warmup 1 \
  --no-cpu-baseline --no-extra-configs --prof-steps 1 > $O/c5_8rank.log 2>&1 || { echo "c5 rc=$?"; tail -20 $O/c5_8rank.log; exit 1; }
tail -c 1500 $O/c5_8rank.log
