#!/bin/bash
# Round 3: co-scheduled half-batch fusions vs the default step, alternating.  The PF_SPLIT knob
# lived in bench.py for this A/B only (measured slower, removed).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/split
for r in 1 2; do
  for v in "1 0" "2 0" "2 1"; do
    set -- $v
    PF_SPLIT=$1 PF_SPLIT_LEVEL=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      > gpurun_out/split/s$1_l$2_$r.log 2>&1 || { echo "split $v failed"; tail -5 gpurun_out/split/s$1_l$2_$r.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],3), d.get('bit_exact_vs_one_process'))" gpurun_out/split/s$1_l$2_$r.log "split=$1 level=$2"
  done
done
