#!/bin/bash
# Under the two-lane default, the row chunking of the streamed levels (PF_JN<w> overrides the cost
# model's choice): fewer chunks waste less fill/drain, the other lane fills the chip.  Alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/lplan
mkdir -p $O
export TMPDIR=/tmp
PF_JPLAN=1 timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra-configs \
  --prof-steps 1 > $O/plan.log 2>&1 && grep "jacobi plan" $O/plan.log | sort | uniq | head -8
for r in 1 2; do
  for v in "base:" "n1k2:PF_JN1024=2" "n2k3:PF_JN2048=3" "n2k2:PF_JN2048=2" "both2:PF_JN1024=2,PF_JN2048=2" "n1k4:PF_JN1024=4"; do
    name=${v%%:*}; envs=${v#*:}
    ( for kv in ${envs//,/ }; do [ -n "$kv" ] && export "$kv"; done
      timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra-configs \
        --prof-steps 1 > $O/$name.$r.log 2>&1 ) || { echo "$name rc=$?"; tail -5 $O/$name.$r.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/$name.$r.log') if l.startswith('{')][-1]); print('$name round $r: %.0f panoramas/s  %.3f ms/step  jacobi(serial) %.3f  bit_exact %s' % (d['value'], d['ms_per_step'], d['stages']['jacobi']['ms_per_step'], d['bit_exact_vs_one_process']))"
  done
done
