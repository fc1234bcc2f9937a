#!/bin/bash
# Per-pass launch cost in the Jacobi planner (PF_JLAUNCH, cost units of best_chunks; ~10 ns each
# at C3): C5 one-call stage times (batch 1), and the C3 bench line with its C2 latency.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/jl
mkdir -p $O
export TMPDIR=/tmp
for v in 0 300 1000 3000; do
  PF_JLAUNCH=$v PF_JPLAN=1 timeout -k 10 200 python3 tools/c5_stages.py > $O/c5_$v.log 2>&1 || { echo "c5 $v rc=$?"; tail -3 $O/c5_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/c5_$v.log') if l.startswith('{')][-1]); print('JLAUNCH $v C5 stages', {k: round(x, 3) for k, x in d['stage_ms'].items() if x})"
  grep "jacobi plan" $O/c5_$v.log | sort -u | sed 's/T[0-9]*\/n[0-9]* //g' | head -0
  grep "jacobi plan" $O/c5_$v.log | sort -u | awk '{print "   ", $3, NF-10, "passes:", $11, $12, $NF}'
done
for v in 0 1000; do
  PF_JLAUNCH=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --prof-steps 3 > $O/b_$v.log 2>&1 || { echo "bench $v rc=$?"; tail -3 $O/b_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/b_$v.log') if l.startswith('{')][-1]); print('JLAUNCH $v C3 %.0f/s jacobi %.3f c2 %.3f ms c5 %.1f/s one-call %.3f ms bit_exact %s' % (d['value'], d['stages']['jacobi']['ms_per_step'], d['c2_batch1_ms'], d['c5_one_gpu']['value'], d['c5_one_gpu']['one_call_ms'], d['bit_exact_vs_one_process']))"
done
