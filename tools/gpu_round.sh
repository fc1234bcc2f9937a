#!/bin/bash
# GPU-box session recipes, one step per word of $STEPS (default: tests smoke bench prof).  Every
# GPU step has its own time limit; a crash / abort / timeout (exit >= 2 other than pytest's
# test-failure code 1) ends the script before any further GPU step.  Outputs under gpurun_out/.
#
#   tests    the -m gpu suite                        -> pytest_gpu.log
#   smoke    __graft_entry__.smoke()                  -> smoke.log
#   bench    the default bench line (C3, two lanes)   -> bench.log
#   prof     kernel trace + stats of a short bench    -> prof/
#   serial   kernel trace of serial steps (--pipeline 0) and the per-level Jacobi times
#            (tools/ktrace_levels.py): the basis of the Jacobi roofline -> serial/
#   pmc      HBM-traffic PMC passes (tools/pmc_round.sh) -> pmc_traffic.txt
#   c5       the C5 line at world 1 (+ the 8-rank byte model)  -> bench_c5.log
#   c4       bench.py --gpus 8 on the one GPU (gloo, --same-device): C4's 8-rank shape
#   rgb      the RGB warp probe (tools/rgb_probe.py)   -> rgb.log
#   warppipe k_warp_depth's vector-memory path counters (TA/TD busy and stalls, three --pmc
#            passes over tools/warp_probe.py)          -> warppipe/summary.txt
#   jsq      SQ counters of the Jacobi kernels over serial steps (two --pmc passes; occupancy,
#            VALU issue, waits)                          -> jsq/summary.txt
#   serials  the serial step per variant: $VARIANTS as for ab -> serial_NAME/levels.txt (one trace
#            each, in $ROUNDS alternating rounds)
#   ab       A/B of environment knobs: $VARIANTS = "NAME:ENV=VAL,ENV=VAL NAME2:" run in $ROUNDS
#            alternating rounds on the default bench line (-> ab/NAME.R.log, one summary line
#            each); BENCH_ARGS adds bench.py flags
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
STEPS="${STEPS:-tests smoke bench prof}"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
summ() {  # one line of a bench JSON: value and stage times
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
st = d.get("stages", {})
print(f"{sys.argv[2]:>10}  value {d['value']:.0f}  ms/step {d['ms_per_step']:.3f}  " +
      "  ".join(f"{k} {v['ms_per_step']:.3f}" for k, v in st.items()
                if v["ms_per_step"] and k != "metrics"))
PY
}
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
      echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log; ok $rc || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1; rc=$?
      echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1; rc=$?
      echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench.log; exit $rc; }; summ $OUT/bench.log bench ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1; rc=$?
      echo "prof rc=$rc"; tail -2 $OUT/prof.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc ;;
    serial)
      rm -rf $OUT/serial; mkdir -p $OUT/serial
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/serial/prof -o run --output-format csv -- \
        python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs --pipeline 0 > $OUT/serial/bench.log 2>&1; rc=$?
      echo "serial rc=$rc"; [ $rc -eq 0 ] || exit $rc
      python3 tools/ktrace_levels.py $(find $OUT/serial/prof -name "run_kernel_trace.csv" | head -1) > $OUT/serial/levels.txt
      tail -12 $OUT/serial/levels.txt ;;
    serials)
      for r in $(seq 1 ${ROUNDS:-1}); do
        for v in ${VARIANTS:-base:}; do
          name=${v%%:*}; envs=${v#*:}; d=$OUT/serial_$name.$r; rm -rf $d; mkdir -p $d
          ( for kv in ${envs//,/ }; do [ -n "$kv" ] && export "$kv"; done
            timeout -k 10 300 rocprofv3 --kernel-trace -d $d/prof -o run --output-format csv -- \
              python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs --pipeline 0 ${BENCH_ARGS:-} > $d/bench.log 2>&1 ); rc=$?
          [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 $d/bench.log; exit $rc; }
          python3 tools/ktrace_levels.py $(find $d/prof -name "run_kernel_trace.csv" | head -1) > $d/levels.txt
          echo "== $name.$r"; cat $d/levels.txt
        done
      done ;;
    pmc)
      bash tools/pmc_round.sh; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
    c5)
      timeout -k 10 300 python bench.py --mode c5 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c5.log 2>&1; rc=$?
      echo "c5 rc=$rc"; tail -c 800 $OUT/bench_c5.log; [ $rc -eq 0 ] || exit $rc ;;
    c4)
      timeout -k 10 600 python3 bench.py --gpus 8 --same-device --backend gloo --steps 3 --warmup 1 \
        --no-cpu-baseline --no-extra-configs --prof-steps 1 > $OUT/c4_8rank.log 2>&1; rc=$?
      echo "c4 rc=$rc"; tail -c 1200 $OUT/c4_8rank.log; [ $rc -eq 0 ] || exit $rc ;;
    rgb)
      timeout -k 10 120 python3 tools/rgb_probe.py > $OUT/rgb.log 2>&1; rc=$?
      echo "rgb rc=$rc"; cat $OUT/rgb.log | tail -2; [ $rc -eq 0 ] || exit $rc ;;
    warppipe)
      rm -rf $OUT/warppipe; mkdir -p $OUT/warppipe; i=0
      for set in "TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
                 "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TCP_STALL_CYCLES_sum TD_SPI_STALL_sum" \
                 "TA_BUFFER_COALESCED_READ_CYCLES_sum TA_BUFFER_COALESCED_WRITE_CYCLES_sum"; do
        i=$((i + 1))
        timeout -k 5 -s KILL 120 rocprofv3 --pmc $set -d $OUT/warppipe/p$i -o run --output-format csv -- \
          python3 tools/warp_probe.py > $OUT/warppipe/p$i.log 2>&1; rc=$?
        [ $rc -eq 0 ] || { echo "warppipe pass $i rc=$rc"; tail -3 $OUT/warppipe/p$i.log; exit $rc; }
      done
      python3 tools/pmc_summary.py "$OUT/warppipe/p*/*counter_collection.csv" | grep -A10 "k_warp_depth" > $OUT/warppipe/summary.txt
      cat $OUT/warppipe/summary.txt ;;
    jsq)
      rm -rf $OUT/jsq; mkdir -p $OUT/jsq; i=0
      for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
                 "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS"; do
        i=$((i + 1))
        timeout -k 5 -s KILL 120 rocprofv3 --pmc $set -d $OUT/jsq/p$i -o run --output-format csv -- \
          python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra-configs --pipeline 0 > $OUT/jsq/p$i.log 2>&1; rc=$?
        [ $rc -eq 0 ] || { echo "jsq pass $i rc=$rc"; tail -3 $OUT/jsq/p$i.log; exit $rc; }
      done
      python3 tools/pmc_summary.py "$OUT/jsq/p*/*counter_collection.csv" | grep -A14 -E "k_jlag|k_jres" > $OUT/jsq/summary.txt
      cat $OUT/jsq/summary.txt | head -60 ;;
    ab)
      mkdir -p $OUT/ab
      for r in $(seq 1 ${ROUNDS:-2}); do
        for v in ${VARIANTS:-base:}; do
          name=${v%%:*}; envs=${v#*:}
          ( for kv in ${envs//,/ }; do [ -n "$kv" ] && export "$kv"; done
            timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra-configs ${BENCH_ARGS:-} \
              > $OUT/ab/$name.$r.log 2>&1 ); rc=$?
          [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 $OUT/ab/$name.$r.log; exit $rc; }
          summ $OUT/ab/$name.$r.log $name
        done
      done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "all done"
