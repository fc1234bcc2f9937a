set -o pipefail
mkdir -p gpurun_out/jsq
timeout -k 5 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d gpurun_out/jsq/a -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra-configs --pipeline 0 > gpurun_out/jsq/a.log 2>&1 || exit $?
timeout -k 5 -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS -d gpurun_out/jsq/b -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra-configs --pipeline 0 > gpurun_out/jsq/b.log 2>&1 || exit $?
echo done
