#!/bin/bash
# PMC counters of the pass kernels, one rocprofv3 pass per counter group
# (kernel trace only; no sys/runtime/hip trace domains with --pmc).
# FETCH_SIZE and WRITE_SIZE need separate passes (TCC slots).
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu-baseline $*"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/g$i -o run -- python3 bench.py $ARGS > gpurun_out/pmc/g$i.json 2> gpurun_out/pmc/g$i.err || { echo "PMC group $i failed"; tail -5 gpurun_out/pmc/g$i.err; exit 1; }
done
python3 tools_pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt && cat gpurun_out/pmc/summary.txt
