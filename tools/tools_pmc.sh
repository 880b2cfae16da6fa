#!/bin/bash
# PMC counters of the pass kernels: one rocprofv3 --pmc run per counter group
# (kernel trace only: no sys/runtime/hip trace domains beside --pmc), each a
# one-step bench.py run without the WPT leg.  FETCH_SIZE and WRITE_SIZE need
# separate runs (TCC slots).  Summary: gpurun_out/pmc/pmc.json (tools_pmc_summary.py).
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--steps 8 --warmup 0 --ceiling 0 --no-cpu-baseline --binary-passes 0 --wpt-passes 0 --closest-shadow-passes 0 --one-pass-leg 0 --prim-passes 0 --c5-passes 0 --dopass-leg 0 --anim-iters 0 $*"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU" \
           "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  echo "pmc group $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/g$i -o run -- python3 bench.py $ARGS > gpurun_out/pmc/g$i.json 2> gpurun_out/pmc/g$i.err || { echo "PMC group $i failed"; tail -5 gpurun_out/pmc/g$i.err; exit 1; }
done
python3 tools/tools_pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt && cat gpurun_out/pmc/summary.txt
