#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c5pmc
ARGS="--config 5 --steps 1 --warmup 0 --no-cpu-baseline --wpt-passes 0 --closest-shadow-passes 0"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU" \
           "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR TA_TA_BUSY_sum GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32"; do
  i=$((i+1))
  echo "group $i"
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/c5pmc/g$i -o run -- python3 bench.py $ARGS > gpurun_out/c5pmc/g$i.json 2> gpurun_out/c5pmc/g$i.err || { echo "group $i failed"; tail -3 gpurun_out/c5pmc/g$i.err; exit 1; }
done
