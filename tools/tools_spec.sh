#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
VARS="base nospec base nospec" bash tools/tools_var.sh && VARS="base nospec" bash tools/tools_c5ab.sh || exit 1
for v in nospec base; do
  if [ $v = base ]; then L=cudatracerlib_amd/_lib/libctl_trace.so; else L=cudatracerlib_amd/_var$v/libctl_trace.so; fi
  CTL_LIB=$PWD/$L timeout -k 10 400 python probes/shard_diag.py > gpurun_out/diag_$v.log 2>&1 || { echo FAIL; tail gpurun_out/diag_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/diag_$v.log | tail -8
done
