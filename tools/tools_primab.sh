#!/bin/bash
# PrimTracer on C3 1080p (probes/prim_bench.py) for variant libraries: VARS="base name ..."
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARS:-base}; do
  if [ $v = base ]; then L=cudatracerlib_amd/_lib/libctl_trace.so; else L=cudatracerlib_amd/_var$v/libctl_trace.so; fi
  echo "== $v"
  CTL_LIB=$PWD/$L timeout -k 10 300 python probes/prim_bench.py > gpurun_out/prim_$v.log 2>&1 || { echo FAIL; tail gpurun_out/prim_$v.log; exit 1; }
  grep "ms/pass" gpurun_out/prim_$v.log
done
