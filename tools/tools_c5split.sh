#!/bin/bash
# C5 material-class split (probes/c5_material_split.py) of variant libraries: VARS="base old"
set -o pipefail
mkdir -p gpurun_out/c5split
export TMPDIR=/tmp
for v in ${VARS:-base}; do
  if [ $v = base ]; then L=cudatracerlib_amd/_lib/libctl_trace.so; else L=cudatracerlib_amd/_var$v/libctl_trace.so; fi
  CTL_LIB=$PWD/$L timeout -k 10 400 python probes/c5_material_split.py > gpurun_out/c5split/$v.txt 2>&1 || { echo "SPLIT $v FAILED"; tail -20 gpurun_out/c5split/$v.txt; exit 1; }
  echo "== $v"; grep "ms/pass" gpurun_out/c5split/$v.txt
done
