#!/bin/bash
# C5 persistent-schedule bench of variant libraries: VARS="base name ..." (cudatracerlib_amd/_var<name>)
set -o pipefail
mkdir -p gpurun_out/c5
export TMPDIR=/tmp
i=0
for v in ${VARS:-base}; do
  if [ $v = base ]; then L=cudatracerlib_amd/_lib/libctl_trace.so; else L=cudatracerlib_amd/_var$v/libctl_trace.so; fi
  CTL_LIB=$PWD/$L timeout -k 10 400 python bench.py --config 5 --steps 16 --warmup 4 --no-cpu-baseline --wpt-passes 0 --dopass-leg 0 --one-pass-leg 0 --closest-shadow-passes 0 --prim-passes 0 --c5-passes 0 > gpurun_out/c5/${i}_$v.json 2> gpurun_out/c5/${i}_$v.err || { echo "C5 $v FAILED"; tail -20 gpurun_out/c5/${i}_$v.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/c5/${i}_$v.json')); print('C5 $v', j['value'], 'Mrays/s', j['roofline']['per_launch_ms'], 'ms/launch')"
  i=$((i+1))
done
