#!/bin/bash
# bench variant libraries on one box: VARS="base name1 name2 base ..." -> cudatracerlib_amd/_var<name>/libctl_trace.so
set -o pipefail
mkdir -p gpurun_out
i=0
for v in ${VARS:-base}; do
  if [ $v = base ]; then L=cudatracerlib_amd/_lib/libctl_trace.so; else L=cudatracerlib_amd/_var$v/libctl_trace.so; fi
  CTL_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps 32 --warmup 8 --no-cpu-baseline --wpt-passes 0 --dopass-leg 0 --one-pass-leg 0 --closest-shadow-passes 0 --prim-passes 0 --c5-passes 0 $BENCH_ARGS > gpurun_out/var_${i}_$v.json 2> gpurun_out/var_${i}_$v.err || { echo "BENCH $v FAILED"; tail -20 gpurun_out/var_${i}_$v.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/var_${i}_$v.json')); print('$v', j['value'], j['roofline']['per_launch_ms'], 'primary', j['primary_rays']['mrays_s'])"
  i=$((i+1))
done
