#!/bin/bash
# WavefrontPathTracer / batch-traversal variants: VARS="base name ..." (cudatracerlib_amd/_var<name>)
set -o pipefail
mkdir -p gpurun_out
for v in ${VARS:-base}; do
  if [ $v = base ]; then L=cudatracerlib_amd/_lib/libctl_trace.so; else L=cudatracerlib_amd/_var$v/libctl_trace.so; fi
  CTL_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --wpt-passes 3 $BENCH_ARGS > gpurun_out/wvar_$v.json 2> gpurun_out/wvar_$v.err || { echo "BENCH $v FAILED"; tail -20 gpurun_out/wvar_$v.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/wvar_$v.json')); print('$v', 'path', j['value'], 'wpt', j['wavefront_tracer']['mrays_s'], j['wavefront_tracer']['ms_per_pass'], 'primary', j['primary_rays']['mrays_s'])"
done
