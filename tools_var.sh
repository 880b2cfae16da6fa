#!/bin/bash
# bench variant libraries: VARS="base name1 name2" -> cudatracerlib_amd/_var<name>/libctl_trace.so
set -o pipefail
mkdir -p gpurun_out
for v in ${VARS:-base}; do
  if [ $v = base ]; then L=cudatracerlib_amd/_lib/libctl_trace.so; else L=cudatracerlib_amd/_var$v/libctl_trace.so; fi
  CTL_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps 16 --no-cpu-baseline $BENCH_ARGS > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || { echo "BENCH $v FAILED"; tail -20 gpurun_out/var_$v.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/var_$v.json')); print('$v', j['value'], j['roofline']['per_launch_ms'], 'primary', j['primary_rays']['mrays_s'], 'wpt', (j.get('wavefront_tracer') or {}).get('mrays_s'))"
done
