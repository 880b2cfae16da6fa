#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 900 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for v in base bv base bv; do
  if [ $v = base ]; then L=cudatracerlib_amd/_lib/libctl_trace.so; else L=cudatracerlib_amd/_var$v/libctl_trace.so; fi
  CTL_LIB=$PWD/$L timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --wpt-passes 3 --dopass-leg 0 --one-pass-leg 0 --closest-shadow-passes 0 --prim-passes 8 --c5-passes 16 > gpurun_out/kab_$v.json 2> gpurun_out/kab_$v.err || { echo "BENCH $v FAILED"; tail -20 gpurun_out/kab_$v.err; exit 1; }
  python3 -c "
import json; j=json.load(open('gpurun_out/kab_$v.json'))
print('$v C3', j['value'], 'primary', j['primary_rays']['mrays_s'], 'wpt', j['wavefront_tracer']['mrays_s'], 'c1', j['prim_tracer_c1']['mrays_s'], 'C5', j['path_tracer_c5']['mrays_s'])"
done
