#!/bin/bash
# A/B of variant libraries (cudatracerlib_amd/_var<name>, "base" = _lib) at the driver's
# bench shape, C3 headline + C5 leg: VARS="base p1 base p1" bash tools/tools_vab.sh [extra bench args]
set -o pipefail
mkdir -p gpurun_out/vab
export TMPDIR=/tmp
i=0
for v in ${VARS:-base}; do
  if [ $v = base ]; then L=cudatracerlib_amd/_lib/libctl_trace.so; else L=cudatracerlib_amd/_var$v/libctl_trace.so; fi
  CTL_LIB=$PWD/$L timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --wpt-passes 0 --dopass-leg 0 --one-pass-leg 0 --closest-shadow-passes 0 --prim-passes 0 ${C5:---c5-passes 16} "$@" > gpurun_out/vab/${i}_$v.json 2> gpurun_out/vab/${i}_$v.err || { echo "BENCH $v FAILED"; tail -20 gpurun_out/vab/${i}_$v.err; exit 1; }
  python3 -c "
import json; j=json.load(open('gpurun_out/vab/${i}_$v.json')); c5=j.get('path_tracer_c5') or {}
print('$v C3', j['value'], 'primary', j['primary_rays']['mrays_s'], 'wpt', (j.get('wavefront_tracer') or {}).get('mrays_s'), 'C5', c5.get('mrays_s'), 'wsum', j.get('image_weight_sum'))"
  i=$((i+1))
done
