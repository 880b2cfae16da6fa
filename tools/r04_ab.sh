#!/bin/bash
# Round-4 A/B on one box: W8 parity tests, then benches of the variants at the
# driver's shape (C3 headline + primary rays + C5 leg).
set -o pipefail
mkdir -p gpurun_out/ab4
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_reference_order.py -m gpu -k "w8" -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/ab4/w8_tests.log 2>&1 || { echo "W8 TESTS FAILED"; tail -40 gpurun_out/ab4/w8_tests.log; exit 1; }
tail -2 gpurun_out/ab4/w8_tests.log
fi
LEGS="--steps 20 --warmup 5 --no-cpu-baseline --wpt-passes 0 --dopass-leg 0 --one-pass-leg 0 --closest-shadow-passes 0 --prim-passes 0 --c5-passes 16"
i=0
for spec in ${RUNS:-"base:wide" "base:w8" "r3:wide" "nolazy:wide" "lazygm:wide" "base:w8" "base:wide"}; do
  v=${spec%%:*}; b=${spec##*:}
  case $v in
    base) L=cudatracerlib_amd/_lib/libctl_trace.so; D=. ; X="--binary-passes 0";;
    r3) L=$PWD/_r3/cudatracerlib_amd/_lib/libctl_trace.so; D=_r3; X="";;
    *) L=cudatracerlib_amd/_var$v/libctl_trace.so; D=. ; X="--binary-passes 0";;
  esac
  ( cd $D && CTL_LIB=$PWD/${L#$PWD/} timeout -k 10 400 python bench.py $LEGS --bvh $b $X ) > gpurun_out/ab4/${i}_${v}_$b.json 2> gpurun_out/ab4/${i}_${v}_$b.err || { echo "BENCH $v $b FAILED"; tail -20 gpurun_out/ab4/${i}_${v}_$b.err; exit 1; }
  python3 -c "
import json; j=json.loads(open('gpurun_out/ab4/${i}_${v}_$b.json').read().strip().splitlines()[-1]); c5=j.get('path_tracer_c5') or {}
print('$v $b C3', j['value'], 'camera', j['primary_rays']['mrays_s'], 'C5', c5.get('mrays_s'), 'wsum', j.get('image_weight_sum'))"
  i=$((i+1))
done
