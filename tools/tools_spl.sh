#!/bin/bash
# driver-shaped bench (--steps 20 --warmup 5) at several --steps-per-launch
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for spl in 8 20 10 8 20; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --steps-per-launch $spl --no-cpu-baseline --wpt-passes 0 --dopass-leg 0 --one-pass-leg 0 --closest-shadow-passes 0 --prim-passes 0 --c5-passes 0 > gpurun_out/spl_$spl.json 2> gpurun_out/spl_$spl.err || { echo FAIL; tail gpurun_out/spl_$spl.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/spl_$spl.json')); print('spl $spl', j['value'], j['roofline']['steps_per_launch'], j['ms_per_step'])"
done
