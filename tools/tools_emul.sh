#!/bin/bash
# rank 0's share of an N-rank job, emulated on one GPU (bench.py --emulate-ranks N), driver shape
set -o pipefail
mkdir -p gpurun_out/emul
export TMPDIR=/tmp
for n in ${NS:-2 4 8}; do
  timeout -k 10 400 python bench.py --emulate-ranks $n --steps 20 --warmup 5 --no-cpu-baseline --wpt-passes 0 --dopass-leg 0 --one-pass-leg 0 --closest-shadow-passes 0 --prim-passes 0 --c5-passes 0 > gpurun_out/emul/rank0_of_$n.json 2> gpurun_out/emul/rank0_of_$n.err || { echo "N=$n FAILED"; tail -20 gpurun_out/emul/rank0_of_$n.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/emul/rank0_of_$n.json')); print('N=$n', j['value'], 'Mrays/s', j['ms_per_step'], 'ms/step', j['config'].get('emulated_ranks'))"
done
