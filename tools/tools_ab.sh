#!/bin/bash
# A/B of bench variants (short runs, no CPU baseline): tools_ab.sh "<args A>" "<args B>" ...
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
i=0
for v in "$@"; do
  timeout -k 10 300 python bench.py --steps 32 --warmup 8 --no-cpu-baseline --wpt-passes 0 --dopass-leg 0 --one-pass-leg 0 --closest-shadow-passes 0 --prim-passes 0 --c5-passes 0 $v > gpurun_out/ab/$i.json 2> gpurun_out/ab/$i.err || { echo "FAILED: $v"; tail -5 gpurun_out/ab/$i.err; exit 1; }
  python -c "import json,sys; j=json.load(open('gpurun_out/ab/$i.json')); r=j['roofline']; v=r['visits_per_launch']; print('$v', '->', j['value'], 'Mrays/s', r['per_launch_ms'], 'ms', 'frac', r['frac'], 'nodes/ray %.1f tris/ray %.2f refs %d' % (v['inner_nodes']/v['rays'], v['tri_tests']/v['rays'], j['config']['bvh_refs']))"
  i=$((i+1))
done
