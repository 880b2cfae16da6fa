#!/bin/bash
# parity tests, then C3 bench over BVH reference-splitting settings and traversal modes
set -o pipefail
mkdir -p gpurun_out/split
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
fi
IFS='|' read -ra LIST <<< "${CFGS:-0 0 wide|4 3 wide|1 4 wide|1 6 wide|1 4 binary}"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  tag=a$1_d$2_$3
  timeout -k 10 300 python bench.py --steps 16 --no-cpu-baseline --split-alpha $1 --split-depth $2 --bvh $3 > gpurun_out/split/$tag.json 2> gpurun_out/split/$tag.err || { echo "BENCH $tag FAILED"; tail -20 gpurun_out/split/$tag.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/split/$tag.json')); r=j['roofline']; v=r['visits_per_launch']; print('$tag', j['value'], 'Mrays/s', r['per_launch_ms'], 'ms', 'nodes/ray %.1f tris/ray %.1f' % (v['inner_nodes']/v['rays'], v['tri_tests']/v['rays']), 'primary', j['primary_rays']['mrays_s'], 'build', j['scene_build_s'], 'refs', j['config']['bvh_refs'])"
done
