#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/bvh
export TMPDIR=/tmp
for b in wide binary; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bvh/$b -o run -- python3 bench.py --steps 8 --warmup 1 --no-cpu-baseline --bvh $b > gpurun_out/bvh/$b.json 2> gpurun_out/bvh/$b.err || { echo "BENCH $b FAILED"; tail -20 gpurun_out/bvh/$b.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/bvh/$b.json')); print('$b', j['value'], j['roofline']['per_launch_ms'], j['primary_rays']['mrays_s'])"
  head -6 gpurun_out/bvh/$b/run_kernel_stats.csv | cut -c1-160
done
