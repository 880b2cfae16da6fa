#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/anim_scale
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in 128 256 512 1024 1448; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/anim_scale/p$n -o run -- python3 tools/tools_anim_bench.py --iters 20 --n $n > gpurun_out/anim_scale/b$n.json 2> gpurun_out/anim_scale/b$n.err || { echo "FAILED $n"; tail -5 gpurun_out/anim_scale/b$n.err; exit 1; }
  echo "n=$n $(cut -c1-200 gpurun_out/anim_scale/b$n.json)"
  grep -E "rebuild|slot|wide" gpurun_out/anim_scale/p$n/run_kernel_stats.csv | cut -d, -f1,4 | sed 's/(.*)//' 
done
