#!/bin/bash
# Timing-only rebuild variants (CTL_REBUILD_DIAG builds in cudatracerlib_amd/_diagN):
# kernel trace of tools_anim_bench.py on the shipped library and on each variant.
set -o pipefail
mkdir -p gpurun_out/anim_diag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 0 1 2 3; do
  lib=""; [ $v != 0 ] && lib="cudatracerlib_amd/_diag$v/lib/libctl_trace.so"
  CTL_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/anim_diag/p$v -o run -- python3 tools/tools_anim_bench.py --iters 20 ${ANIM_ARGS:-} > gpurun_out/anim_diag/b$v.json 2> gpurun_out/anim_diag/b$v.err || { echo "FAILED $v"; tail -5 gpurun_out/anim_diag/b$v.err; exit 1; }
  echo "variant $v: $(grep -E "anim_rebuild" gpurun_out/anim_diag/p$v/run_kernel_stats.csv | cut -d, -f1,4 | sed 's/(.*)//')"
done
