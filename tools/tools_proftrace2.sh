#!/bin/bash
# CTL_PROFILE_TRACE build (_varprof): trace / whole-wave time split of one-pass launches, C3 and C5
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in 3 5; do
  CTL_LIB=$PWD/cudatracerlib_amd/_varprof/libctl_trace.so timeout -k 10 400 python bench.py --config $cfg --steps 4 --warmup 2 --no-cpu-baseline --wpt-passes 0 --dopass-leg 0 --one-pass-leg 3 --closest-shadow-passes 0 --prim-passes 0 --c5-passes 0 > gpurun_out/proftrace_c$cfg.json 2> gpurun_out/proftrace_c$cfg.err || { echo FAIL; tail -20 gpurun_out/proftrace_c$cfg.err; exit 1; }
  echo "config $cfg"; grep "\[profile\]" gpurun_out/proftrace_c$cfg.err | tail -2
done
