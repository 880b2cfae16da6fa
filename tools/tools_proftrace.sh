#!/bin/bash
# CTL_PROFILE_TRACE build: wall-clock split (trace / whole wave time) and loop occupancy of one-pass launches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CTL_LIB=$PWD/cudatracerlib_amd/_varprof/libctl_trace.so timeout -k 10 400 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --wpt-passes 0 --dopass-leg 0 --one-pass-leg 3 --closest-shadow-passes 0 --prim-passes 0 --c5-passes 0 "$@" > gpurun_out/proftrace.json 2> gpurun_out/proftrace.err || { echo FAIL; tail -20 gpurun_out/proftrace.err; exit 1; }
grep "\[profile\]" gpurun_out/proftrace.err | tail -4
