#!/bin/bash
# Round measurement: rocprofv3 kernel trace + stats, PMC traffic (separate
# passes), then the default bench (with CPU baseline) reading that traffic.
set -o pipefail
export TMPDIR=/tmp
./tools_profile.sh > gpurun_out/profile.log 2>&1 || { echo "PROFILE FAILED"; tail -20 gpurun_out/profile.log; exit 1; }
./tools_pmc.sh > gpurun_out/pmc.log 2>&1 || { echo "PMC FAILED"; tail -20 gpurun_out/pmc.log; exit 1; }
cp gpurun_out/pmc/traffic.json profiles/traffic.json
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
grep -E "path_kernel_persistent<false|intersect_kernel<false, false" gpurun_out/prof/kt/run_kernel_stats.csv | cut -c1-60,150-260
