#!/bin/bash
# Round measurement: rocprofv3 kernel trace + stats, the PMC counter runs
# (tools_pmc.sh), then the default bench reading that counter summary.
# Results land in gpurun_out/ (copy the summaries into profiles/rNN_*).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/tools_profile.sh > gpurun_out/profile.log 2>&1 || { echo "PROFILE FAILED"; tail -20 gpurun_out/profile.log; exit 1; }
bash tools/tools_pmc.sh > gpurun_out/pmc.log 2>&1 || { echo "PMC FAILED"; tail -20 gpurun_out/pmc.log; exit 1; }
cp gpurun_out/pmc/pmc.json profiles/r99_pmc.json   # box-local: the bench below reads the newest profile
timeout -k 10 900 python bench.py "$@" > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
cat gpurun_out/pmc/summary.txt | grep -v "^    "
