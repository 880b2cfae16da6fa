#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no counters: see tools_pmc.sh)
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt -o run -- python3 bench.py --steps 16 --warmup 8 --ceiling 0 --no-cpu-baseline --closest-shadow-passes 0 --one-pass-leg 0 --dopass-leg 0 --c5-passes 0 --binary-passes 0 --anim-iters 0 "$@" > gpurun_out/prof/bench_prof.json 2> gpurun_out/prof/bench_prof.err || { echo PROF FAILED; tail -20 gpurun_out/prof/bench_prof.err; exit 1; }
cat gpurun_out/prof/bench_prof.json
find gpurun_out/prof -name "*stats*" | head
for f in $(find gpurun_out/prof -name "*kernel_stats.csv"); do cat $f; done
