#!/bin/bash
# Default bench at the driver's shape (reads the newest profiles/rNN_pmc.json), then a short A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_full.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_full.json
NOTEST=1 bash tools/r04_ab.sh
