#!/bin/bash
# Round GPU check: the whole -m gpu suite (one process), smoke, then the
# driver-shaped bench.  Every GPU step has its own time limit; the first
# failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 900 --timeout-method thread "$@" > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench.json
