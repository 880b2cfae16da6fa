#!/bin/bash
# GPU parity suite (one process, per-test timeout), then smoke
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 900 --timeout-method thread "$@" > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
