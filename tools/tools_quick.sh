#!/bin/bash
# parity tests (gpu) + one short bench: quick check after a kernel change
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/tools_ab.sh "$@"
