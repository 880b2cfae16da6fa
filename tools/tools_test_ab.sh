#!/bin/bash
# GPU parity suite, then bench A/B runs of the given variants (tools_ab.sh)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 900 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/tools_ab.sh "$@"
