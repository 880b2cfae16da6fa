#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/park_tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/park_tests.log; exit 1; }
tail -2 gpurun_out/park_tests.log
VARS="base nopark base nopark" bash tools/tools_var.sh && VARS="base crool full4 base" bash tools/tools_c5ab.sh
