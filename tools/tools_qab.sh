#!/bin/bash
# parity of the quantized wide nodes, then A/B wide vs wideq (and any extra variants)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "wideq" --timeout 300 --timeout-method thread > gpurun_out/q_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/q_tests.log; exit 1; }
tail -2 gpurun_out/q_tests.log
bash tools/tools_ab.sh "$@"
