#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CTL_LIB=$PWD/cudatracerlib_amd/_varka/libctl_trace.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ka_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/ka_tests.log; exit 1; }
tail -1 gpurun_out/ka_tests.log
VARS="base ka base ka" bash tools/tools_var.sh && VARS="base ka" bash tools/tools_c5ab.sh
