#!/bin/bash
# Round-4 A/B 2: parity of the unified-fetch (if-if) variant against the
# oracle's no-speculation order, then the benches of RUNS (tools/r04_ab.sh).
set -o pipefail
mkdir -p gpurun_out/ab4
export TMPDIR=/tmp
CTL_LIB=$PWD/cudatracerlib_amd/_varifif/libctl_trace.so ORACLE_WIDE_NOSPEC=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "wide and not wideq" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab4/ifif_tests.log 2>&1 || { echo "IFIF TESTS FAILED"; tail -40 gpurun_out/ab4/ifif_tests.log; exit 1; }
tail -2 gpurun_out/ab4/ifif_tests.log
NOTEST=1 bash tools/r04_ab.sh
