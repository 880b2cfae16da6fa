#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 900 --timeout-method thread > gpurun_out/slack_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/slack_tests.log; exit 1; }
tail -2 gpurun_out/slack_tests.log
VARS="base noslack base noslack" bash tools/tools_var.sh || exit 1
CTL_LIB=$PWD/cudatracerlib_amd/_lib/libctl_trace.so NP=16 timeout -k 10 400 python probes/shard_diag.py > gpurun_out/diag_base.log 2>&1 || { echo FAIL; tail gpurun_out/diag_base.log; exit 1; }
grep -v amdgpu.ids gpurun_out/diag_base.log | tail -8
