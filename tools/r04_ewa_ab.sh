#!/bin/bash
# EWA reciprocal variant: C5 parity (textured quad with every filter, C5 renders, full-size C5 pass,
# hand-flattened C5 materials, textured environment) through the variant library, then C5 benches.
set -o pipefail
mkdir -p gpurun_out/ab4
export TMPDIR=/tmp
CTL_LIB=$PWD/cudatracerlib_amd/_var${VAR:-ewa}/libctl_trace.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_c5_flatten.py tests/test_env_light.py -m gpu -k "c5 or textured" -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/ab4/ewa_tests.log 2>&1 || { echo "EWA TESTS FAILED"; tail -40 gpurun_out/ab4/ewa_tests.log; exit 1; }
tail -2 gpurun_out/ab4/ewa_tests.log
NOTEST=1 bash tools/r04_ab.sh
