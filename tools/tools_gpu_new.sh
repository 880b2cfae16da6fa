#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_scene_update.py tests/test_gpu_instances.py tests/test_env_light.py tests/test_gpu_mgpu.py -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/gpu_new.log 2>&1 || { echo "NEW TESTS FAILED"; tail -60 gpurun_out/gpu_new.log; exit 1; }
tail -3 gpurun_out/gpu_new.log
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 900 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
