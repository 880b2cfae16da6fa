#!/bin/bash
# Round 6: the rebuild (rotation) path first, then the whole GPU suite, then the
# animation timing; each step under its own limit, the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_anim.py tests/test_gpu_instances.py tests/test_gpu_scene_update.py > gpurun_out/r06_anim_tests.log 2>&1 || { echo "ANIM TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/r06_anim_tests.log | head -20; tail -40 gpurun_out/r06_anim_tests.log; exit 1; }
tail -2 gpurun_out/r06_anim_tests.log
timeout -k 10 200 python3 tools/tools_anim_bench.py --iters 40 > gpurun_out/r06_anim_bench.json 2> gpurun_out/r06_anim_bench.err || { echo "ANIM BENCH FAILED"; tail -5 gpurun_out/r06_anim_bench.err; exit 1; }
cut -c1-400 gpurun_out/r06_anim_bench.json
[ "${ANIM_ONLY:-0}" = 1 ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 1200 --timeout-method thread > gpurun_out/r06_gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/r06_gpu_tests.log | head -20; tail -30 gpurun_out/r06_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r06_gpu_tests.log
