#!/bin/bash
# animation GPU tests, then the timing-only rebuild variants (tools/anim_diag.sh)
set -o pipefail
mkdir -p gpurun_out/anim2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/anim2
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_anim.py tests/test_gpu_instances.py tests/test_gpu_scene_update.py > $O/tests.log 2>&1 || { echo "ANIM TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head -20; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python3 tools/tools_anim_bench.py --iters 40 > $O/bench.json 2> $O/bench.err || { echo "ANIM BENCH FAILED"; tail -5 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json
bash tools/anim_diag.sh
