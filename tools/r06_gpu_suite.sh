#!/bin/bash
# Round 6: the GPU suite, then the default bench line; each step under its own
# limit, the first failure ends the call.  Logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SEL=${1:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 1200 --timeout-method thread $SEL > gpurun_out/r06_gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r06_gpu_tests.log
[ $rc -eq 0 ] || { echo "GPU TESTS FAILED rc=$rc"; grep -E "FAILED|Error|error" gpurun_out/r06_gpu_tests.log | head -20; exit 1; }
[ "${NOBENCH:-0}" = 1 ] && exit 0
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_bench.json 2> gpurun_out/r06_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/r06_bench.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/r06_bench.json || true
