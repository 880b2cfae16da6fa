#!/bin/bash
# Round 6, rebuild v5 (records-only climb, slot and 4-wide passes): the animation
# GPU tests, the animation timing (4-wide and binary scenes), a kernel trace.
# Each step under its own limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out/anim2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/anim2
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_anim.py tests/test_gpu_instances.py tests/test_gpu_scene_update.py > $O/tests.log 2>&1 || { echo "ANIM TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head -20; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 tools/tools_anim_bench.py --iters 40 > $O/bench.json 2> $O/bench.err || { echo "ANIM BENCH FAILED"; tail -5 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 200 python3 tools/tools_anim_bench.py --iters 40 --binary > $O/bench_bin.json 2> $O/bench_bin.err || { echo "ANIM BENCH (binary) FAILED"; tail -5 $O/bench_bin.err; exit 1; }
cut -c1-300 $O/bench_bin.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/tools_anim_bench.py --iters 20 > $O/prof.json 2> $O/prof.err || { echo "PROF FAILED"; tail -5 $O/prof.err; exit 1; }
for f in $(find $O/prof -name "*kernel_stats.csv"); do cut -c1-200 $f; done
[ "${ANIM_PMC:-0}" = 1 ] && bash tools/anim_pmc.sh
exit 0
