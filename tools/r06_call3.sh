#!/bin/bash
# Round 6 call 3: the coherent-access rebuild (animation tests + timing), render-ahead
# tests, the C5 reference-order record with 1 M refraction rays, then the default bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_anim.py tests/test_gpu_instances.py tests/test_gpu_render_ahead.py > gpurun_out/r06_call3_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/r06_call3_tests.log | head -20; tail -30 gpurun_out/r06_call3_tests.log; exit 1; }
tail -2 gpurun_out/r06_call3_tests.log
timeout -k 10 200 python3 tools/tools_anim_bench.py --iters 40 > gpurun_out/r06_anim_bench.json 2> gpurun_out/r06_anim_bench.err || { echo "ANIM BENCH FAILED"; tail -5 gpurun_out/r06_anim_bench.err; exit 1; }
cut -c1-300 gpurun_out/r06_anim_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/anim_prof -o run -- python3 tools/tools_anim_bench.py --iters 20 > gpurun_out/anim_prof.json 2> gpurun_out/anim_prof.err || { echo "ANIM PROF FAILED"; tail -5 gpurun_out/anim_prof.err; exit 1; }
find gpurun_out/anim_prof -name "*kernel_stats.csv" -exec head -12 {} \;
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 400 --timeout-method thread "tests/test_reference_order.py::test_full_size_reference_order_distance[c5]" > gpurun_out/r06_c5_order.log 2>&1 || { echo "C5 ORDER FAILED"; tail -30 gpurun_out/r06_c5_order.log; exit 1; }
tail -2 gpurun_out/r06_c5_order.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_bench.json 2> gpurun_out/r06_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/r06_bench.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/r06_bench.json || true
