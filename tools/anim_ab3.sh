#!/bin/bash
# Animation A/B over several builds: the animation GPU tests on the in-tree build,
# then tools_anim_bench.py interleaved twice over LIBS="tag=path ...", then a
# kernel trace of the in-tree build.
set -o pipefail
mkdir -p gpurun_out/anim_ab3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/anim_ab3
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_anim.py tests/test_gpu_instances.py tests/test_gpu_scene_update.py > $O/tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do for kv in $LIBS; do
  tag=${kv%%=*}; lib=${kv#*=}
  CTL_LIB=$lib timeout -k 10 200 python3 tools/tools_anim_bench.py --iters 40 > $O/${tag}_$i.json 2> $O/${tag}_$i.err || { echo "anim $tag FAILED"; tail -5 $O/${tag}_$i.err; exit 1; }
  echo "$tag $i $(python3 -c "import json,sys; j=json.load(open(sys.argv[1])); print(j['ms_per_animate_median'], j['ms_min'])" $O/${tag}_$i.json)"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/tools_anim_bench.py --iters 20 > $O/prof.json 2> $O/prof.err || { echo PROF FAILED; exit 1; }
for f in $(find $O/prof -name "*kernel_stats.csv"); do cut -d, -f1,4 $f | sed 's/(.*)//' | head -12; done
