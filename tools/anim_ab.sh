set -o pipefail
mkdir -p gpurun_out/anim_ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_anim.py tests/test_gpu_scene_update.py > gpurun_out/anim_ab/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/anim_ab/tests.log; exit 1; }
tail -3 gpurun_out/anim_ab/tests.log
for i in 1 2; do for kv in base=_ab/base.so new=cudatracerlib_amd/_lib/libctl_trace.so; do
  tag=${kv%%=*}; lib=${kv#*=}
  CTL_LIB=$lib timeout -k 10 200 python3 tools/tools_anim_bench.py --iters 40 > gpurun_out/anim_ab/${tag}_$i.json 2> gpurun_out/anim_ab/${tag}_$i.err || { echo "anim $tag FAILED"; tail -5 gpurun_out/anim_ab/${tag}_$i.err; exit 1; }
  echo "$tag $i $(cat gpurun_out/anim_ab/${tag}_$i.json | cut -c1-220)"
done; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/anim_ab/prof -o run -- python3 tools/tools_anim_bench.py --iters 20 > gpurun_out/anim_ab/prof.json 2> gpurun_out/anim_ab/prof.err || { echo PROF FAILED; exit 1; }
