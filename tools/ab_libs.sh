#!/bin/bash
# A/B of several library builds: the headline C3 leg (bench.py, other legs off)
# twice per library, interleaved, then the C5 material split once per library.
#   LIBS="base=_ab/base.so v1=_ab/v1.so new=cudatracerlib_amd/_lib/libctl_trace.so" bash tools/ab_libs.sh
set -o pipefail
LIBS=${LIBS:-"base=_ab/base.so new=cudatracerlib_amd/_lib/libctl_trace.so"}
mkdir -p gpurun_out/ab_libs
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --wpt-passes 0 --closest-shadow-passes 0 --prim-passes 0 --binary-passes 0 --one-pass-leg 0 --dopass-leg 0 --c5-passes 0 --anim-iters 0"
for i in 1 2; do
  for kv in $LIBS; do
    tag=${kv%%=*}; lib=${kv#*=}
    CTL_LIB=$lib timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/ab_libs/c3_${tag}_$i.json 2> gpurun_out/ab_libs/c3_${tag}_$i.err \
      || { echo "bench $tag $i FAILED"; tail -5 gpurun_out/ab_libs/c3_${tag}_$i.err; exit 1; }
    python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C3', sys.argv[2], b['value'], b['ms_per_step'])" gpurun_out/ab_libs/c3_${tag}_$i.json "$tag $i"
  done
done
export C5SPLIT_ONLY=${C5SPLIT_ONLY:-"C5;neither, full;rough only;textures only"}
for kv in $LIBS; do
  tag=${kv%%=*}; lib=${kv#*=}
  echo "== C5 split $tag"
  CTL_LIB=$lib timeout -k 10 300 python3 probes/c5_material_split.py > gpurun_out/ab_libs/c5_${tag}.txt 2> gpurun_out/ab_libs/c5_${tag}.err \
    || { echo "split $tag FAILED"; tail -5 gpurun_out/ab_libs/c5_${tag}.err; exit 1; }
  cat gpurun_out/ab_libs/c5_${tag}.txt
done
