#!/bin/bash
# A/B of two library builds on the headline C3 leg only (bench.py with the other
# legs off), interleaved base, new, base, new.  BASE defaults to _ab/base.so.
set -o pipefail
BASE=${BASE:-_ab/base.so}
NEW=${NEW:-cudatracerlib_amd/_lib/libctl_trace.so}
mkdir -p gpurun_out/ab_c3
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --wpt-passes 0 --closest-shadow-passes 0 --prim-passes 0 --binary-passes 0 --one-pass-leg 0 --dopass-leg 0 --c5-passes 0"
for i in 1 2; do
  for tag in base new; do
    lib=$BASE; [ $tag = new ] && lib=$NEW
    CTL_LIB=$lib timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/ab_c3/${tag}_$i.json 2> gpurun_out/ab_c3/${tag}_$i.err \
      || { echo "bench $tag $i FAILED"; tail -5 gpurun_out/ab_c3/${tag}_$i.err; exit 1; }
    python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], b['value'], b['ms_per_step'])" gpurun_out/ab_c3/${tag}_$i.json "$tag $i"
  done
done
