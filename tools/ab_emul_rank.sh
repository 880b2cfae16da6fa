set -o pipefail
mkdir -p gpurun_out/ab_emul
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --wpt-passes 0 --closest-shadow-passes 0 --prim-passes 0 --binary-passes 0 --one-pass-leg 0 --dopass-leg 0 --c5-passes 0"
for i in 1 2; do for tag in base new; do
  lib=_ab/base.so; [ $tag = new ] && lib=cudatracerlib_amd/_lib/libctl_trace.so
  CTL_LIB=$lib timeout -k 10 300 python3 bench.py $ARGS --emulate-ranks 8 --emulate-rank 3 > gpurun_out/ab_emul/${tag}_$i.json 2> gpurun_out/ab_emul/${tag}_$i.err || { echo FAIL; tail -5 gpurun_out/ab_emul/${tag}_$i.err; exit 1; }
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rank3/8', sys.argv[2], b['value'], b['ms_per_step'])" gpurun_out/ab_emul/${tag}_$i.json "$tag $i"
done; done
