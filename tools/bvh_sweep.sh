#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/bvh_sweep
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --wpt-passes 0 --closest-shadow-passes 0 --prim-passes 0 --binary-passes 0 --one-pass-leg 0 --dopass-leg 0 --c5-passes 0 --anim-iters 0 --ceiling 0"
IFS=';' read -ra VS <<< "$VARIANTS"
for kv in "${VS[@]}"; do
  tag=${kv%%=*}; fl=${kv#*=}
  timeout -k 10 300 python3 bench.py $ARGS $fl > gpurun_out/bvh_sweep/${tag}.json 2> gpurun_out/bvh_sweep/${tag}.err || { echo "bench $tag FAILED"; tail -5 gpurun_out/bvh_sweep/${tag}.err; exit 1; }
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=b['config']; print('C3', sys.argv[2], b['value'], b['ms_per_step'], c.get('bvh_inner_nodes'), c.get('bvh_refs'))" gpurun_out/bvh_sweep/${tag}.json "$tag"
done
