#!/bin/bash
# Every rank's share of an N-GPU job (default 8), emulated on one GPU at the
# driver's bench shape: profiles/rNN_emulated_rank{r}_of_N.json.
set -o pipefail
mkdir -p gpurun_out/emul
export TMPDIR=/tmp
N=${N:-8}
for r in $(seq 0 $((N - 1))); do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --emulate-ranks $N --emulate-rank $r --no-cpu-baseline \
      --wpt-passes 0 --prim-passes 0 --c5-passes 0 --closest-shadow-passes 0 $EXTRA > gpurun_out/emul/rank${r}_of_$N.json 2> gpurun_out/emul/rank${r}_of_$N.err || { echo "RANK $r FAILED"; tail -20 gpurun_out/emul/rank${r}_of_$N.err; exit 1; }
  python3 -c "import json; j=json.loads(open('gpurun_out/emul/rank${r}_of_$N.json').read().strip().splitlines()[-1]); print('rank $r of $N', j['value'], j['ms_per_step'])"
done
