#!/bin/bash
# parity tests, then the C3 bench under each requested pass schedule
# usage: tools_sched.sh [schedule ...]   (default: persistent)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
SCHEDS="${*:-persistent}"
for sch in $SCHEDS; do
  timeout -k 10 300 python bench.py --steps 16 --no-cpu-baseline --schedule $sch > gpurun_out/sched_$sch.json 2> gpurun_out/sched_$sch.err || { echo "BENCH $sch FAILED"; tail -20 gpurun_out/sched_$sch.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('gpurun_out/sched_$sch.json')); print('$sch', j['value'], 'Mrays/s', j['ms_per_step'], 'ms/step', 'kernel', j['roofline']['per_launch_ms'], 'ms')"
done
