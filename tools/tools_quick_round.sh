#!/bin/bash
# parity + full-size suites, then the driver-shaped bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 900 --timeout-method thread > gpurun_out/quick_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/quick_tests.log; exit 1; }
tail -2 gpurun_out/quick_tests.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "
import json; j=json.load(open('gpurun_out/bench.json'))
print('C3', j['value'], j['roofline']['steps_per_launch'], 'C5', (j.get('path_tracer_c5') or {}).get('mrays_s'), 'onepass', (j.get('one_pass_launches') or {}).get('mrays_s'), 'dopass', (j.get('reference_dopass') or {}).get('mrays_s'), 'wpt', (j.get('wavefront_tracer') or {}).get('mrays_s'))"
