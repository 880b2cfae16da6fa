#!/bin/bash
# rocprofv3 PC sampling (host trap) of a short bench run
set -o pipefail
mkdir -p gpurun_out/pcs
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pcs/avail.txt 2>&1 || true
grep -i -A3 "pc_sampling\|PC Sampling" gpurun_out/pcs/avail.txt | head -20
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 100 --output-format csv -d gpurun_out/pcs/run -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pcs/bench.json 2> gpurun_out/pcs/bench.err
echo "rc=$?"
ls -la gpurun_out/pcs/run | head
tail -5 gpurun_out/pcs/bench.err
