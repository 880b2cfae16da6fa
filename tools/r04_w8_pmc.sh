#!/bin/bash
# PMC counters of the 8-wide traversal (bench.py --bvh w8), the same six passes as tools/tools_pmc.sh.
set -o pipefail
bash tools/tools_pmc.sh --bvh w8 > gpurun_out/pmc_w8.log 2>&1 || { echo "W8 PMC FAILED"; tail -20 gpurun_out/pmc_w8.log; exit 1; }
grep -v "^    " gpurun_out/pmc/summary.txt
