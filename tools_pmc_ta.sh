#!/bin/bash
# Vector-memory pipeline counters of the path kernel (TA / TCP), one rocprofv3 pass per group.
set -o pipefail
mkdir -p gpurun_out/pmcta
export TMPDIR=/tmp
i=0
for grp in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TA_TCP_STATE_READ_sum" "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcta/g$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --wpt-passes 0 > gpurun_out/pmcta/g$i.json 2> gpurun_out/pmcta/g$i.err || { echo "PMC group $i failed"; tail -5 gpurun_out/pmcta/g$i.err; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float)
for f in glob.glob("gpurun_out/pmcta/g*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "path_kernel_persistent<false" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(tot.items()):
    print(f"{k:40s} {v:.4g}")
PY
