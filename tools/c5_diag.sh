#!/bin/bash
# C5 cost split by material class (probes/c5_material_split.py) and the
# instruction / cache counters of the lean and FULL path kernels on the same
# geometry ("neither": constant diffuse, lean kernel; "neither, full": the same
# hits through the FULL kernel; C5).  One rocprofv3 --pmc pass per group.
set -o pipefail
mkdir -p gpurun_out/c5diag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/c5diag/avail.txt 2>&1 || true
grep -o "SQC_[A-Z_0-9]*\|SQ_INSTS_[A-Z_0-9]*\|SQ_IFETCH[A-Z_0-9]*" gpurun_out/c5diag/avail.txt | sort -u > gpurun_out/c5diag/counters.txt
timeout -k 10 600 python3 probes/c5_material_split.py > gpurun_out/c5diag/split.txt 2> gpurun_out/c5diag/split.err || { echo SPLIT FAILED; tail -5 gpurun_out/c5diag/split.err; exit 1; }
cat gpurun_out/c5diag/split.txt
export C5SPLIT_ONLY="neither;neither, full;C5"
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS"
G2="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES"
G3=$(grep -x "SQC_ICACHE_HITS\|SQC_ICACHE_MISSES\|SQC_ICACHE_MISSES_DUPLICATE\|SQC_ICACHE_REQ" gpurun_out/c5diag/counters.txt | head -4 | tr '\n' ' ')
i=0
for grp in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  [ -z "$grp" ] && continue
  echo "pmc group $i: $grp"
  timeout -k 10 400 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/c5diag/g$i -o run -- python3 probes/c5_material_split.py > gpurun_out/c5diag/g$i.txt 2> gpurun_out/c5diag/g$i.err || { echo "PMC $i FAILED"; tail -5 gpurun_out/c5diag/g$i.err; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(set))
for f in glob.glob("gpurun_out/c5diag/g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "path_kernel_persistent" not in n:
            continue
        k = n.split("(")[0].split("path_kernel_persistent")[1]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]].add((f, r["Dispatch_Id"]))
for k, a in agg.items():
    print(k, {c: round(v / max(1, len(cnt[k][c])) / 1e6, 2) for c, v in sorted(a.items())}, "(M per launch)")
PY
