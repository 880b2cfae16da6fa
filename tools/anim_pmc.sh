#!/bin/bash
# HBM bytes of the animation kernels (tools_anim_bench.py, 2 M-triangle skinned
# grid): FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc runs, then a
# per-kernel summary (bytes per launch, with the gfx950 FETCH_SIZE x 2
# correction for 16-B-per-lane reads, as tools_pmc_summary.py applies it).
set -o pipefail
mkdir -p gpurun_out/anim_pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/anim_pmc/g$i -o run -- python3 tools/tools_anim_bench.py --iters 10 > gpurun_out/anim_pmc/g$i.json 2> gpurun_out/anim_pmc/g$i.err || { echo "PMC group $i failed"; tail -5 gpurun_out/anim_pmc/g$i.err; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/anim_pmc/g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("ctl::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, c in sorted(agg.items()):
    if "rocclr" in n:
        continue
    avg = {k: sum(v) / len(v) for k, v in c.items()}
    fetch, write = avg.get("FETCH_SIZE", 0.0), avg.get("WRITE_SIZE", 0.0)
    hit, miss = avg.get("TCC_HIT_sum", 0.0), avg.get("TCC_MISS_sum", 0.0)
    print(f"{n:40s} hbm_read {2 * fetch * 1024 / 1e6:8.2f} MB  hbm_write {write * 1024 / 1e6:8.2f} MB  "
          f"l2_hit {hit / max(1.0, hit + miss):.3f}")
PY
