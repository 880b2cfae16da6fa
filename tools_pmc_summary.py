"""Summarise rocprofv3 --pmc csv output per kernel family (sum over dispatches)
and write profiles/traffic.json for bench.py's roofline "traffic" field.

HBM bytes per launch of the timed pass kernel = (2 x FETCH_SIZE + WRITE_SIZE)
x 1024 / launches: FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of 16-B-per-lane reads (MI355X_MICROARCH.md, HBM
section), hence the factor 2 on the read side."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
FAMILIES = ["path_kernel_persistent<false", "path_kernel_persistent<true", "path_kernel<false", "path_kernel<true",
            "wf_trace_kernel<0", "wf_trace_kernel<1", "wf_trace_kernel<2", "wf_shade_kernel", "wf_resolve_kernel",
            "wf_gen_kernel", "sampler_kernel"]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for f in sorted(glob.glob(os.path.join(root, "g*", "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        fam = "other"
        for key in FAMILIES:
            if key in name:
                fam = key
                break
        cname = row.get("Counter_Name")
        agg[fam][cname] += float(row.get("Counter_Value", 0))
        disp[fam][cname].add((f, row.get("Dispatch_Id")))
for fam in sorted(agg):
    print(fam)
    for k, v in sorted(agg[fam].items()):
        print(f"   {k:28s} {v:20.6g}   ({len(disp[fam][k])} dispatches)")
    a = agg[fam]
    if a.get("TCC_HIT_sum", 0) + a.get("TCC_MISS_sum", 0) > 0:
        print(f"   L2 hit rate {a['TCC_HIT_sum'] / (a['TCC_HIT_sum'] + a['TCC_MISS_sum']):.4f}")
    if a.get("SQ_WAVE_CYCLES"):
        for k in ["SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"]:
            if k in a:
                print(f"   {k} / SQ_WAVE_CYCLES = {a[k] / a['SQ_WAVE_CYCLES']:.3f}")
    if a.get("SQ_ACTIVE_INST_VALU") and a.get("SQ_THREAD_CYCLES_VALU"):
        print(f"   VALU lane utilisation {a['SQ_THREAD_CYCLES_VALU'] / (64 * a['SQ_ACTIVE_INST_VALU']):.3f}")

main = "path_kernel_persistent<false"
if main in agg and "FETCH_SIZE" in agg[main] and "WRITE_SIZE" in agg[main]:
    a = agg[main]
    launches = len(disp[main]["FETCH_SIZE"])
    hbm = (2.0 * a["FETCH_SIZE"] + a["WRITE_SIZE"]) * 1024.0 / launches
    out = {"kernel": main + ",...>", "config": [3, 1.0, 1920, 1080], "launches": launches,
           "fetch_size_kib": a["FETCH_SIZE"] / launches, "write_size_kib": a["WRITE_SIZE"] / launches,
           "hbm_bytes_per_launch": hbm,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of "
                     "`bench.py --steps 1 --warmup 0`; (2*FETCH_SIZE + WRITE_SIZE) KiB per launch "
                     "(gfx950 FETCH_SIZE half-count correction)"}
    os.makedirs("profiles", exist_ok=True)
    json.dump(out, open("gpurun_out/pmc/traffic.json", "w"), indent=1)
    print("traffic:", json.dumps(out))
