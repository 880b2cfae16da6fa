"""Summarise rocprofv3 --pmc csv output per kernel family (sum over dispatches)."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(lambda: collections.defaultdict(int))
for f in sorted(glob.glob(os.path.join(root, "g*", "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        fam = "other"
        for key in ["wf_trace_kernel<0", "wf_trace_kernel<1", "wf_trace_kernel<2", "wf_shade_kernel",
                    "wf_resolve_kernel", "wf_gen_kernel", "sampler_kernel", "path_kernel<false", "path_kernel<true"]:
            if key in name:
                fam = key
        cname = row.get("Counter_Name")
        agg[fam][cname] += float(row.get("Counter_Value", 0))
        calls[fam][cname] += 1
for fam in sorted(agg):
    print(fam)
    for k, v in sorted(agg[fam].items()):
        print(f"   {k:28s} {v:20.6g}   ({calls[fam][k]} rows)")
