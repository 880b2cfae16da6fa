"""Summarise rocprofv3 --pmc csv output (tools_pmc.sh) per kernel family and
write gpurun_out/pmc/pmc.json, which bench.py reads (copied to
profiles/rNN_pmc.json) for the roofline fractions of the same binary:

  hbm_bytes      (2 x FETCH_SIZE + WRITE_SIZE) x 1024 per launch; FETCH_SIZE /
                 WRITE_SIZE are KiB, and on gfx950 FETCH_SIZE reports half the
                 bytes of 16-B-per-lane reads (MI355X_MICROARCH.md, HBM)
  l2_read_bytes  TCP_TCC_READ_REQ x 128 B per launch (an upper bound: a request
                 moves at most one 128-B line)
  ta_busy        TA_TA_BUSY_sum / (256 TAs x GRBM_GUI_ACTIVE / 8 XCDs): the
                 fraction of the kernel's cycles the vector-memory address
                 unit of a CU is busy
  cycles         GRBM_GUI_ACTIVE / 8 per launch (kernel cycles of one XCD)

The path-kernel families also carry units_per_launch (render passes per
profiled launch; tools_pmc.sh profiles one 8-pass ctl_render_passes launch)
and rays_per_launch (the rays that launch traced, from the bench line), so a
sharded launch (1/N of the image) is scaled by its rays,
and primary_intersect its rays per launch (the profiled runs' bench lines,
primary_rays.rays_per_launch), so bench.py scales the counters to whatever
launch shape it times (a rank's 1/N image included).
Usage: tools_pmc_summary.py <dir> [passes per profiled path-kernel launch]
"""
import collections
import csv
import glob
import hashlib
import json
import os
import subprocess
import sys

root = sys.argv[1]
PASSES = int(sys.argv[2]) if len(sys.argv) > 2 else 8
FAMILIES = {
    "path_kernel": "path_kernel_persistent<false, true, 1, 0>",
    "path_kernel_full": "path_kernel_persistent<false, true, 1, 1>",
    "primary_intersect": "intersect_kernel<0, false, true, 1>",
    "prim_kernel": "prim_kernel<",
    "fold_samples": "fold_samples_kernel",
    "sampler": "sampler_",          # sampler_kernel (ctl_sampler_generate) and sampler_batch_kernel (render_passes)
}
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for f in sorted(glob.glob(os.path.join(root, "g*", "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        fam = next((k for k, key in FAMILIES.items() if key in name), None)
        if fam is None:
            continue
        c = row.get("Counter_Name")
        agg[fam][c] += float(row.get("Counter_Value", 0))
        disp[fam][c].add((f, row.get("Dispatch_Id")))

missing = [k for k in ("path_kernel", "primary_intersect", "sampler") if k not in agg]
if missing:   # a renamed template must not silently drop a roofline (it did once: bool -> int ANY)
    raise SystemExit(f"no counter rows matched families {missing}; check FAMILIES against the kernel names")
here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # the repo root
sys.path.insert(0, here)
from buildid import source_fingerprint  # noqa: E402
libp = os.path.join(here, "cudatracerlib_amd", "_lib", "libctl_trace.so")
out = {"method": __doc__.strip(), "lib_sha256": hashlib.sha256(open(libp, "rb").read()).hexdigest(),
       "src_sha256": source_fingerprint(here), "config": [3, 1.0, 1920, 1080], "shards": 1,
       "passes_per_launch": PASSES, "kernels": {}}
try:
    out["git_head"] = subprocess.check_output(["git", "rev-parse", "--short", "HEAD"], cwd=here,
                                              stderr=subprocess.DEVNULL).decode().strip()
except Exception:
    out["git_head"] = None
# rays per primary_intersect launch and rays per path-kernel launch (the timed
# region's traced rays over its path-kernel launches), from the bench lines of
# the profiled runs
prim_rays, path_rays = set(), set()
for f in glob.glob(os.path.join(root, "g*.json")):
    for line in open(f):
        if line.startswith("{"):
            j = json.loads(line)
            pr = (j.get("primary_rays") or {}).get("rays_per_launch")
            if pr:
                prim_rays.add(int(pr))
            tr, nl = (j.get("config") or {}).get("total_rays"), (j.get("roofline") or {}).get("launches_timed")
            if tr and nl:
                path_rays.add(tr / nl)
if len(prim_rays) > 1:
    raise SystemExit(f"profiled runs disagree on primary rays per launch: {sorted(prim_rays)}")
if len(path_rays) > 1:
    raise SystemExit(f"profiled runs disagree on rays per path-kernel launch: {sorted(path_rays)}")
for fam, a in sorted(agg.items()):
    n = {c: max(1, len(d)) for c, d in disp[fam].items()}
    per = {c: v / n[c] for c, v in a.items()}
    k = {"launches": max(n.values()), "counters_per_launch": {c: round(v, 1) for c, v in sorted(per.items())}}
    if fam.startswith("path_kernel"):
        k["units_per_launch"] = PASSES
        if fam == "path_kernel" and path_rays:
            k["rays_per_launch"] = next(iter(path_rays))
    if fam == "primary_intersect" and prim_rays:
        k["units_per_launch"] = prim_rays.pop()   # rays
    if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
        k["hbm_bytes"] = (2.0 * per["FETCH_SIZE"] + per["WRITE_SIZE"]) * 1024.0
    if "TCP_TCC_READ_REQ_sum" in per:
        k["l2_read_bytes"] = per["TCP_TCC_READ_REQ_sum"] * 128.0
    if "GRBM_GUI_ACTIVE" in per:
        k["cycles"] = per["GRBM_GUI_ACTIVE"] / 8.0
        if "TA_TA_BUSY_sum" in per:
            k["ta_busy"] = per["TA_TA_BUSY_sum"] / (256.0 * k["cycles"])
    if per.get("TA_FLAT_READ_WAVEFRONTS_sum") and "TA_TA_BUSY_sum" in per:
        k["ta_cycles_per_vmem_wave_inst"] = per["TA_TA_BUSY_sum"] / per["TA_FLAT_READ_WAVEFRONTS_sum"]
    if per.get("TCC_HIT_sum", 0) + per.get("TCC_MISS_sum", 0) > 0:
        k["l2_hit_rate"] = per["TCC_HIT_sum"] / (per["TCC_HIT_sum"] + per["TCC_MISS_sum"])
    if per.get("SQ_WAVE_CYCLES"):
        for c in ["SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"]:
            if c in per:
                k[c.lower() + "_frac"] = per[c] / per["SQ_WAVE_CYCLES"]
    if per.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in per:
        k["valu_lane_util"] = per["SQ_THREAD_CYCLES_VALU"] / (64.0 * per["SQ_ACTIVE_INST_VALU"])
    out["kernels"][fam] = k
json.dump(out, open(os.path.join(root, "pmc.json"), "w"), indent=1)
for fam, k in out["kernels"].items():
    print(fam, {x: (round(y, 4) if isinstance(y, float) else y) for x, y in k.items() if x != "counters_per_launch"})
    for c, v in k["counters_per_launch"].items():
        print(f"    {c:34s} {v:.6g}")
