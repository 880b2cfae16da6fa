#!/bin/bash
# Round measurement on one box, each GPU step under its own limit, the first failure
# ends the call: rocprofv3 kernel trace + stats (tools_profile.sh), the PMC counter
# passes (tools_pmc.sh -> gpurun_out/pmc/pmc.json), the default bench reading that
# profile, rank 5's share of an 8-GPU job reading it too (its primary-ray roofline
# must equal the N = 1 line's per ray), and the 2-rank rehearsal of the N-GPU path.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
# Stages (one gpurun call each fits the call limit): "profile" = kernel trace + PMC
# passes; "bench" = the bench runs, reading the newest committed profiles/rNN_pmc.json
# (copy gpurun_out/pmc/pmc.json there after the profile stage); no argument = both,
# the bench runs reading the fresh gpurun_out/pmc/pmc.json through CTL_PMC_PROFILE.
STAGE=${1:-all}
if [ "$STAGE" != bench ]; then
bash tools/tools_profile.sh > gpurun_out/profile.log 2>&1 || { echo "PROFILE FAILED"; tail -20 gpurun_out/profile.log; exit 1; }
bash tools/tools_pmc.sh > gpurun_out/pmc.log 2>&1 || { echo "PMC FAILED"; tail -20 gpurun_out/pmc.log; exit 1; }
cat gpurun_out/pmc/summary.txt
[ "$STAGE" = profile ] && exit 0
export CTL_PMC_PROFILE=gpurun_out/pmc/pmc.json   # box-local: the runs below read this profile
fi
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_full.err; exit 1; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --emulate-ranks 8 --emulate-rank 5 --no-cpu-baseline \
    --wpt-passes 0 --prim-passes 0 --c5-passes 0 --closest-shadow-passes 0 --anim-iters 0 > gpurun_out/emul_rank5_of_8.json 2> gpurun_out/emul.err || { echo "EMULATED RANK FAILED"; tail -20 gpurun_out/emul.err; exit 1; }
bash tools/rehearsal_2rank.sh > gpurun_out/rehearsal.log 2>&1 || { echo "REHEARSAL FAILED"; tail -20 gpurun_out/rehearsal.log; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_full.json
python3 - <<'PY'
import json
def last(p):
    return json.loads([l for l in open(p) if l.startswith("{")][-1])
a, b = last("gpurun_out/bench_full.json"), last("gpurun_out/emul_rank5_of_8.json")
for name, j in (("N=1", a), ("rank 5 of 8", b)):
    r = j["primary_rays"]["roofline"]
    print(name, "primary rays", j["primary_rays"]["rays_per_launch"], "frac_hbm", r.get("frac_hbm"),
          "traffic/ray", r.get("traffic_per_unit"), "matches", r.get("profile_matches_binary"))
    r = j["roofline"]
    print(name, "path kernel frac", r.get("frac"), "traffic", r.get("traffic"), "per unit", r.get("traffic_per_unit"),
          "scaled by", r.get("scaled_by"), "frac_chain", r.get("frac_chain"))
print("ranks (rehearsal):", json.dumps(last("gpurun_out/rehearsal_2rank.json").get("ranks")))
PY
