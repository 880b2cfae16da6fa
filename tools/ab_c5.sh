#!/bin/bash
# A/B of two library builds on the C5 material split (probes/c5_material_split.py),
# interleaved: base, new, base, new.  BASE = path of the baseline .so (default
# _ab/base.so), NEW = the in-tree build.  Then the C5-related GPU tests on NEW.
#   bash tools/ab_c5.sh [pytest -k expression]
set -o pipefail
BASE=${BASE:-_ab/base.so}
NEW=${NEW:-cudatracerlib_amd/_lib/libctl_trace.so}
mkdir -p gpurun_out/ab_c5
for i in 1 2; do
  for tag in base new; do
    lib=$BASE; [ $tag = new ] && lib=$NEW
    echo "== $tag run $i ($lib)"
    CTL_LIB=$lib timeout -k 10 300 python3 probes/c5_material_split.py > gpurun_out/ab_c5/${tag}_$i.txt 2> gpurun_out/ab_c5/${tag}_$i.err \
      || { echo "split $tag $i FAILED"; tail -5 gpurun_out/ab_c5/${tag}_$i.err; exit 1; }
    cat gpurun_out/ab_c5/${tag}_$i.txt
  done
done
K=${1:-"c5 or texture or rough or alpha or env"}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" \
  > gpurun_out/ab_c5/tests.txt 2>&1; rc=$?
tail -5 gpurun_out/ab_c5/tests.txt
exit $rc
