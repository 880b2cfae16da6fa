#!/bin/bash
# C5 material split (probes/c5_material_split.py) on several library builds,
# interleaved twice: LIBS="tag=path tag=path ..."; then the C5-related GPU tests
# on the in-tree build.
set -o pipefail
mkdir -p gpurun_out/ab_c5m
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for tl in $LIBS; do
    tag=${tl%%=*}; lib=${tl#*=}
    echo "== $tag run $i"
    CTL_LIB=$lib timeout -k 10 300 python3 probes/c5_material_split.py > gpurun_out/ab_c5m/${tag}_$i.txt 2> gpurun_out/ab_c5m/${tag}_$i.err \
      || { echo "split $tag $i FAILED"; tail -5 gpurun_out/ab_c5m/${tag}_$i.err; exit 1; }
    cat gpurun_out/ab_c5m/${tag}_$i.txt
  done
done
[ "${NOTESTS:-0}" = 1 ] && exit 0
K=${1:-"c5 or texture or rough or alpha or env"}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" \
  > gpurun_out/ab_c5m/tests.txt 2>&1; rc=$?
tail -5 gpurun_out/ab_c5m/tests.txt
exit $rc
