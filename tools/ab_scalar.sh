#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export C5SPLIT_ONLY="C5;neither, full;rough only;textures only"
LIBS="base=_ab/base.so scalar=cudatracerlib_amd/_lib/libctl_trace.so" bash tools/ab_libs.sh || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wide or parity or reference_order or fullsize or intersect or occluded" > gpurun_out/ab_libs/tests.txt 2>&1; rc=$?
tail -3 gpurun_out/ab_libs/tests.txt
exit $rc
