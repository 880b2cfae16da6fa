#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python probes/shard_diag.py > gpurun_out/diag_base.log 2>&1 || { echo FAIL; tail gpurun_out/diag_base.log; exit 1; }
tail -15 gpurun_out/diag_base.log
CTL_LIB=$PWD/cudatracerlib_amd/_varnopark/libctl_trace.so timeout -k 10 400 python probes/shard_diag.py > gpurun_out/diag_nopark.log 2>&1 || { echo FAIL; tail gpurun_out/diag_nopark.log; exit 1; }
tail -15 gpurun_out/diag_nopark.log
