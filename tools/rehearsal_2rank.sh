#!/bin/bash
# 2-rank rehearsal of bench.py's N-GPU path on the one-GPU box (both ranks on GPU 0, gloo for the
# collectives; RCCL needs one GPU per rank): the launcher, tile shards, max-over-ranks timing and
# the framebuffer reduce end to end.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 8 --warmup 2 --backend gloo --no-cpu-baseline --c5-passes 0 --wpt-passes 0 \
  --closest-shadow-passes 0 --one-pass-leg 0 --dopass-leg 0 --prim-passes 0 --binary-passes 0 \
  > gpurun_out/rehearsal_2rank.json 2> gpurun_out/rehearsal_2rank.err || { echo "REHEARSAL FAILED"; tail -30 gpurun_out/rehearsal_2rank.err; exit 1; }
cat gpurun_out/rehearsal_2rank.json
