#!/bin/bash
# Rehearse bench.py's multi-rank path (search + measured verification vs DP + timed steps) with two
# ranks sharing the one GPU of a gpurun box over gloo (RCCL refuses two ranks on one device).
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
FF_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --model ${1:-bert-base} --batch-per-gpu ${2:-8} \
  --steps 3 --warmup 2 --verify-steps 2 > $OUT/rehearse_n2.log 2>&1
