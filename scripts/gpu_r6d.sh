#!/bin/bash
# round 6: bench.py's multi-rank path rehearsed with 2 ranks on the one GPU (gloo), the 1-GPU zoo,
# and the CNN step profiles. Stop at the first failure.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
bash scripts/rehearse_n2.sh bert-large 8; rc=$?; tail -2 $OUT/rehearse_n2.log | cut -c1-1500; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_zoo.sh || exit $?
cat $OUT/zoo.jsonl | cut -c1-200
bash scripts/gpu_cnn_prof.sh inception_v3 resnet50
