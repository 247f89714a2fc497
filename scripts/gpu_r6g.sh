#!/bin/bash
# round 6: numerics (BERT losses) and same-box bench A/B of W^T refresh placement and the wgrad stream
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
for cfg in "FF_WT_COPY=0" "FF_WT_STREAM=main" "FF_WT_STREAM=main FF_WGRAD_STREAM=1"; do
  env $cfg timeout -k 10 300 python scripts/bert_loss_check.py 8 4 4 > $OUT/loss.log 2>&1
  rc=$?; echo "[$cfg] $(tail -1 $OUT/loss.log)"; [ $rc -ne 0 ] && exit $rc
done
ROUNDS=2 bash scripts/gpu_ab_multi.sh "FF_WT_COPY=0" "FF_WT_STREAM=main" "FF_WT_STREAM=main FF_WGRAD_STREAM=1"
