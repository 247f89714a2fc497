#!/bin/bash
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
bash scripts/gpu_ab_model.sh resnet50 "FF_FOLD_BATCH=0" "FF_FOLD_BATCH=1" 2 20 || exit 1
bash scripts/gpu_ab_model.sh dlrm "FF_FOLD_BATCH=0" "FF_FOLD_BATCH=1" 2 20 || exit 1
bash scripts/gpu_ab_model.sh bert-base "FF_FOLD_BATCH=0" "FF_FOLD_BATCH=1" 2 20 || exit 1
