#!/bin/bash
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_runtime_gpu.py -m gpu -k "batched" > gpurun_out/t_cnnfold.log 2>&1 || { tail -40 gpurun_out/t_cnnfold.log; exit 1; }
tail -1 gpurun_out/t_cnnfold.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_models_gpu.py tests/test_runtime_gpu.py -m gpu > gpurun_out/t_cnnfold2.log 2>&1 || { tail -40 gpurun_out/t_cnnfold2.log; exit 1; }
tail -1 gpurun_out/t_cnnfold2.log
bash scripts/gpu_ab_model.sh inception_v3 "FF_FOLD_BATCH=0" "FF_FOLD_BATCH=1" 3 20 || exit 1
bash scripts/gpu_ab_model.sh resnet50 "FF_FOLD_BATCH=0" "FF_FOLD_BATCH=1" 2 20 || exit 1
