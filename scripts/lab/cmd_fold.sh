#!/bin/bash
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_runtime_gpu.py tests/test_transfer_gpu.py tests/test_models_gpu.py -m gpu > gpurun_out/t_fold.log 2>&1 || { tail -40 gpurun_out/t_fold.log; exit 1; }
tail -2 gpurun_out/t_fold.log
ROUNDS=3 bash scripts/gpu_ab_multi.sh "FF_FOLD_BATCH=0" "FF_FOLD_BATCH=1" || exit 1
cd /tmp && export TMPDIR=/tmp
FF_FOLD_BATCH=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_fold -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_fold.log 2>&1 || exit 1
