#!/bin/bash
# Round-4 kernel checks: MoE kernels, fp32 GEMM / attention path, zoo fp32-vs-bf16. Stop at the
# first failure, abort, fault or timeout.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_moe_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "moe or topk or route or groupby or aggregate or f32" > $OUT/r4a_tests.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -15 $OUT/r4a_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "tracks_fp32" > $OUT/r4a_models.log 2>&1
rc=$?; echo "model tests rc=$rc"; tail -15 $OUT/r4a_models.log
exit $rc
