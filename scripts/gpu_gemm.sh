#!/bin/bash
# GEMM numerics (gpu tests for gemm only) + per-impl timings on BERT-Large shapes.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k gemm > $OUT/gemm_tests.log 2>&1
rc=$?; echo "gemm_tests rc=$rc" >> $OUT/steps.log; [ $rc -ne 0 ] && exit $rc
: > $OUT/gemm_probe.log
for shp in "8192 8192 8192 1 1" "8192 3072 1024 1 1" "8192 1024 1024 1 1" "8192 4096 1024 1 1" "8192 1024 4096 1 1" \
           "8192 1024 1024 1 0" "8192 4096 1024 1 0" "8192 1024 4096 1 0" "8192 1024 3072 1 0" \
           "1024 1024 8192 0 0" "1024 4096 8192 0 0" "4096 1024 8192 0 0" "3072 1024 8192 0 0" \
           "16384 1024 4096 1 1" "16384 4096 1024 1 1" "2048 4096 16384 0 0"; do
  for impl in k256 big lib; do
    timeout -k 10 60 python scripts/gemm_probe.py $shp $impl 30 >> $OUT/gemm_probe.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "probe $shp $impl rc=$rc" >> $OUT/steps.log; exit $rc; }
  done
done
echo "probe done" >> $OUT/steps.log
