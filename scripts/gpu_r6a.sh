#!/bin/bash
# round 6: fused-dgrad pp epilogue + kept attention kernels + overlapping add boxes (tests), then
# the FFN2-dgrad probe. Each GPU step under its own limit; stop at the first failure.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_transfer_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "dact or flash or add_mode" > $OUT/r6a_tests.log 2>&1
rc=$?; tail -3 $OUT/r6a_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/gemm_dact_probe.py > $OUT/r6a_probe.log 2>&1
rc=$?; cat $OUT/r6a_probe.log; exit $rc
