#!/bin/bash
# GEMM kernel check: numerics of every GEMM kernel, then the BERT-Large shape probe.
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm" --timeout 120 --timeout-method thread > $OUT/gemm_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/gemm_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/gemm_bert_probe.py ${1:-pp,k256,lib} 3 20 ${2:-fwd,dgrad,wgrad} > $OUT/gemm_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; cat $OUT/gemm_probe.log
exit $rc
