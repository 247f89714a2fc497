#!/bin/bash
# Persistent 4-wave GEMM: numerics (GPU tests), then the BERT-Large call-site probe against the
# one-tile-per-workgroup kernel and hipBLASLt. Each step has its own time limit; stop at the first
# failure, abort, fault or timeout.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "gemm_persistent or gemm_layouts or gemm256_shapes" > $OUT/w4p_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/w4p_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/gemm_bert_probe.py ${PROBE_IMPLS:-w4p,w4,lib} 3 20 > $OUT/w4p_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -32 $OUT/w4p_probe.log
exit $rc
