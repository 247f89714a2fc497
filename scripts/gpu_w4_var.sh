#!/bin/bash
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
for v in ${VARS:-0 1 2 3 4 7}; do echo "VAR=$v"; FF_W4_VAR=$v timeout -k 10 120 python -u scripts/gemm_bert_probe.py ${IMPLS:-w4,lib} 2 20 fwd 2>&1 | grep -E "^fwd" | head -4; done > $OUT/var_probe.log 2>&1
cat $OUT/var_probe.log
