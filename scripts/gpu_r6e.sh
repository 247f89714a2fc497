#!/bin/bash
# round 6 (session 2): W^T copies for TN dgrads — tests, layout probe, same-box bench A/B
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transfer_gpu.py -k "transpose" > $OUT/t_wt.log 2>&1
rc=$?; tail -3 $OUT/t_wt.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/dgrad_layout_probe.py 3 20 > $OUT/dgrad_layout.txt 2>&1
rc=$?; cat $OUT/dgrad_layout.txt; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_ab_bench.sh "FF_WT_COPY=0" "FF_WT_COPY=1" 2 20
