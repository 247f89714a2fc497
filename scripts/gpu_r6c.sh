#!/bin/bash
# round 6 checkpoint: the whole GPU test suite, smoke, bench (+ tune log), a kernel-trace profile of
# the bench step, then PMC passes over the default attention backward. Stop at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r6c_tests.log 2>&1
rc=$?; tail -3 $OUT/r6c_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/r6c_smoke.log 2>&1
rc=$?; tail -1 $OUT/r6c_smoke.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_bench_prof.sh || exit $?
python3 scripts/prof_steps.py $OUT/prof/run_kernel_trace.csv --top 30 > $OUT/steps.txt 2>&1
bash scripts/gpu_attn_bwd_pmc.sh 10 > $OUT/r6c_attn_pmc.txt 2>&1
rc=$?; tail -30 $OUT/r6c_attn_pmc.txt; exit $rc
