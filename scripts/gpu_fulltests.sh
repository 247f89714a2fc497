#!/bin/bash
# the whole GPU test suite + smoke, stop at the first failure
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/full_tests.log 2>&1
rc=$?; tail -5 $OUT/full_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; exit $rc
