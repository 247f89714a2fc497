#!/bin/bash
# bench (tune log) then a rocprof kernel-trace profile of the same step; stop at the first failure
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
FF_TUNE_LOG=$OUT/tune.json timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup 3 > $OUT/bench.log 2>&1
rc=$?; tail -1 $OUT/bench.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-hip-graphs > $OUT/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
