#!/bin/bash
# end-of-round check: whole GPU suite + smoke, then the driver-style bench (default config) and a
# step profile of it; stops at the first failure
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
bash $R/scripts/gpu_fulltests.sh || exit $?
cd $R && timeout -k 10 400 python bench.py > $OUT/bench_final.log 2>&1 || { tail -20 $OUT/bench_final.log; exit 1; }
tail -1 $OUT/bench_final.log
