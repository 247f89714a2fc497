#!/bin/bash
# Same-box A/B of the flagship bench between environment settings, interleaved:
#   bash scripts/gpu_ab_bench.sh "FF_DEFER_FOLDS=0" "FF_DEFER_FOLDS=1" [rounds=2] [steps=20]
# Stops at the first failing / timed-out run.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
A=$1; B=$2; R=${3:-2}; S=${4:-20}
: > $OUT/ab.log
for r in $(seq 1 $R); do
  for cfg in "$A" "$B"; do
    env $cfg timeout -k 10 300 python bench.py --steps $S --warmup 5 > $OUT/ab_run.log 2>&1
    rc=$?
    echo "[$cfg] round $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_run.log)" | tee -a $OUT/ab.log
    [ $rc -ne 0 ] && { tail -20 $OUT/ab_run.log; exit $rc; }
  done
done
