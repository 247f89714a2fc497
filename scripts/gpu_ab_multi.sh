#!/bin/bash
# Same-box interleaved bench A/B/C... between environment settings:
#   ROUNDS=2 STEPS=20 bash scripts/gpu_ab_multi.sh "FF_X=0" "FF_X=1" "FF_X=1 FF_Y=2"
# Stops at the first failing / timed-out run; exits 0 when every run passed.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
R=${ROUNDS:-2}; S=${STEPS:-20}
: > $OUT/ab.log
for r in $(seq 1 $R); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 300 python bench.py --steps $S --warmup 5 > $OUT/ab_run.log 2>&1
    rc=$?
    echo "[$cfg] round $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_run.log)" | tee -a $OUT/ab.log
    if [ $rc -ne 0 ]; then tail -20 $OUT/ab_run.log; exit $rc; fi
  done
done
exit 0
