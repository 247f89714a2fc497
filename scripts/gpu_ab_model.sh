#!/bin/bash
# Same-box A/B of a zoo model's bench between environment settings, interleaved:
#   bash scripts/gpu_ab_model.sh MODEL "ENV=a" "ENV=b" [rounds=2] [steps=20]
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
M=$1; shift
A=$1; B=$2; R=${3:-2}; S=${4:-20}
for r in $(seq 1 $R); do
  for cfg in "$A" "$B"; do
    env $cfg timeout -k 10 300 python bench.py --model $M --steps $S --warmup 5 > $OUT/abm_run.log 2>&1
    rc=$?
    echo "[$M $cfg] round $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/abm_run.log)"
    [ $rc -ne 0 ] && { tail -20 $OUT/abm_run.log; exit $rc; }
  done
done
exit 0
