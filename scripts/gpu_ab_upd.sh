#!/bin/bash
# A/B of the overlapped optimizer update's scheduling: the step on a high-priority stream
# (FF_COMPUTE_PRIO) x update workgroup shape (FF_UPD_BLOCKS: 0 = 2048-block sweep, -N = short-lived
# blocks of N float4 per thread), interleaved rounds of bench.py on one box.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
: > $OUT/ab_upd.txt
for rnd in 1 2 3; do
  for cfg in "default:0" "high:0" "high:-2" "default:-2"; do
    p=${cfg%%:*}; b=${cfg##*:}
    FF_COMPUTE_PRIO=$p FF_UPD_BLOCKS=$b timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/ab_upd_run.log 2>&1 || { tail -5 $OUT/ab_upd_run.log; exit 1; }
    echo "round $rnd compute_prio=$p upd_blocks=$b $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_upd_run.log)" | tee -a $OUT/ab_upd.txt
  done
done
