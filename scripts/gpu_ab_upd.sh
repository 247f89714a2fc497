#!/bin/bash
# A/B of the overlapped optimizer update's scheduling: stream priority (FF_UPD_PRIO) x workgroup
# shape (FF_UPD_BLOCKS: 0 = 2048-block sweep, -N = short-lived blocks of N float4 per thread),
# interleaved rounds of bench.py on one box.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
python -c "import torch; print('priority_range', torch.cuda.Stream.priority_range())"
: > $OUT/ab_upd.txt
for rnd in 1 2; do
  for cfg in "default:0" "low:0" "default:-2" "low:-2" "low:-8"; do
    p=${cfg%%:*}; b=${cfg##*:}
    FF_UPD_PRIO=$p FF_UPD_BLOCKS=$b timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/ab_upd_run.log 2>&1 || { tail -5 $OUT/ab_upd_run.log; exit 1; }
    echo "round $rnd prio=$p blocks=$b $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_upd_run.log)" | tee -a $OUT/ab_upd.txt
  done
done
