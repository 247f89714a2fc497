#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/catprof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  FF_CAT_KERNEL=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/p$v -o run --output-format csv -- \
      python $R/bench.py --model inception_v3 --batch-per-gpu 64 --steps 6 --warmup 3 --no-hip-graphs > $OUT/p$v.log 2>&1 || exit $?
  f=$(ls $OUT/p$v/run_kernel_trace.csv $OUT/p$v/*/run_kernel_trace.csv 2>/dev/null | head -n 1)
  python $R/scripts/prof_steps.py "$f" --skip 3 --top 45 --delim adam_kernel > $OUT/steps_$v.txt 2>&1
  grep -o '"ms_per_step": [0-9.]*' $OUT/p$v.log
done
