#!/bin/bash
# round 6: step profiles with and without the W^T copies (FF_WT_COPY), tune logs kept
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
for v in 1 0; do
  export FF_WT_COPY=$v
  FF_TUNE_LOG=$OUT/tune_wt$v.json timeout -k 10 600 python bench.py --steps 10 --warmup 3 > $OUT/bench_wt$v.log 2>&1
  rc=$?; tail -1 $OUT/bench_wt$v.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
  (cd /tmp && TMPDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_wt$v -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 2 --no-hip-graphs > $OUT/prof_wt$v.log 2>&1)
  rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 scripts/prof_steps.py $(find $OUT/prof_wt$v -name "*kernel_trace.csv" | head -1) --top 32 > $OUT/steps_wt$v.txt 2>&1
  cat $OUT/steps_wt$v.txt
done
exit 0
