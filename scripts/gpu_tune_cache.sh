#!/bin/bash
# The ResNet-50 / AlexNet native examples twice with FF_TUNE_CACHE: the second run reuses the
# first run's autotune choices (first-step timing skipped)
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
export FF_TUNE_CACHE=$OUT/tune_cache.json
rm -f $FF_TUNE_CACHE
: > $OUT/tune_cache_runs.log
cd examples/python/native
for run in cold warm; do
  for ex in resnet alexnet; do
    timeout -k 10 300 python $ex.py -b 64 -e 1 --samples 1024 > $OUT/tc_${ex}_$run.log 2>&1 || exit $?
    echo "$run $ex: $(grep THROUGHPUT $OUT/tc_${ex}_$run.log | tail -1)" | tee -a $OUT/tune_cache_runs.log
  done
done
python -c "import json; d=json.load(open('$FF_TUNE_CACHE')); print({k: len(v) for k, v in d.items()})" | tee -a $OUT/tune_cache_runs.log
