#!/bin/bash
# CNN path on one GPU: channel-last kernel tests, CNN model gradient tests, zoo CNN throughput,
# a kernel-trace profile of an Inception-v3 b64 step and the conv layer probe.
# usage: gpu_cnn.sh [tests|models|bench|prof|probe]...   (default: all, in that order)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/cnn
mkdir -p $OUT
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then tail -n 30 $OUT/$name.log; exit $rc; fi
}
steps=${*:-tests models bench prof probe}
for s in $steps; do
  case $s in
    tests) run tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
             -k "batchnorm or pool or conv2d or chan_sum or elementwise_channel" ;;
    models) run models 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_models_gpu.py ;;
    bench) for spec in "inception_v3 64" "resnet50 64" "alexnet 256"; do
             set -- $spec
             run bench_$1 300 python bench.py --model $1 --batch-per-gpu $2 --steps 10 --warmup 5
             tail -n 1 $OUT/bench_$1.log >> $OUT/bench.jsonl
           done ;;
    prof) cd /tmp && export TMPDIR=/tmp
          run prof 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
              python $R/bench.py --model inception_v3 --batch-per-gpu 64 --steps 6 --warmup 3 --no-hip-graphs
          cd - > /dev/null
          f=$(ls $OUT/prof/*/run_kernel_trace.csv 2>/dev/null | head -n 1 || true)
          [ -n "$f" ] && python $R/scripts/prof_steps.py "$f" --skip 3 --top 40 --delim adam_kernel > $OUT/prof_steps.txt 2>&1
          ;;
    probe) run probe 400 python scripts/conv_probe.py ;;
  esac
done
echo all-ok
