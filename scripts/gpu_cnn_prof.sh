#!/bin/bash
# Kernel-trace step profiles of the CNN benches (ResNet-50 and Inception-v3, b64, eager) plus the
# driver-style bench line of each. usage: gpu_cnn_prof.sh [models...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/cnnprof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for m in ${*:-resnet50 inception_v3}; do
  timeout -k 10 300 python $R/bench.py --model $m --batch-per-gpu 64 --steps 10 --warmup 5 > $OUT/bench_$m.log 2>&1 || exit $?
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$m -o run --output-format csv -- \
      python $R/bench.py --model $m --batch-per-gpu 64 --steps 6 --warmup 3 --no-hip-graphs > $OUT/prof_$m.log 2>&1 || exit $?
  f=$(ls $OUT/prof_$m/run_kernel_trace.csv $OUT/prof_$m/*/run_kernel_trace.csv 2>/dev/null | head -n 1)
  python $R/scripts/prof_steps.py "$f" --skip 3 --top 45 --delim adam_kernel > $OUT/steps_$m.txt 2>&1
done
echo all-ok
