#!/bin/bash
# The GEMM autotuner's choice at every call site of every zoo model (FF_TUNE_LOG per model), for the
# consolidation of the GEMM family: which kernels still win a site.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/zootune
mkdir -p $OUT
for spec in "bert-large 32" "bert-base 32" "alexnet 256" "resnet50 64" "resnext50 64" "inception_v3 64" \
            "dlrm 2048 --optimizer sgd" "xdl 1024" "candle_uno 256" "mlp_unify 256" "transformer 32" "moe 256" "nmt 64" "mnist_mlp 256"; do
  set -- $spec
  FF_TUNE_LOG=$OUT/tune_$1.json timeout -k 10 300 python bench.py --model $1 --batch-per-gpu $2 "${@:3}" --steps 3 --warmup 3 \
    > $OUT/bench_$1.log 2>&1
  rc=$?
  echo "$1 rc=$rc $(tail -c 300 $OUT/bench_$1.log | tr '\n' ' ' | cut -c1-200)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
exit 0
