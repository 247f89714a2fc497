#!/bin/bash
# 1-GPU throughput of the zoo models named in BASELINE.json's configs (synthetic data, bf16).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
: > $OUT/zoo.jsonl
for spec in "alexnet 256" "resnet50 64" "inception_v3 64" "dlrm 2048 --optimizer sgd" "bert-base 32"; do
  set -- $spec
  timeout -k 10 300 python bench.py --model $1 --batch-per-gpu $2 "${@:3}" --steps 10 --warmup 5 > $OUT/zoo_$1.log 2>&1
  rc=$?
  echo "$1 rc=$rc" >> $OUT/steps.log
  tail -n 1 $OUT/zoo_$1.log >> $OUT/zoo.jsonl
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
