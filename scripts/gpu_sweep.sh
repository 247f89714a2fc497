#!/bin/bash
# Batch-size sweep of the flagship bench on one GPU (each run under its own time limit).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
for b in "$@"; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --batch-per-gpu $b > $OUT/sweep_b$b.log 2>&1
  rc=$?
  echo "b=$b rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
