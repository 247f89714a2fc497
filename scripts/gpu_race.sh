#!/bin/bash
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
for cfg in "3 512 512 512 1 0 0" "3 512 512 512 1 1 1" "3 512 512 512 1 1 0" "3 2048 2048 2048 3 0 0" "3 2048 1024 16384 8 0 0" "3 8192 1024 4096 1 1 0"; do
  echo "== $cfg"; timeout -k 10 60 python -u scripts/gemm_race_check.py $cfg ${REPS:-40} | tail -4 || exit $?
done > $OUT/race.log 2>&1
rc=$?; cat $OUT/race.log; exit $rc
