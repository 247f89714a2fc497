#!/bin/bash
# Simulator calibration at N = 1 for the three calibrated model classes:
# BERT-Large b32, ResNet-50 b64, Inception-v3 b64. Stops at the first failing run.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
MODELS=${1:-"bert-large:32 resnet50:64 inception_v3:64"}
for mb in $MODELS; do
  m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 400 python -u scripts/calibrate_sim.py $m $b 4 > $OUT/calib_$m.txt 2>&1
  rc=$?
  echo "[$m b$b] rc=$rc"; grep -E "^OP_|simulated step" $OUT/calib_$m.txt
  [ $rc -ne 0 ] && { tail -20 $OUT/calib_$m.txt; exit $rc; }
done
exit 0
