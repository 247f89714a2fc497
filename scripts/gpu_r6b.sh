#!/bin/bash
# round 6: simulator calibration (BERT-Large b32, per-op errors) then the measured-cost table and
# its determinism check (scripts/gpu_cost_table.sh). Stop at the first failure.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
timeout -k 10 500 python -u scripts/calibrate_sim.py bert-large 32 4 > $OUT/calib_bert-large_r6.txt 2>&1
rc=$?; grep -E "^OP_|simulated step|worst" $OUT/calib_bert-large_r6.txt; [ $rc -ne 0 ] && { tail -20 $OUT/calib_bert-large_r6.txt; exit $rc; }
bash scripts/gpu_cost_table.sh all
