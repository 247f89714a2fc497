#!/bin/bash
# Same-box interleaved A/B between two builds of the HIP extension (abso/_C_A.so vs abso/_C_B.so,
# copied over flexflow_amd/_C.so before each run): ROUNDS=2 STEPS=20 bash scripts/gpu_ab_so.sh [bench args]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
N=${ROUNDS:-2}; S=${STEPS:-20}
: > $OUT/ab_so.log
for r in $(seq 1 $N); do
  for arm in A B; do
    cp abso/_C_$arm.so flexflow_amd/_C.so || exit 1
    timeout -k 10 300 python bench.py --steps $S --warmup 5 "$@" > $OUT/ab_so_run.log 2>&1
    rc=$?
    echo "[$arm] round $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_so_run.log)" | tee -a $OUT/ab_so.log
    if [ $rc -ne 0 ]; then tail -20 $OUT/ab_so_run.log; exit $rc; fi
  done
done
cp abso/_C_B.so flexflow_amd/_C.so
exit 0
