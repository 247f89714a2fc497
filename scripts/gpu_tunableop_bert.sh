#!/bin/bash
# Re-tune TunableOp's library GEMM table on every BERT-Large bench call site (TN dgrads through
# the W^T copies, the padded 30528 vocabulary), then a same-box A/B of the old vs the merged table.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
FF_TUNABLEOP=tune FF_TUNABLEOP_FILE=$OUT/tunable_bert.csv PYTORCH_TUNABLEOP_VERBOSE=1 \
  timeout -k 10 1000 python bench.py --steps 2 --warmup 1 > $OUT/tunable_bert.log 2>&1
rc=$?; tail -2 $OUT/tunable_bert.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
ls -la $OUT/tunable_bert*.csv
exit 0
