#!/bin/bash
# HBM bytes per kernel over a short BERT-Large run (one counter group per pass: FETCH_SIZE takes 3
# TCC slots, WRITE_SIZE 2, at most 4 per run) + the attention PMC passes.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $OUT/bw
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $OUT/bw/f -o run --output-format csv -- \
  python3 $R/bench.py --steps 2 --warmup 1 > $OUT/bw/f.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d $OUT/bw/w -o run --output-format csv -- \
  python3 $R/bench.py --steps 2 --warmup 1 > $OUT/bw/w.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/bw/t -o run --output-format csv -- \
  python3 $R/bench.py --steps 2 --warmup 1 > $OUT/bw/t.log 2>&1
