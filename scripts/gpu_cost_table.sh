#!/bin/bash
# Measured-cost table for bench.py's N > 1 search, and the determinism check of the measured costs
# (VERDICT r5 item 4): two independent measurement passes of the N = 8 plan, then the shipped table
# for N = 2, 4, 8 (flexflow_amd/pcg/data/op_costs_mi355x.json, copied back via gpurun_out/).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
step() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; grep '^{' $OUT/$name.log || tail -5 $OUT/$name.log
  return $rc
}
WHICH=${1:-all}
if [ "$WHICH" = all ] || [ "$WHICH" = det ]; then
  FF_COST_CACHE=0 step cost_det 900 python -u scripts/cost_table.py 8 8 || exit $?
fi
if [ "$WHICH" = all ] || [ "$WHICH" = table ]; then
  rm -f $OUT/op_costs_mi355x.json
  FF_COST_CACHE=$OUT/op_costs_mi355x.json step cost_table 900 python -u scripts/cost_table.py 8 4 2 || exit $?
  FF_COST_CACHE=$OUT/op_costs_mi355x.json step cost_table_reread 300 python -u scripts/cost_table.py 8 || exit $?
fi
exit 0
