#!/bin/bash
# BASELINE configs #3 / #4 with MEASURED op costs: one process on the GPU box
# plans for N = 8 devices; op costs are timed on the card, the comm terms come from the machine
# model. Writes gpurun_out/search_*_r5.json (+ .log); stops at the first failing run.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
export FF_SEARCH_PROGRESS=1
export FF_JOINT_MAX_GRAPHS=${FF_JOINT_MAX_GRAPHS:-256}
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 $limit python -u scripts/export_search.py "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -c 400 $OUT/$name.log; echo
  return $rc
}
WHICH=${1:-all}
if [ "$WHICH" = all ] || [ "$WHICH" = inception ]; then
  run search_inception_v3_8dev_unity_attr_r5 500 inception_v3 8 $OUT/search_inception_v3_8dev_unity_attr_r5.json unity 64 \
      --enable-attribute-parallel --budget 10 || exit $?
  run search_inception_v3_8dev_mcmc_attr_r5 500 inception_v3 8 $OUT/search_inception_v3_8dev_mcmc_attr_r5.json mcmc 64 \
      --enable-attribute-parallel --budget 2000 || exit $?
fi
if [ "$WHICH" = all ] || [ "$WHICH" = bert ]; then
  # b8 and b32 per GPU: global 64 and 256
  run search_bert-large_8dev_b8_r5 500 bert-large 8 $OUT/search_bert-large_8dev_b8_r5.json unity 64 --budget 30 || exit $?
  run search_bert-large_8dev_b32_r5 500 bert-large 8 $OUT/search_bert-large_8dev_b32_r5.json unity 256 --budget 30 || exit $?
fi
exit 0
