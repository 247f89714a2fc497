#!/bin/bash
# The native model examples at their full sizes on one GPU (10 timed iterations each). A Python
# error in one example is recorded and the next runs; an abort / fault / timeout stops the script.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
: > $OUT/examples.log
cd examples/python/native
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python $name.py "$@" > $OUT/ex_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(grep -E 'THROUGHPUT|Error' $OUT/ex_$name.log | tail -1)" | tee -a $OUT/examples.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name"; exit $rc; fi
}
run alexnet 240 -b 256 --iterations 10
run resnet 300 -b 64 -e 1 --samples 1024
run resnext50 300 -b 64 --iterations 10
run inception 300 -b 64 --iterations 10
run dlrm 240 -b 2048 --iterations 10
run xdl 240 -b 2048 --iterations 10
run candle_uno 240 -b 256 --iterations 10
run mlp_unify 240 -b 64 --iterations 10
run transformer 300 -b 8 --iterations 10
run mixture_of_experts 240 -b 64 --iterations 10
run nmt 300 -b 64 --iterations 10
