#!/bin/bash
# One GPU session: tests, bench, profile. Each GPU step has its own time limit; stop at the first
# abort / fault / timeout (rc >= 124) so nothing else touches a possibly-wedged GPU.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $OUT/steps.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
: > $OUT/steps.log
for step in "$@"; do
  case $step in
    tests) run tests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ;;
    ktests) run ktests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q --timeout 120 --timeout-method thread ;;
    attn) run attn 300 python -u -m pytest tests/test_kernels_gpu.py -q -k flash --timeout 120 --timeout-method thread ;;
    probe) run probe 200 python scripts/attn_probe.py 32 16 512 64 20 ;;
    mtests) run mtests 900 python -u -m pytest tests/test_models_gpu.py -q --timeout 400 --timeout-method thread ;;
    dtests) run dtests 600 python -u -m pytest tests/test_distributed_gpu.py -q --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    calib) run calib 600 python -u scripts/calibrate_sim.py bert-large 32 6 ;;
    gemmprobe) run gemmprobe 400 python -u scripts/gemm_bert_probe.py w4,lib 3 20 ;;
    bench) FF_TUNE_LOG=$OUT/tune.json run bench 600 python bench.py --steps 10 --warmup 3 ;;
    microbench) run microbench 400 python scripts/bench_kernels.py ;;
    prof) cd /tmp && export TMPDIR=/tmp && run prof 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-hip-graphs; cd - >/dev/null ;;
  esac
done
