#!/bin/bash
# PMC counters for one GEMM config (counters only with --kernel-trace-free --pmc runs, per pool rules).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $OUT/pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/pmc/counters_list.txt 2>&1 || true
i=0
for cfg in "$@"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES \
    -d $OUT/pmc/c$i -o run --output-format csv -- python3 $R/scripts/gemm_probe.py $cfg > $OUT/pmc/c$i.log 2>&1
  rc=$?
  echo "pmc $cfg rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    -d $OUT/pmc/d$i -o run --output-format csv -- python3 $R/scripts/gemm_probe.py $cfg > $OUT/pmc/d$i.log 2>&1
  rc=$?
  echo "pmc2 $cfg rc=$rc" >> $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
