#!/bin/bash
# PMC counters (two passes, counters only) for GEMM configs given as "M N K a_k b_k impl" strings
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $OUT/pmc
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES \
    -d $OUT/pmc/c$i -o run --output-format csv -- python3 $R/scripts/gemm_probe.py $cfg > $OUT/pmc/c$i.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE \
    -d $OUT/pmc/d$i -o run --output-format csv -- python3 $R/scripts/gemm_probe.py $cfg > $OUT/pmc/d$i.log 2>&1 || exit $?
  echo "== cfg $i: $cfg"
  python3 $R/scripts/pmc_summary.py "gemm|Cijk" $(find $OUT/pmc/c$i $OUT/pmc/d$i -name "*counter_collection.csv")
done
