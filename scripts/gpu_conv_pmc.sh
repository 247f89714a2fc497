#!/bin/bash
# PMC counters of one convolution pass (scripts/conv_one.py args), two counter passes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/cpmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
tag=$1; shift
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES \
  -d $OUT/${tag}_a -o run --output-format csv -- python3 $R/scripts/conv_one.py "$@" > $OUT/${tag}_a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE \
  -d $OUT/${tag}_b -o run --output-format csv -- python3 $R/scripts/conv_one.py "$@" > $OUT/${tag}_b.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum \
  -d $OUT/${tag}_c -o run --output-format csv -- python3 $R/scripts/conv_one.py "$@" > $OUT/${tag}_c.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $OUT/${tag}_t -o run --output-format csv -- python3 $R/scripts/conv_one.py "$@" > $OUT/${tag}_t.log 2>&1 || exit $?
echo done
