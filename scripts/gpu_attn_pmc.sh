#!/bin/bash
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $OUT/apmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES \
  -d $OUT/apmc/c -o run --output-format csv -- python3 $R/scripts/attn_probe.py 32 16 512 64 5 > $OUT/apmc/c.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  -d $OUT/apmc/d -o run --output-format csv -- python3 $R/scripts/attn_probe.py 32 16 512 64 5 > $OUT/apmc/d.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/apmc/t -o run --output-format csv -- python3 $R/scripts/attn_probe.py 32 16 512 64 20 > $OUT/apmc/t.log 2>&1
