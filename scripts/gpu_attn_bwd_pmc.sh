#!/bin/bash
# PMC passes over attention-backward variants (one kernel per run): usage gpu_attn_bwd_pmc.sh v1 v2 ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abpmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES \
    -d $OUT/a$v -o run --output-format csv -- python3 $R/scripts/attn_bwd_only.py 32 16 512 64 $v 5 > $OUT/a$v.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
    -d $OUT/b$v -o run --output-format csv -- python3 $R/scripts/attn_bwd_only.py 32 16 512 64 $v 5 > $OUT/b$v.log 2>&1 || exit 1
  echo "variant $v"
  python3 $R/scripts/pmc_summary.py 'attn_bwd' $(find $OUT/a$v $OUT/b$v -name '*counter_collection.csv')
done
