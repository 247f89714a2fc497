#!/bin/bash
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
bash scripts/rehearse_n2.sh bert-large 8 || { tail -30 gpurun_out/rehearse_n2.log; exit 1; }
tail -1 gpurun_out/rehearse_n2.log
