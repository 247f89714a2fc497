#!/usr/bin/env bash
# dlrm: the searched strategy against data parallelism on every visible GPU (reference
# scripts/osdi22ae/dlrm.sh, which runs the same model with the Unity search and with
# --only-data-parallel). One process per GPU over RCCL; synthetic data, random-init weights.
set -euo pipefail
cd "$(dirname "$0")/../../.."
N=${N:-$(python -c 'import torch; print(max(1, torch.cuda.device_count()))')}
run() {
  if [ "$N" -gt 1 ]; then
    python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
      --master-port ${PORT:-29511} bench.py --gpus "$N" "$@"
  else
    python bench.py --gpus 1 "$@"
  fi
}
echo "Running dlrm with a parallelization strategy discovered by the unity search"
run --model dlrm --search unity --verify-steps 0 --steps ${STEPS:-10} --warmup ${WARMUP:-3}
echo "Running dlrm with data parallelism"
run --model dlrm --search dp --steps ${STEPS:-10} --warmup ${WARMUP:-3}
