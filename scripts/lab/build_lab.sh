#!/bin/bash
# Build the attention-backward lab executable (CPU cross-compile for gfx950).
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../csrc/kernels attn_bwd_lab.hip \
  ../../csrc/kernels/attention.hip -o attn_bwd_lab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../csrc/kernels attn_fwd_lab.hip \
  ../../csrc/kernels/attention.hip -o attn_fwd_lab
