#!/usr/bin/env python3
"""Run flash attention fwd+bwd repeatedly on one shape (for rocprofv3 --pmc / --kernel-trace).
usage: attn_probe.py B H S D [reps]"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from flexflow_amd import kernels as Kn  # noqa: E402

B, H, S, D = (int(v) for v in sys.argv[1:5])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 10
dev = "cuda"
qkv = torch.randn(B, S, 3, H, D, device=dev).bfloat16()
o = torch.empty(B, S, H, D, device=dev, dtype=torch.bfloat16)
do = torch.randn_like(o)
dqkv = torch.empty_like(qkv)
sq = (S * 3 * H * D, D, 3 * H * D)  # (b, h, s) strides of q/k/v inside qkv
so = (S * H * D, D, H * D)
base, dbase = qkv.view(-1), dqkv.view(-1)
q, k, v = base, base[H * D:], base[2 * H * D:]
dq, dk, dv = dbase, dbase[H * D:], dbase[2 * H * D:]
scale = D ** -0.5
for i in range(reps + 2):
    if i == 2:
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
    lse = Kn.flash_attn_fwd(q, sq, k, sq, v, sq, o, so, B, H, S, S, D, scale, False)
    Kn.flash_attn_bwd(q, sq, k, sq, v, sq, o, so, do, so, lse, dq, sq, dk, sq, dv, sq, B, H, S, S, D, scale, False)
e.record()
e.synchronize()
ms = s.elapsed_time(e) / reps
fl = 4.0 * B * H * S * S * D * 3.5
print(f"attn fwd+bwd B={B} H={H} S={S} D={D}: {ms:.3f} ms  {fl / ms / 1e9:.1f} TFLOPS (fwd+bwd)")
