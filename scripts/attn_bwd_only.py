#!/usr/bin/env python3
"""Flash attention backward only, one variant (for rocprofv3 --pmc passes on a single kernel).
usage: attn_bwd_only.py B H S D variant [reps]"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from flexflow_amd import kernels as Kn  # noqa: E402

B, H, S, D, var = (int(v) for v in sys.argv[1:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
dev = "cuda"
qkv = torch.randn(B, S, 3, H, D, device=dev).bfloat16()
o = torch.empty(B, S, H, D, device=dev, dtype=torch.bfloat16)
do = torch.randn_like(o)
dqkv = torch.empty_like(qkv)
sq = (S * 3 * H * D, D, 3 * H * D)
so = (S * H * D, D, H * D)
base, dbase = qkv.view(-1), dqkv.view(-1)
q, k, v = base, base[H * D:], base[2 * H * D:]
dq, dk, dv = dbase, dbase[H * D:], dbase[2 * H * D:]
X = Kn.ext()
lse = Kn.flash_attn_fwd(q, sq, k, sq, v, sq, o, so, B, H, S, S, D, D ** -0.5, False)
X.attn_set_bwd_variant(var)
for _ in range(reps):
    Kn.flash_attn_bwd(q, sq, k, sq, v, sq, o, so, do, so, lse, dq, sq, dk, sq, dv, sq, B, H, S, S, D, D ** -0.5, False)
torch.cuda.synchronize()
print("ok")
