#!/usr/bin/env python3
"""Forward flash attention throughput over sequence lengths at fixed total work (B * S^2 const):
separates the per-block cost (Q load, first K/V tile, O store) from the KV-loop cost.
usage: attn_fwd_sweep.py [H=16] [D=64] [variants=1]  (forward structures, attn_set_fwd_variant)"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from flexflow_amd import kernels as Kn  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 16
D = int(sys.argv[2]) if len(sys.argv) > 2 else 64
VARS = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "1").split(",")]
X = Kn.ext()
for B, S in ((128, 256), (32, 512), (8, 1024), (2, 2048), (1, 4096)):
    qkv = torch.randn(B, S, 3, H, D, device="cuda").bfloat16()
    o = torch.empty(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    sq, so = (S * 3 * H * D, D, 3 * H * D), (S * H * D, D, H * D)
    base = qkv.view(-1)
    f = lambda: Kn.flash_attn_fwd(base, sq, base[H * D:], sq, base[2 * H * D:], sq, o, so, B, H, S, S, D, D ** -0.5, False)
    fl = 4.0 * B * H * S * S * D
    for var in VARS:
        X.attn_set_fwd_variant(var)
        f()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                f()
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e) / 20)
        print(f"fwd variant {var} B={B} H={H} S={S} D={D}: {best * 1e3:.1f} us  {fl / best / 1e9:.0f} TF/s", flush=True)
