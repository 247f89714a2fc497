#!/usr/bin/env python3
"""Column-fold (col_reduce_add3) time vs row chunks per column block, at the BERT-Large shapes:
LayerNorm backward slabs (R = 1024 rows x 1024 columns, 3 outputs) and bias_act_bwd slabs
(R = 64 x 4096 / R = 256 x 1024, 1 output). usage: fold_probe.py"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from flexflow_amd import kernels as Kn  # noqa: E402

X = Kn.ext()
for R, C, nz in ((1024, 1024, 3), (64, 4096, 1), (256, 1024, 1), (1024, 4096, 1)):
    part = torch.randn(3 * R * C, device="cuda")
    outs = [torch.zeros(C, device="cuda") if i < nz else None for i in range(3)]
    ref = part.view(3, R, C)[:nz].sum(1)
    line = []
    for gy in (0, 1, 4, 8, 32):
        X.col_reduce_set_gy(gy)
        for o in outs[:nz]:
            o.zero_()
        X.col_reduce_add3(part, *outs, R, C)
        err = max((o - ref[i]).abs().max().item() for i, o in enumerate(outs[:nz]))
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(3):
            s.record()
            for _ in range(50):
                X.col_reduce_add3(part, *outs, R, C)
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e) / 50 * 1e3)
        line.append(f"gy={gy}: {best:6.1f} us (err {err:.1e})")
    print(f"R={R} C={C} outs={nz}: " + "  ".join(line), flush=True)
