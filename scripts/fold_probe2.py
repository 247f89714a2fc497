#!/usr/bin/env python3
"""Bias-gradient column fold timing at BERT-Large shapes (16384 rows): bias_act_bwd(act NONE) =
column-sum pass + fold, and layernorm_bwd (dgamma, dbeta, dsum folds)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from flexflow_amd import kernels as Kn  # noqa: E402

X = Kn.ext()
dev = "cuda"


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


rows = 16384
for cols in (1024, 3072, 4096):
    dy = torch.randn(rows, cols, device=dev).bfloat16()
    db = torch.zeros(cols, device=dev)
    print(f"bias colsum {rows}x{cols}: {timed(lambda: X.bias_act_bwd(dy, None, None, db, rows, cols, 10)):7.1f} us", flush=True)
cols = 1024
x = torch.randn(rows, cols, device=dev).bfloat16()
g = torch.randn(cols, device=dev).bfloat16()
mean = torch.zeros(rows, device=dev)
rstd = torch.ones(rows, device=dev)
dx = torch.empty_like(x)
dg = torch.zeros(cols, device=dev)
dbb = torch.zeros(cols, device=dev)
dsum = torch.zeros(cols, device=dev)
print(f"layernorm_bwd {rows}x{cols} (+dsum): {timed(lambda: X.layernorm_bwd(x, x, g, mean, rstd, dx, None, dg, dbb, rows, cols, False, dsum)):7.1f} us", flush=True)
