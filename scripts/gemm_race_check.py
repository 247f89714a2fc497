#!/usr/bin/env python3
"""Repeat one GEMM kernel on fixed inputs and report which 256x256 output tiles ever differ from the
fp32 reference (and from the kernel's own first result): a diagnostic for intermittent wrong tiles.
usage: gemm_race_check.py impl M N K splitk a_k b_k reps"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from flexflow_amd import kernels as Kn  # noqa: E402

impl, M, N, K, sk = (int(x) for x in sys.argv[1:6])
a_k, b_k = sys.argv[6] == "1", sys.argv[7] == "1"
reps = int(sys.argv[8])
X = Kn.ext()
torch.manual_seed(11)
Am = torch.randn(M, K, device="cuda").bfloat16()
Bn = torch.randn(N, K, device="cuda").bfloat16()
A = Am if a_k else Am.t().contiguous()
B = Bn if b_k else Bn.t().contiguous()
ref = Am.float() @ Bn.float().t()
ws = torch.empty(M * N * sk, device="cuda") if sk > 1 else None
first = None
bad_tiles = {}
for r in range(reps):
    C = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    X.gemm(A, B, C, None, None, M, N, K, A.shape[-1], B.shape[-1], N, 0, 0, 0, 1, a_k, b_k, 1.0, 0.0, 10, sk, ws, impl)
    torch.cuda.synchronize()
    err = ((C.float() - ref).abs() > 0.05 * ref.abs().clamp_min(1.0))
    if first is None:
        first = C.clone()
    diff_self = (C != first).sum().item()
    nbad = err.sum().item()
    if nbad:
        t = err.reshape((M + 255) // 256, 256, (N + 255) // 256, 256).any(3).any(1).nonzero().tolist()
        for tt in t:
            bad_tiles[tuple(tt)] = bad_tiles.get(tuple(tt), 0) + 1
        rows = err.any(1).nonzero().flatten()
        cols = err.any(0).nonzero().flatten()
        print(f"rep {r}: {nbad} bad elems, tiles {t[:8]}, rows {rows.min().item()}..{rows.max().item()} "
              f"({rows.numel()}), cols {cols.min().item()}..{cols.max().item()} ({cols.numel()}), self-diff {diff_self}")
    else:
        print(f"rep {r}: ok, self-diff {diff_self}")
print("bad tiles:", sorted(bad_tiles.items())[:20])
