#!/usr/bin/env python3
"""Quick numerics + repeatability screen of one GEMM impl (default 6: gemm_pp.hip) against fp32
torch over layouts, edge shapes, bias and output dtypes. usage: pp_check.py [impl]"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from flexflow_amd import kernels as Kn  # noqa: E402

impl = int(sys.argv[1]) if len(sys.argv) > 1 else 6
X = Kn.ext()
dev = "cuda"
bad = 0
for (M, N, K) in [(512, 512, 512), (256, 256, 64), (8192, 4096, 1024), (8200, 2056, 512), (3000, 1000, 1152),
                  (16384, 1024, 256), (2048, 768, 128), (1024, 1024, 4096)]:
    for a_k, b_k in [(True, True), (True, False), (False, True)]:
        for out in ("bf16", "f32"):
            for bias in (None, "f32", "bf16"):
                torch.manual_seed(M + N + K)
                Am = torch.randn(M, K, device=dev).bfloat16()
                Bn = torch.randn(N, K, device=dev).bfloat16()
                A = Am if a_k else Am.t().contiguous()
                B = Bn if b_k else Bn.t().contiguous()
                ref = Am.float() @ Bn.float().t()
                bv = None
                if bias:
                    bv = torch.randn(N, device=dev)
                    if bias == "bf16":
                        bv = bv.bfloat16()
                    ref = ref + bv.float()
                C = torch.full((M, N), 7.0, device=dev, dtype=torch.float32 if out == "f32" else torch.bfloat16)
                X.gemm(A, B, C, bv, None, M, N, K, A.shape[-1], B.shape[-1], N, 0, 0, 0, 1, a_k, b_k, 1.0, 0.0, 10,
                       1, None, impl)
                rel = ((C.float() - ref).norm() / ref.norm()).item()
                first = C.clone()
                same = True
                for _ in range(3):
                    C.fill_(-3.0)
                    X.gemm(A, B, C, bv, None, M, N, K, A.shape[-1], B.shape[-1], N, 0, 0, 0, 1, a_k, b_k, 1.0, 0.0, 10,
                           1, None, impl)
                    same = same and torch.equal(C, first)
                ok = rel < (1e-3 if out == "f32" else 1e-2) and same
                bad += not ok
                if not ok or (bias is None and out == "bf16"):
                    print(f"{'OK ' if ok else 'BAD'} M={M} N={N} K={K} a_k={a_k} b_k={b_k} out={out} bias={bias} "
                          f"rel={rel:.2e} repeat_equal={same}", flush=True)
print("FAILURES:", bad)
sys.exit(1 if bad else 0)
