#!/usr/bin/env python3
"""Run one GEMM configuration repeatedly (for rocprofv3 --pmc / kernel-trace of a single kernel).

usage: gemm_probe.py M N K a_k b_k [impl=w4|k256|big|128|lib] [reps=20] [out=bf16|f32]
"""
import sys
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from flexflow_amd import kernels as Kn  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
a_k, b_k = sys.argv[4] == "1", sys.argv[5] == "1"
impl = sys.argv[6] if len(sys.argv) > 6 else "big"
reps = int(sys.argv[7]) if len(sys.argv) > 7 else 20
out = sys.argv[8] if len(sys.argv) > 8 else "bf16"
dev = "cuda"
A = (torch.randn(M, K, device=dev) if a_k else torch.randn(K, M, device=dev)).bfloat16()
B = (torch.randn(N, K, device=dev) if b_k else torch.randn(K, N, device=dev)).bfloat16()
C = torch.empty(M, N, device=dev, dtype=torch.bfloat16 if out == "bf16" else torch.float32)
lda = K if a_k else M
ldb = K if b_k else N
X = Kn.ext()
IMP = {"pp": 6, "k256": 2, "big": 1, "128": 0}.get(impl, 2)
splitk = X.gemm_pick_splitk(M, N, K, 1, IMP)
ws = torch.empty(M * N * splitk, device=dev) if splitk > 1 else None
for _ in range(reps):
    if impl == "lib":
        Kn._lib_gemm(A, B, C, M, N, K, a_k, b_k, lda, ldb, N, 1.0, 0.0, None, 1, 0, 0, 0)
    else:
        X.gemm(A, B, C, None, None, M, N, K, lda, ldb, N, 0, 0, 0, 1, a_k, b_k, 1.0, 0.0, 10, splitk, ws, IMP)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    if impl == "lib":
        Kn._lib_gemm(A, B, C, M, N, K, a_k, b_k, lda, ldb, N, 1.0, 0.0, None, 1, 0, 0, 0)
    else:
        X.gemm(A, B, C, None, None, M, N, K, lda, ldb, N, 0, 0, 0, 1, a_k, b_k, 1.0, 0.0, 10, splitk, ws, IMP)
e.record()
e.synchronize()
ms = s.elapsed_time(e) / reps
print(f"{impl} M={M} N={N} K={K} a_k={a_k} b_k={b_k} splitk={splitk}: {ms:.4f} ms {2.0 * M * N * K / ms / 1e9:.1f} TFLOPS")
