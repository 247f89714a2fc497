#!/usr/bin/env python3
"""FFN2 dgrad of BERT-Large (16384 x 4096 x 1024, NN) fused with FFN1's activation backward:
persistent ping-pong kernel multiplying a stored act' (pp), the 256-row kernel evaluating GELU'
(k256, act 14), and the library GEMM + bias_act_bwd pass (lib+pass, act 14 and stored act' 15).
Interleaved rounds, best of rounds, uniform random data."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from flexflow_amd import kernels as Kn  # noqa: E402

X = Kn.ext()
Kn.tunable_setup()
dev = "cuda"
M, N, K = 16384, 4096, 1024
dy = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
w = (torch.rand(K, N, device=dev) * 2 - 1).bfloat16()
z = torch.randn(M, N, device=dev).bfloat16()
g = torch.rand(M, N, device=dev).bfloat16()
C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
db = torch.zeros(N, device=dev)


def lib_pass(act, zz):
    Kn._lib_gemm(dy, w, C, M, N, K, True, False, K, N, N, 1.0, 0.0, None, 1, 0, 0, 0)
    X.bias_act_bwd(C, zz, C, db, M, N, act)


fns = {
    "pp(g)": lambda: X.gemm_dact(dy, w, C, g, db, M, N, K, K, N, N, True, False, 15, 6),
    "pp(g) no db": lambda: X.gemm_dact(dy, w, C, g, None, M, N, K, K, N, N, True, False, 15, 6),
    "k256(gelu)": lambda: X.gemm_dact(dy, w, C, z, db, M, N, K, K, N, N, True, False, 14, 2),
    "lib+pass(gelu)": lambda: lib_pass(14, z),
    "lib+pass(g)": lambda: lib_pass(15, g),
    "pp plain": lambda: X.gemm(dy, w, C, None, None, M, N, K, K, N, N, 0, 0, 0, 1, True, False, 1.0, 0.0, 10, 1, None, 6),
    "lib plain": lambda: Kn._lib_gemm(dy, w, C, M, N, K, True, False, K, N, N, 1.0, 0.0, None, 1, 0, 0, 0),
}


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


best = {}
for _ in range(3):
    for k, f in fns.items():
        t = timed(f)
        best[k] = min(best.get(k, t), t)
for k, t in best.items():
    print(f"{k:16s} {t * 1e3:8.1f} us", flush=True)
