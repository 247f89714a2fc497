#!/usr/bin/env python3
"""Weight-gradient GEMM variants on the library path: dW[N,K] (+)= dY^T X with dY [T,N], X [T,K]."""
import json
import torch

def t(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record(); e.synchronize()
    return s.elapsed_time(e) / reps

T = 8192
for N, K in ((1024, 3072 // 3 * 3), (3072, 1024), (4096, 1024), (1024, 4096), (1024, 1024)):
    dy = torch.randn(T, N, device="cuda").bfloat16()
    x = torch.randn(T, K, device="cuda").bfloat16()
    dw = torch.zeros(N, K, device="cuda")
    dwt = torch.zeros(K, N, device="cuda")
    dwb = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
    r = {"N": N, "K": K, "T": T}
    r["mm_f32_out"] = t(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=dw))
    r["mm_f32_swapped"] = t(lambda: torch.mm(x.t(), dy, out_dtype=torch.float32, out=dwt))
    r["mm_bf16_out"] = t(lambda: torch.mm(dy.t(), x, out=dwb))
    r["mm_bf16_swapped"] = t(lambda: torch.mm(x.t(), dy))
    try:
        r["addmm_f32_inplace"] = t(lambda: torch.addmm(dw, dy.t(), x, out_dtype=torch.float32, out=dw))
    except Exception as ex:  # noqa: BLE001
        r["addmm_f32_inplace"] = str(ex)[:80]
    fl = 2.0 * T * N * K
    r["best_tflops"] = round(fl / min(v for v in r.values() if isinstance(v, float)) / 1e9, 1)
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
