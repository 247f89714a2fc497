#!/usr/bin/env python3
"""Micro-benchmark of flexflow_amd HIP kernels vs the PyTorch-ROCm library path on BERT-Large shapes.

Interleaves variants in one process (cdna_hip_programming.md §5.4 rule 24) on random data
(rule 25) and prints one JSON line per case.
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexflow_amd import _C  # noqa: E402


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    st = torch.cuda.Event(enable_timing=True)
    en = torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(3):
        st.record()
        for _ in range(iters):
            fn()
        en.record()
        torch.cuda.synchronize()
        ts.append(st.elapsed_time(en) / iters)
    return min(ts)


def gemm_case(M, N, K, a_k, b_k, out_f32=False, act=10, splitk=1):
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16() if a_k else (torch.rand(K, M, device="cuda") * 2 - 1).bfloat16()
    B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16() if b_k else (torch.rand(K, N, device="cuda") * 2 - 1).bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.float32 if out_f32 else torch.bfloat16)
    ws = torch.empty(max(1, M * N * splitk), device="cuda") if splitk > 1 else None
    lda, ldb = A.shape[1], B.shape[1]

    def mine():
        _C.gemm(A, B, C, None, None, M, N, K, lda, ldb, N, 0, 0, 0, 1, a_k, b_k, 1.0, 0.0, act, splitk, ws, True)

    def mine128():
        _C.gemm(A, B, C, None, None, M, N, K, lda, ldb, N, 0, 0, 0, 1, a_k, b_k, 1.0, 0.0, act, splitk, ws, False)

    At = A if a_k else A.t()
    Bt = B.t() if b_k else B

    def lib():
        torch.matmul(At, Bt)

    t_m = timeit(mine)
    t_s = timeit(mine128)
    t_l = timeit(lib)
    fl = 2.0 * M * N * K
    return {"op": "gemm", "M": M, "N": N, "K": K, "a_k": a_k, "b_k": b_k, "splitk": splitk,
            "ours_ms": round(t_m, 4), "lib_ms": round(t_l, 4), "ours_tflops": round(fl / t_m / 1e9, 1),
            "ours128_tflops": round(fl / t_s / 1e9, 1), "lib_tflops": round(fl / t_l / 1e9, 1)}


def attn_case(B, H, S, D):
    q = torch.randn(B, H, S, D, device="cuda").bfloat16()
    k = torch.randn_like(q)
    v = torch.randn_like(q)
    o = torch.empty_like(q)
    lse = torch.empty(B * H * S, device="cuda")
    st = [H * S * D, S * D, D]
    sc = 1 / math.sqrt(D)

    def mine():
        _C.attn_fwd(q, st, k, st, v, st, o, st, lse, B, H, S, S, D, sc, False)

    def lib():
        torch.nn.functional.scaled_dot_product_attention(q, k, v)

    do = torch.randn_like(q)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
    ws = torch.empty(_C.attn_bwd_ws(B, H, S, S, D), device="cuda")
    mine()

    def mine_b():
        _C.attn_bwd(q, st, k, st, v, st, o, st, do, st, lse, dq, st, dk, st, dv, st, ws, B, H, S, S, D, sc, False)

    qr, kr, vr = (t.clone().requires_grad_() for t in (q, k, v))
    out = torch.nn.functional.scaled_dot_product_attention(qr, kr, vr)

    def lib_b():
        torch.autograd.grad(out, (qr, kr, vr), do, retain_graph=True)

    fl = 4.0 * B * H * S * S * D
    t_m, t_l = timeit(mine), timeit(lib)
    t_mb, t_lb = timeit(mine_b), timeit(lib_b)
    return {"op": "attn", "B": B, "H": H, "S": S, "D": D, "fwd_ours_ms": round(t_m, 4), "fwd_lib_ms": round(t_l, 4),
            "fwd_ours_tflops": round(fl / t_m / 1e9, 1), "fwd_lib_tflops": round(fl / t_l / 1e9, 1),
            "bwd_ours_ms": round(t_mb, 4), "bwd_lib_ms": round(t_lb, 4),
            "bwd_ours_tflops": round(2.5 * fl / t_mb / 1e9, 1), "bwd_lib_tflops": round(2.5 * fl / t_lb / 1e9, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    T = a.tokens
    cases = [
        (T, 3072, 1024, True, True), (T, 1024, 1024, True, True), (T, 4096, 1024, True, True),
        (T, 1024, 4096, True, True),
        (T, 1024, 3072, True, False), (T, 1024, 4096, True, False), (T, 4096, 1024, True, False),
        (3072, 1024, T, False, False), (4096, 1024, T, False, False), (1024, 4096, T, False, False),
        (4096, 4096, 4096, True, True), (8192, 8192, 8192, True, True),
    ]
    if a.quick:
        cases = cases[:3]
    for c in cases:
        print(json.dumps(gemm_case(*c)), flush=True)
    for c in [(3072, 1024, T, False, False), (1024, 1024, T, False, False), (4096, 1024, T, False, False)]:
        sk = _C.gemm_pick_splitk(c[0], c[1], c[2], 1)
        print(json.dumps(gemm_case(*c, splitk=max(sk, 2))), flush=True)
    print(json.dumps(attn_case(T // 512, 16, 512, 64)), flush=True)
    if not a.quick:
        print(json.dumps(attn_case(4, 16, 2048, 64)), flush=True)
        print(json.dumps(attn_case(4, 16, 2048, 128)), flush=True)


if __name__ == "__main__":
    main()
