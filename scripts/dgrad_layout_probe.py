#!/usr/bin/env python3
"""BERT-Large (batch 32, seq 512) input-gradient GEMMs in the NN form (W [out, in] read
N-contiguous) against the TN form (a transposed W^T copy read K-contiguous), library and ping-pong
kernel, plus the cost of the transpose16 kernel that refreshes the copy. One process, interleaved
rounds, best of rounds.

usage: dgrad_layout_probe.py [rounds=3] [reps=20]
"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from flexflow_amd import kernels as Kn  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
T = 16384
# (name, out, in, calls per step): dx [T, in] = dy [T, out] . W [out, in]
SITES = [("qkv", 3072, 1024, 24), ("attn_out", 1024, 1024, 25), ("ffn1", 4096, 1024, 24), ("ffn2", 1024, 4096, 24),
         ("vocab", 30528, 1024, 1)]
X = Kn.ext()
Kn.tunable_setup()


def timed(fn):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


tot = {}
for name, n_out, n_in, calls in SITES:
    g = torch.Generator(device="cuda").manual_seed(0)
    dy = (torch.rand(T, n_out, device="cuda", generator=g) * 2 - 1).bfloat16()
    w = ((torch.rand(n_out, n_in, device="cuda", generator=g) * 2 - 1) / 32).bfloat16()
    wt = torch.empty(n_in, n_out, device="cuda", dtype=torch.bfloat16)
    X.transpose2d(w, wt)
    dx = torch.empty(T, n_in, device="cuda", dtype=torch.bfloat16)
    M, N, K = T, n_in, n_out

    def pp(b, b_k, ldb):
        return lambda: X.gemm(dy, b, dx, None, None, M, N, K, K, ldb, N, 0, 0, 0, 1, True, b_k, 1.0, 0.0, 10, 1,
                              None, 6)
    fns = {
        "lib_nn": lambda: Kn._lib_gemm(dy, w, dx, M, N, K, True, False, K, N, N, 1.0, 0.0, None, 1, 0, 0, 0),
        "lib_tn": lambda: Kn._lib_gemm(dy, wt, dx, M, N, K, True, True, K, K, N, 1.0, 0.0, None, 1, 0, 0, 0),
        "pp_nn": pp(w, False, N),
        "pp_tn": pp(wt, True, K),
        "transpose": lambda: X.transpose2d(w, wt),
    }
    best = {}
    for _ in range(rounds):
        for k, fn in fns.items():
            t = timed(fn)
            best[k] = min(best.get(k, t), t)
    ref = (dy.float() @ w.float())
    Kn._lib_gemm(dy, wt, dx, M, N, K, True, True, K, K, N, 1.0, 0.0, None, 1, 0, 0, 0)
    e1 = (dx.float() - ref).abs().max().item()
    pp(wt, True, K)()
    e2 = (dx.float() - ref).abs().max().item()
    fl = 2.0 * M * N * K
    gb = 4.0 * n_out * n_in / 1e9
    print(f"{name:8s} M={M} N={N} K={K} x{calls}: " + " ".join(
        f"{k}={v * 1e3:7.1f}us" + (f"({fl / v / 1e9:5.0f}TF)" if k != "transpose" else f"({gb / v * 1e3:5.0f}GB/s)")
        for k, v in best.items()) + f"  maxerr lib_tn {e1:.3g} pp_tn {e2:.3g}", flush=True)
    for k, v in best.items():
        tot[k] = tot.get(k, 0.0) + v * calls
    tot["best_nn"] = tot.get("best_nn", 0.0) + min(best["lib_nn"], best["pp_nn"]) * calls
    tot["best_tn"] = tot.get("best_tn", 0.0) + min(best["lib_tn"], best["pp_tn"]) * calls
    del dy, w, wt, dx
for k, v in tot.items():
    print(f"step total {k:9s}: {v:7.3f} ms")
