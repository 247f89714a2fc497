#!/usr/bin/env python3
"""Every BERT-Large (batch 32, seq 512) GEMM call-site shape, our MFMA kernels against the vendor
library, timed in ONE process in interleaved rounds (best of rounds), on uniform random data.

usage: gemm_bert_probe.py [impls=k256,lib] [rounds=3] [reps=20] [filter=fwd,dgrad,wgrad]
Prints one line per (shape, impl) plus a per-orientation summary weighted by call counts.
"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from flexflow_amd import kernels as Kn  # noqa: E402

impls = (sys.argv[1] if len(sys.argv) > 1 else "k256,lib").split(",")
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
kinds = (sys.argv[4] if len(sys.argv) > 4 else "fwd,dgrad,wgrad").split(",")
T = 16384
# (kind, M, N, K, a_k, b_k, calls per step, fp32 out)
SHAPES = [
    ("fwd", T, 3072, 1024, True, True, 24, False),
    ("fwd", T, 1024, 1024, True, True, 25, False),
    ("fwd", T, 4096, 1024, True, True, 24, False),
    ("fwd", T, 1024, 4096, True, True, 24, False),
    ("fwd", T, 30528, 1024, True, True, 1, False),
    ("dgrad", T, 1024, 3072, True, False, 24, False),
    ("dgrad", T, 1024, 1024, True, False, 25, False),
    ("dgrad", T, 4096, 1024, True, False, 24, False),
    ("dgrad", T, 1024, 4096, True, False, 24, False),
    ("dgrad", T, 1024, 30528, True, False, 1, False),
    ("wgrad", 3072, 1024, T, False, False, 24, True),
    ("wgrad", 1024, 1024, T, False, False, 25, True),
    ("wgrad", 4096, 1024, T, False, False, 24, True),
    ("wgrad", 1024, 4096, T, False, False, 24, True),
    ("wgrad", 30528, 1024, T, False, False, 1, True),
]
IMP = {"pp": 6, "pp_nodma": 61, "k256": 2, "big": 1, "128": 0}
dev = "cuda"
X = Kn.ext()


def runner(impl, A, B, C, M, N, K, a_k, b_k):
    lda = K if a_k else M
    ldb = K if b_k else N
    if impl == "lib":
        return lambda: Kn._lib_gemm(A, B, C, M, N, K, a_k, b_k, lda, ldb, N, 1.0, 0.0, None, 1, 0, 0, 0)
    if impl.startswith("lib_sk"):
        return lambda: Kn._lib_gemm_splitk(A, B, C, M, N, K, a_k, b_k, lda, ldb, 0.0, int(impl[6:]))
    if "_sk" in impl:  # e.g. pp_sk4: that kernel with a fixed split-K factor
        i = IMP[impl.split("_sk")[0]]
        sk = int(impl.split("_sk")[1])
    else:
        i = IMP[impl]
        sk = X.gemm_pick_splitk(M, N, K, 1, i)
    ws = torch.empty(M * N * sk, device=dev) if sk > 1 else None
    return lambda: X.gemm(A, B, C, None, None, M, N, K, lda, ldb, N, 0, 0, 0, 1, a_k, b_k, 1.0, 0.0, 10, sk, ws, i)


def timed(fn):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


summary = {}
for kind, M, N, K, a_k, b_k, calls, f32 in SHAPES:
    if kind not in kinds:
        continue
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand((M, K) if a_k else (K, M), device=dev, generator=g) * 2 - 1).bfloat16()
    B = (torch.rand((N, K) if b_k else (K, N), device=dev, generator=g) * 2 - 1).bfloat16()
    C = torch.empty(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
    use = [im for im in impls if f32 or "_sk" not in im]  # split-K: fp32 weight gradients only
    fns = {im: runner(im, A, B, C, M, N, K, a_k, b_k) for im in use}
    best = {}
    for _ in range(rounds):
        for im, fn in fns.items():
            t = timed(fn)
            best[im] = min(best.get(im, t), t)
    fl = 2.0 * M * N * K
    line = " ".join(f"{im}={best[im] * 1e3:8.1f}us({fl / best[im] / 1e9:6.0f}TF)" for im in use)
    win = min(best, key=best.get)
    print(f"{kind:5s} M={M:5d} N={N:5d} K={K:5d} x{calls:2d}: {line}  best={win}", flush=True)
    for im in use:
        summary.setdefault((kind, im), 0.0)
        summary[(kind, im)] += best[im] * calls
    summary.setdefault((kind, "best_ours"), 0.0)
    summary[(kind, "best_ours")] += min(best[im] for im in use if not im.startswith("lib")) * calls
    summary.setdefault((kind, "best_lib"), 0.0)
    summary[(kind, "best_lib")] += min([best[im] for im in use if im.startswith("lib")] or [0.0]) * calls
    del A, B, C
for (kind, im), ms in sorted(summary.items()):
    print(f"step total {kind:5s} {im:9s}: {ms:7.3f} ms")
