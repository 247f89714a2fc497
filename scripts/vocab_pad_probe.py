#!/usr/bin/env python3
"""MLM-decoder GEMMs at vocab 30522 vs padded to a multiple of 128 (30592): forward, data-gradient
and weight-gradient shapes through kernels.gemm (tuned choices, as in a step)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_amd import kernels as K  # noqa: E402

K.tunable_setup()
T, H = 16384, 1024


def timed(fn, reps=10):
    fn()
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


for V in (30522, 30592):
    x = torch.randn(T, H, device="cuda").bfloat16()
    w = torch.randn(V, H, device="cuda").bfloat16()
    b = torch.zeros(V, device="cuda").bfloat16()
    y = torch.empty(T, V, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, V, device="cuda").bfloat16()
    dx = torch.empty(T, H, device="cuda", dtype=torch.bfloat16)
    dw = torch.zeros(V, H, device="cuda")
    f = timed(lambda: K.gemm(x, w, y, T, V, H, True, True, H, H, V, bias=b))
    d = timed(lambda: K.gemm(dy, w, dx, T, H, V, True, False, V, H, H))
    g = timed(lambda: K.gemm(dy, x, dw, V, H, T, False, False, V, H, H, beta=0.0))
    print(f"vocab {V}: fwd {f * 1e3:7.1f} us  dgrad {d * 1e3:7.1f} us  wgrad {g * 1e3:7.1f} us  total {(f + d + g) * 1e3:7.1f} us",
          flush=True)
