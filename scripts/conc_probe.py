#!/usr/bin/env python3
"""Do a layer's data-gradient and weight-gradient GEMMs gain from running concurrently on two HIP
streams? BERT-Large shapes (T = 16384 tokens) through kernels.gemm (same tuned kernels as a step).
Usage: python scripts/conc_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
K.tunable_setup()
T = 16384
SHAPES = [("qkv", 1024, 3072), ("out", 1024, 1024), ("ffn1", 1024, 4096), ("ffn2", 4096, 1024)]
side = torch.cuda.Stream()


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


tot_s = tot_c = 0.0
for name, kin, nout in SHAPES:
    x = torch.randn(T, kin, device=dev).bfloat16()
    w = torch.randn(nout, kin, device=dev).bfloat16()
    dy = torch.randn(T, nout, device=dev).bfloat16()
    dx = torch.empty(T, kin, device=dev, dtype=torch.bfloat16)
    dw = torch.zeros(nout, kin, device=dev)

    def dgrad():
        K.gemm(dy, w, dx, T, kin, nout, True, False, nout, kin, kin)

    def wgrad():
        K.gemm(dy, x, dw, nout, kin, T, False, False, nout, kin, kin, beta=0.0)

    def serial():
        dgrad()
        wgrad()

    def conc():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            wgrad()
        dgrad()
        cur.wait_stream(side)

    serial(), conc()  # tune outside the timed region
    td, tw, ts, tc = timed(dgrad), timed(wgrad), timed(serial), timed(conc)
    tot_s += ts
    tot_c += tc
    print(f"{name:5s} dgrad {td * 1e3:7.1f} us  wgrad {tw * 1e3:7.1f} us  serial {ts * 1e3:7.1f} us  "
          f"concurrent {tc * 1e3:7.1f} us  ({100 * (ts - tc) / ts:+.1f} %)", flush=True)
print(f"layer total serial {tot_s * 1e3:.1f} us concurrent {tot_c * 1e3:.1f} us")
