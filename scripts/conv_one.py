#!/usr/bin/env python3
"""Run one convolution's forward / backward-data / backward-filter (ours) repeatedly, for
rocprofv3 --pmc / --kernel-trace. usage: conv_one.py N C H W K kh kw s p [reps] [fwd|dgrad|wgrad]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_amd import kernels as K  # noqa: E402

N, C, H, W, Ko, kh, kw, s, p = (int(v) for v in sys.argv[1:10])
reps = int(sys.argv[10]) if len(sys.argv) > 10 else 20
what = sys.argv[11] if len(sys.argv) > 11 else "wgrad"
x = K.cl_dense(torch.randn(N, C, H, W, device="cuda").bfloat16(), True)
w = (torch.randn(Ko, C, kh, kw, device="cuda") * 0.05).bfloat16()
g = K.conv_geometry(x, w, (s, s), (p, p), 1)
dy = K.cl_dense(torch.randn(N, Ko, g[5], g[6], device="cuda").bfloat16(), True)
dx = torch.empty_like(x)
dw = torch.zeros(w.shape, device="cuda")
b = torch.zeros(Ko, device="cuda").bfloat16()
fn = {"fwd": lambda: K._conv_ours_fwd(x, w, b, g, False, True),
      "dgrad": lambda: K._conv_ours_bwd(x, w, dy, g, dx, None),
      "wgrad": lambda: K._conv_ours_bwd(x, w, dy, g, None, dw)}[what]
for _ in range(reps):
    fn()
torch.cuda.synchronize()
print("ok", what, g)
