#!/usr/bin/env python3
"""Our implicit-GEMM convolution vs MIOpen (torch) on CNN-zoo layer shapes, bf16, forward and
backward (data + filter), in the layout the framework runs (channel-last unless
FF_CHANNELS_LAST=0). Usage: python scripts/conv_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_amd import kernels as K  # noqa: E402

SHAPES = [  # name, N, C, H, W, K, (kh, kw), (sh, sw), (ph, pw), groups
    ("alexnet.conv1", 64, 3, 224, 224, 64, (11, 11), (4, 4), (2, 2), 1),
    ("alexnet.conv2", 64, 64, 27, 27, 192, (5, 5), (1, 1), (2, 2), 1),
    ("alexnet.conv3", 64, 192, 13, 13, 384, (3, 3), (1, 1), (1, 1), 1),
    ("resnet.c2_3x3", 64, 64, 56, 56, 64, (3, 3), (1, 1), (1, 1), 1),
    ("resnet.c2_1x1", 64, 64, 56, 56, 256, (1, 1), (1, 1), (0, 0), 1),
    ("resnet.c4_3x3", 64, 256, 14, 14, 256, (3, 3), (1, 1), (1, 1), 1),
    ("resnet.c5_1x1", 64, 2048, 7, 7, 512, (1, 1), (1, 1), (0, 0), 1),
    ("inception.1x7", 32, 128, 17, 17, 128, (1, 7), (1, 1), (0, 3), 1),
    ("inception.A1x1", 64, 192, 35, 35, 64, (1, 1), (1, 1), (0, 0), 1),
    ("inception.A5x5", 64, 48, 35, 35, 64, (5, 5), (1, 1), (2, 2), 1),
    ("inception.A3x3", 64, 64, 35, 35, 96, (3, 3), (1, 1), (1, 1), 1),
    ("inception.stem3", 64, 32, 147, 147, 64, (3, 3), (1, 1), (1, 1), 1),
    ("inception.E1x1", 64, 1280, 8, 8, 320, (1, 1), (1, 1), (0, 0), 1),
    ("resnext.g32", 32, 256, 28, 28, 256, (3, 3), (1, 1), (1, 1), 32),
    ("resnet.c4_ds1x1s2", 64, 512, 28, 28, 1024, (1, 1), (2, 2), (0, 0), 1),
    ("resnet.c5_3x3s2", 64, 512, 14, 14, 512, (3, 3), (2, 2), (1, 1), 1),
    ("resnet.c3_3x3s2", 64, 128, 56, 56, 128, (3, 3), (2, 2), (1, 1), 1),
    ("resnet.c5_7x7_3x3", 64, 512, 7, 7, 512, (3, 3), (1, 1), (1, 1), 1),
    ("inception.B3x3s2", 64, 288, 35, 35, 384, (3, 3), (2, 2), (0, 0), 1),
    ("inception.D3x3s2", 64, 192, 17, 17, 320, (3, 3), (2, 2), (0, 0), 1),
    ("inception.7x1_192", 64, 192, 17, 17, 192, (7, 1), (1, 1), (3, 0), 1),
]


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


for name, N, C, H, W, Ko, k, st, pad, G in SHAPES:
    x = torch.randn(N, C, H, W, device="cuda").bfloat16()
    x = K.cl_dense(x, K.cl_ok(x, C // G))
    w = (torch.randn(Ko, C // G, *k, device="cuda") * 0.05).bfloat16()
    b = torch.zeros(Ko, device="cuda").bfloat16()
    g = K.conv_geometry(x, w, st, pad, G)
    fl = 2.0 * N * Ko * g[5] * g[6] * (C // G) * k[0] * k[1]
    y_cl = K.cl_ok(x, Ko // G)
    f_o = timed(lambda: K._conv_ours_fwd(x, w, b, g, True, y_cl))
    f_l = timed(lambda: K._conv_lib_fwd(x, w, b, g, True))
    dy = torch.randn(N, Ko, g[5], g[6], device="cuda").bfloat16()
    dy = K.cl_dense(dy, y_cl)
    dx = torch.empty_like(x)
    dw = torch.zeros(w.shape, device="cuda")
    b_o = timed(lambda: K._conv_ours_bwd(x, w, dy, g, dx, dw))
    b_l = timed(lambda: K._conv_lib_bwd(x, w, dy, g, True, True))
    d_o = timed(lambda: K._conv_ours_bwd(x, w, dy, g, dx, None))
    w_o = timed(lambda: K._conv_ours_bwd(x, w, dy, g, None, dw))
    print(f"{name:16s} fwd ours {f_o * 1e3:8.1f} us ({fl / f_o / 1e9:6.1f} TF) lib {f_l * 1e3:8.1f} us | "
          f"bwd ours {b_o * 1e3:8.1f} us ({2 * fl / b_o / 1e9:6.1f} TF) lib {b_l * 1e3:8.1f} us | "
          f"ours dgrad {d_o * 1e3:8.1f} us wgrad {w_o * 1e3:8.1f} us", flush=True)
