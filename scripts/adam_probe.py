"""Fused Adam bandwidth probe: one update of an N-parameter arena (fp32 master / grad / m / v and
the bf16 compute copy, 30 B moved per parameter), timed over repeated launches on one GPU.
Variants measured in round 3 (non-temporal streams, two groups per lane) were within box-to-box
noise of the plain kernel: profiles/adam_probe_r3.txt.

    python scripts/adam_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexflow_amd import kernels as K  # noqa: E402


def main():
    n = int(os.environ.get("ADAM_N", 335_000_000))
    dev = torch.device("cuda:0")
    w = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev) * 1e-3
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    lowp = torch.empty(n, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        K.adam_update(w, g, m, v, lowp, 1e-4, 0.9, 0.999, 0.0, 1e-8)
    torch.cuda.synchronize()
    reps = 20
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    best = 1e9
    for _ in range(3):
        ev[0].record()
        for _ in range(reps):
            K.adam_update(w, g, m, v, lowp, 1e-4, 0.9, 0.999, 0.0, 1e-8)
        ev[1].record()
        torch.cuda.synchronize()
        best = min(best, ev[0].elapsed_time(ev[1]) / reps)
    print("adam n=%d: %.3f ms/update, %.2f TB/s" % (n, best, 30.0 * n / best / 1e9))


if __name__ == "__main__":
    main()
