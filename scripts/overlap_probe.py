#!/usr/bin/env python3
"""Can a memory-bound optimizer pass hide under compute-bound GEMMs on MI355X? Times a chain of
BERT-shaped GEMMs and a fused Adam pass over 64M parameters, serially on one stream and
concurrently on two streams. Usage: python scripts/overlap_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
K.tunable_setup()
T = 16384
x = torch.randn(T, 1024, device=dev).bfloat16()
w1 = torch.randn(4096, 1024, device=dev).bfloat16()
w2 = torch.randn(1024, 4096, device=dev).bfloat16()
h = torch.empty(T, 4096, device=dev, dtype=torch.bfloat16)
y = torch.empty(T, 1024, device=dev, dtype=torch.bfloat16)
n = 64 << 20
P = [torch.randn(n, device=dev) for _ in range(4)]
lowp = torch.empty(n, device=dev, dtype=torch.bfloat16)


def gemms(reps=12):
    for _ in range(reps):
        torch.mm(x, w1.t(), out=h)
        torch.mm(h, w2.t(), out=y)


def adam():
    K.adam_update(P[0], P[1], P[2], P[3], lowp, 1e-4, 0.9, 0.999, 0.0, 1e-8)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / reps


side = torch.cuda.Stream()


def both():
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        adam()
    gemms()
    cur.wait_stream(side)


tg = timed(gemms)
ta = timed(adam)
ts = timed(lambda: (gemms(), adam()))
tc = timed(both)
print(f"gemms {tg:.3f} ms  adam(64M) {ta:.3f} ms  serial {ts:.3f} ms  concurrent {tc:.3f} ms  "
      f"hidden {100 * (ts - tc) / ta:.0f}% of the adam pass")

# mixed read/write roofline: a plain copy (read n*4 B, write n*4 B) and a read-only reduction
dst = torch.empty_like(P[0])
tcp = timed(lambda: dst.copy_(P[0]))
trd = timed(lambda: P[0].sum())
print(f"copy {2 * n * 4 / tcp / 1e9:.2f} TB/s  read-only sum {n * 4 / trd / 1e9:.2f} TB/s  "
      f"adam {30 * n / ta / 1e9:.2f} TB/s (30 B/param)")
