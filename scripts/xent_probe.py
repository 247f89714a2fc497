#!/usr/bin/env python3
"""Time the fused softmax-xent kernel on the BERT-Large MLM shape (16384 x 30522 bf16)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from flexflow_amd import _C as ffC  # noqa: E402

rows, cols = (int(v) for v in sys.argv[1:3]) if len(sys.argv) > 2 else (16384, 30522)
x = torch.randn(rows, cols, device="cuda").bfloat16()
labels = torch.randint(0, cols, (rows,), device="cuda", dtype=torch.int32)
loss = torch.empty(rows, device="cuda")
dl = torch.empty_like(x)
acc3 = torch.zeros(3, device="cuda")
for _ in range(3):
    ffC.softmax_xent(x, labels, loss, dl, rows, cols, 1.0 / rows, acc3)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20):
    ffC.softmax_xent(x, labels, loss, dl, rows, cols, 1.0 / rows, acc3)
e.record()
e.synchronize()
ms = s.elapsed_time(e) / 20
print(f"softmax_xent {rows}x{cols}: {ms * 1e3:.1f} us  {2 * rows * cols * 2 / ms / 1e9:.2f} TB/s (2 x logits bytes)")
