#!/usr/bin/env python3
"""Column-sum (bias gradient) pass microbenchmark: our bias_act_bwd(ACT_NONE) kernel (+ its
col_reduce tail) vs torch.sum(0), on the BERT-Large shapes (QKV 16384x3072, decoder 16384x30522)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_amd import kernels as K  # noqa: E402

X = K.ext()


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    en.synchronize()
    return st.elapsed_time(en) / reps


for rows, cols in [(16384, 1024), (16384, 3072), (16384, 4096), (16384, 30522)]:
    dy = torch.randn(rows, cols, device="cuda").bfloat16()
    db = torch.zeros(cols, device="cuda")
    t_ours = timeit(lambda: X.bias_act_bwd(dy, None, None, db, rows, cols, K.ACT_NONE))
    t_torch = timeit(lambda: dy.float().sum(0) if False else torch.sum(dy, 0, dtype=torch.float32))
    gb = rows * cols * 2 / 1e9
    db.zero_()
    X.bias_act_bwd(dy, None, None, db, rows, cols, K.ACT_NONE)
    err = (db - dy.float().sum(0)).abs().max().item()
    print(f"{rows}x{cols}: ours {t_ours * 1e3:.1f} us ({gb / t_ours:.2f} TB/s)  torch.sum {t_torch * 1e3:.1f} us "
          f"({gb / t_torch:.2f} TB/s)  err {err:.3g}")
