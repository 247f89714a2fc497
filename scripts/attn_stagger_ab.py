#!/usr/bin/env python3
"""A/B of the attention backward's wave stagger (attn_set_stagger) at BERT-Large shape, fused QKV
layout: interleaved rounds in one process, best of rounds; outputs must be bitwise equal.
usage: attn_stagger_ab.py [B=32] [H=16] [S=512] [D=64] [rounds=5]"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from flexflow_amd import kernels as Kn  # noqa: E402

B, H, S, D = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (32, 16, 512, 64)))
rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 5
dev = "cuda"
X = Kn.ext()
qkv = torch.randn(B, S, 3, H, D, device=dev).bfloat16()
o = torch.empty(B, S, H, D, device=dev, dtype=torch.bfloat16)
do = torch.randn_like(o)
dqkv = torch.empty_like(qkv)
sq, so = (S * 3 * H * D, D, 3 * H * D), (S * H * D, D, H * D)
base, dbase = qkv.view(-1), dqkv.view(-1)
q, k, v = base, base[H * D:], base[2 * H * D:]
dq, dk, dv = dbase, dbase[H * D:], dbase[2 * H * D:]
lse = Kn.flash_attn_fwd(q, sq, k, sq, v, sq, o, so, B, H, S, S, D, D ** -0.5, False)


def bwd():
    Kn.flash_attn_bwd(q, sq, k, sq, v, sq, o, so, do, so, lse, dq, sq, dk, sq, dv, sq, B, H, S, S, D, D ** -0.5, False)


def timed(reps=20):
    bwd()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        bwd()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


res, outs = {0: [], 1: []}, {}
for _ in range(rounds):
    for st in (0, 1):
        X.attn_set_stagger(st)
        res[st].append(timed())
        outs[st] = dqkv.clone()
fl = 2.5 * 4.0 * B * H * S * S * D
for st in (0, 1):
    ms = min(res[st])
    print(f"attn bwd stagger={st}: {ms:.4f} ms {fl / ms / 1e9:.1f} TFLOPS (rounds {[round(t, 4) for t in res[st]]})")
print("bitwise equal:", torch.equal(outs[0], outs[1]))
X.attn_set_stagger(0)
