#!/usr/bin/env python3
"""Run flash attention fwd+bwd repeatedly on one shape (for rocprofv3 --pmc / --kernel-trace).
usage: attn_probe.py B H S D [reps]"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from flexflow_amd import kernels as Kn  # noqa: E402

B, H, S, D = (int(v) for v in sys.argv[1:5])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 10
dev = "cuda"
qkv = torch.randn(B, S, 3, H, D, device=dev).bfloat16()
o = torch.empty(B, S, H, D, device=dev, dtype=torch.bfloat16)
do = torch.randn_like(o)
dqkv = torch.empty_like(qkv)
sq = (S * 3 * H * D, D, 3 * H * D)  # (b, h, s) strides of q/k/v inside qkv
so = (S * H * D, D, H * D)
base, dbase = qkv.view(-1), dqkv.view(-1)
q, k, v = base, base[H * D:], base[2 * H * D:]
dq, dk, dv = dbase, dbase[H * D:], dbase[2 * H * D:]
scale = D ** -0.5
X = Kn.ext()


def timed(fn):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


fl_f = 4.0 * B * H * S * S * D
# forward structures (0: registers, 1: LDS-DMA, 3: 64 rows/wave), interleaved
default_fwd = X.attn_fwd_variant()
FV = (0, 1, 3)
fres, fouts = {v: [] for v in FV}, {}
for rnd in range(3):
    for var in FV:
        X.attn_set_fwd_variant(var)
        lse = Kn.flash_attn_fwd(q, sq, k, sq, v, sq, o, so, B, H, S, S, D, scale, False)
        fouts[var] = (o.clone(), lse.clone())
        fres[var].append(timed(lambda: Kn.flash_attn_fwd(q, sq, k, sq, v, sq, o, so, B, H, S, S, D, scale, False)))
for var in FV:
    ms = min(fres[var])
    print(f"attn fwd variant {var} B={B} H={H} S={S} D={D}: {ms:.4f} ms {fl_f / ms / 1e9:.1f} TFLOPS "
          f"(rounds {[round(t, 4) for t in fres[var]]})")
print("fwd variants identical: " + str(all(torch.equal(fouts[0][0], fouts[v][0]) and torch.equal(fouts[0][1], fouts[v][1])
                                           for v in FV[1:])))
X.attn_set_fwd_variant(default_fwd)
# deferred-max threshold A/B (0 = textbook rescale on every max increase; default 8)
default_thr = X.attn_rescale_thr()
tres, touts = {0.0: [], default_thr: []}, {}
for rnd in range(3):
    for thr in tres:
        X.attn_set_rescale_thr(thr)
        Kn.flash_attn_fwd(q, sq, k, sq, v, sq, o, so, B, H, S, S, D, scale, False)
        touts[thr] = o.clone()
        tres[thr].append(timed(lambda: Kn.flash_attn_fwd(q, sq, k, sq, v, sq, o, so, B, H, S, S, D, scale, False)))
for thr in tres:
    ms = min(tres[thr])
    print(f"attn fwd rescale_thr {thr}: {ms:.4f} ms {fl_f / ms / 1e9:.1f} TFLOPS (rounds {[round(t, 4) for t in tres[thr]]})")
print(f"max |thr0 - thr{default_thr}|: {(touts[0.0].float() - touts[default_thr].float()).abs().max().item():.4g}")
X.attn_set_rescale_thr(default_thr)
lse = Kn.flash_attn_fwd(q, sq, k, sq, v, sq, o, so, B, H, S, S, D, scale, False)
# backward variants A/B'd in this one process, interleaved rounds (guide rule 24)
default_variant = X.attn_bwd_variant()
BV = tuple(int(x) for x in (sys.argv[6].split(',') if len(sys.argv) > 6 else '2,10'.split(',')))
res = {v: [] for v in BV}
outs = {}
for rnd in range(3):
    for var in BV:
        X.attn_set_bwd_variant(var)
        res[var].append(timed(lambda: Kn.flash_attn_bwd(q, sq, k, sq, v, sq, o, so, do, so, lse, dq, sq, dk, sq,
                                                        dv, sq, B, H, S, S, D, scale, False)))
        outs[var] = dqkv.clone()
fl_b = 2.5 * fl_f
for var in BV:
    ms = min(res[var])
    print(f"attn bwd variant {var}: {ms:.3f} ms {fl_b / ms / 1e9:.1f} TFLOPS  (rounds {[round(t, 3) for t in res[var]]})")
for var in BV[1:]:
    d = (outs[BV[0]].float() - outs[var].float()).abs().max().item()
    print(f"max |variant{BV[0]} - variant{var}| over dq/dk/dv: {d:.4g}")
X.attn_set_bwd_variant(default_variant)
