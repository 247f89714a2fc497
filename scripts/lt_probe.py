#!/usr/bin/env python3
"""hipBLASLt epilogue probe (GPU): numerics of the fused epilogues against an fp32 reference, and
timing of every candidate algorithm against the unfused path (library GEMM + our elementwise
pass) on the BERT-Large shapes. Usage: python scripts/lt_probe.py [T] [all]"""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flexflow_amd import kernels as K  # noqa: E402

X = K.ext()
dev = torch.device("cuda")
T = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
ALL = len(sys.argv) > 2 and sys.argv[2] == "all"
WS = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
EPI = dict(none=0, bias=1, gelu_aux_bias=2, dgelu_bgrad=3, bgradb=4, relu_bias=5, gelu_bias=6, dgelu=7, gelu_aux=9)


def gelu_tanh(z):
    return 0.5 * z * (1 + torch.tanh(0.7978845608028654 * (z + 0.044715 * z ** 3)))


def gelu_tanh_grad(z):
    u = 0.7978845608028654 * (z + 0.044715 * z ** 3)
    t = torch.tanh(u)
    return 0.5 * (1 + t) + 0.5 * z * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * z * z)


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


def plan(M, N, Kd, a_k, b_k, epi, out_f32=False, bias_f32=False, beta_nz=False, bias=None, aux=None):
    lda = Kd if a_k else M
    ldb = Kd if b_k else N
    pid, n = X.lt_plan(M, N, Kd, lda, ldb, N, 1, 0, 0, 0, a_k, b_k, out_f32, bias_f32, beta_nz, EPI[epi], N,
                       256 if ALL else 24, ALL, WS.numel(), bias, aux)
    return pid, n


def best(pid, n, A, B, C, bias, aux, beta=0.0):
    res = []
    for a in range(n):
        try:
            st = X.lt_run(pid, a, A, B, C, bias, aux, 1.0, beta, WS)
            if st != 0:
                continue
            res.append((timeit(lambda: X.lt_run(pid, a, A, B, C, bias, aux, 1.0, beta, WS), 10), a))
        except RuntimeError as e:
            print("  algo", a, "failed", e)
    res.sort()
    return res


torch.manual_seed(0)
SHAPES = [(4096, 1024, "ffn1"), (1024, 4096, "ffn2"), (3072, 1024, "qkv"), (1024, 1024, "proj")]
if ALL:
    SHAPES = SHAPES[:2]
for (N, Kd, name) in SHAPES:
    M = T
    x = (torch.randn(M, Kd, device=dev) * 0.5).bfloat16()
    w = (torch.randn(N, Kd, device=dev) / math.sqrt(Kd)).bfloat16()
    b = (torch.randn(N, device=dev) * 0.1).bfloat16()
    fl = 2.0 * M * N * Kd
    # ---- forward: plain, bias, gelu_aux_bias
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    z = torch.empty_like(y)
    K.tunable_setup()
    t_mm = timeit(lambda: torch.mm(x, w.t(), out=y))
    t_addmm = timeit(lambda: torch.addmm(b, x, w.t(), out=y))
    print(f"[{name}] M={M} N={N} K={Kd}: torch.mm {t_mm:.4f} ms ({fl / t_mm / 1e9:.0f} TF)  addmm {t_addmm:.4f}")
    for epi in (("none", "bias", "gelu_aux_bias", "gelu_bias", "gelu_aux") if ALL else ("none", "bias", "gelu_aux_bias", "gelu_bias", "relu_bias", "gelu_aux")):
        bb, zz = (b if "bias" in epi else None), (z if "aux" in epi else None)
        pid, n = plan(M, N, Kd, True, True, epi, bias=bb, aux=zz)
        r = best(pid, n, x, w, y, bb, zz)
        if not r:
            print(f"  lt {epi}: no algorithm ({n} candidates)")
            continue
        t, a = r[0]
        print(f"  lt {epi}: best {t:.4f} ms ({fl / t / 1e9:.0f} TF) of {n} cands [{X.lt_algo_name(pid, a)[:70]}]"
              f" sol={X.lt_algo_index(pid, a)}; heuristic#0 {[tt for tt, aa in r if aa == 0][:1]}")
        if epi == "gelu_aux_bias":
            X.lt_run(pid, a, x, w, y, b, z, 1.0, 0.0, WS)
            zr = x.float() @ w.float().t() + b.float()
            yr = gelu_tanh(zr)
            print(f"    numerics: |z-zr| max {(z.float() - zr).abs().max().item():.4f}  |y-gelu_tanh| max "
                  f"{(y.float() - yr).abs().max().item():.4f}  vs erf-gelu "
                  f"{(y.float() - torch.nn.functional.gelu(zr)).abs().max().item():.4f}")
    if name == "ffn1":
        # unfused reference path: library GEMM + our activation pass
        t_un = timeit(lambda: (torch.addmm(b, x, w.t(), out=z), X.bias_act_fwd(z, None, None, y, M, N, K.ACT_GELU)))
        print(f"  unfused addmm + bias_act_fwd: {t_un:.4f} ms")
    # ---- backward dgrad with dGELU + bias grad: dh[M, Kd] = dy[M, N] . W[N, Kd] -> dz = dh * gelu'(zin)
    if name == "ffn2":
        # here: the FFN2 layer has input width Kd=4096; its dgrad produces dz of FFN1 (width 4096)
        dy = (torch.randn(M, N, device=dev) * 0.1).bfloat16()
        zin = (torch.randn(M, Kd, device=dev)).bfloat16()
        dz = torch.empty(M, Kd, device=dev, dtype=torch.bfloat16)
        db = torch.zeros(Kd, device=dev, dtype=torch.float32)
        fl2 = 2.0 * M * N * Kd
        t_dmm = timeit(lambda: torch.mm(dy, w, out=dz))
        dh = torch.empty_like(dz)
        t_un = timeit(lambda: (torch.mm(dy, w, out=dh), X.bias_act_bwd(dh, zin, dz, db, M, Kd, K.ACT_GELU)))
        print(f"  dgrad torch.mm {t_dmm:.4f} ms ({fl2 / t_dmm / 1e9:.0f} TF); unfused mm + bias_act_bwd {t_un:.4f}")
        for bf32 in (True, False):
            dbb = db if bf32 else torch.zeros(Kd, device=dev, dtype=torch.bfloat16)
            pid, n = plan(M, Kd, N, True, False, "dgelu_bgrad", bias_f32=bf32, bias=dbb, aux=zin)
            r = best(pid, n, dy, w, dz, dbb, zin)
            if not r:
                print(f"  lt dgelu_bgrad(bias_f32={bf32}): no algorithm ({n} candidates)")
                continue
            t, a = r[0]
            X.lt_run(pid, a, dy, w, dz, dbb, zin, 1.0, 0.0, WS)
            dhr = dy.float() @ w.float()
            dzr = dhr * gelu_tanh_grad(zin.float())
            print(f"  lt dgelu_bgrad(bias_f32={bf32}): best {t:.4f} ms of {n} [{X.lt_algo_name(pid, a)[:70]}] "
                  f"|dz-ref| max {(dz.float() - dzr).abs().max().item():.4f} (ref max {dzr.abs().max().item():.3f}) "
                  f"|db-ref| max {(dbb.float() - dzr.sum(0)).abs().max().item():.4f} (ref max "
                  f"{dzr.sum(0).abs().max().item():.2f})")
    torch.cuda.synchronize()
print("done")
