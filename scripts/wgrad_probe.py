"""Weight-gradient GEMM formulations for the BERT-Large shapes (T = 16384 tokens):
dW[N][K] (+)= dZ[T][N]^T . X[T][K].

  lib_f32       torch.mm(dZ^T, X, out_dtype=fp32)   (current library path, MN-contiguous operands)
  lib_bf16      torch.mm(dZ^T, X) with bf16 output    (a TunableOp-eligible GEMM)
  tn_gemm_only  K-contiguous operands (transposed copies made beforehand)
  transpose_copies  the two transposed copies alone
  ours_<impl>   our MFMA kernels, fp32 accumulate into dW (beta = 1), split-K picked per kernel

Run under PYTORCH_TUNABLEOP_ENABLED=1 / PYTORCH_TUNABLEOP_TUNING=1 to let TunableOp pick among
the hipBLASLt and rocBLAS solutions for the bf16-output GEMMs.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexflow_amd import kernels as K  # noqa: E402


def t_ms(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    en.synchronize()
    return st.elapsed_time(en) / reps


def ours(X, dz, x, dw, N, Kd, T, impl):
    s = X.gemm_pick_splitk(N, Kd, T, 1, impl)
    ws = torch.empty(N * Kd * s, device=dw.device, dtype=torch.float32) if s > 1 else None
    X.gemm(dz, x, dw, None, None, N, Kd, T, N, Kd, Kd, 0, 0, 0, 1, False, False, 1.0, 1.0, K.ACT_NONE, s, ws, impl)


def main():
    T = int(os.environ.get("T", "16384"))
    dev = torch.device("cuda")
    X = K.ext()
    for N, Kd in [(3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096)]:
        dz = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        x = torch.randn(T, Kd, device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(N, Kd, device=dev, dtype=torch.float32)
        wb = torch.empty(N, Kd, device=dev, dtype=torch.bfloat16)
        dzt = dz.t().contiguous()
        xt = x.t().contiguous()
        r = {"N": N, "K": Kd, "T": T}
        r["lib_f32"] = t_ms(lambda: torch.mm(dz.t(), x, out_dtype=torch.float32, out=dw))
        r["lib_bf16"] = t_ms(lambda: torch.mm(dz.t(), x, out=wb))
        r["lib_bf16_plus_add"] = t_ms(lambda: (torch.mm(dz.t(), x, out=wb), dw.add_(wb)))
        r["tn_gemm_only"] = t_ms(lambda: torch.mm(dzt, xt.t(), out=wb))
        r["transpose_copies"] = t_ms(lambda: (dzt.copy_(dz.t()), xt.copy_(x.t())))
        for S in (2, 4, 8):  # split-K over the token dim as one strided-batched library GEMM
            a3 = dz.view(S, T // S, N).transpose(1, 2)
            b3 = x.view(S, T // S, Kd)
            try:
                part = torch.empty(S, N, Kd, device=dev, dtype=torch.float32)
                r[f"bmm_split{S}_f32"] = t_ms(lambda: (torch.bmm(a3, b3, out_dtype=torch.float32, out=part),
                                                        torch.sum(part, 0, out=dw)))
            except (RuntimeError, TypeError) as e:
                r[f"bmm_split{S}_f32_err"] = str(e)[:80]
            partb = torch.empty(S, N, Kd, device=dev, dtype=torch.bfloat16)
            r[f"bmm_split{S}_bf16"] = t_ms(lambda: (torch.bmm(a3, b3, out=partb), dw.add_(partb.float().sum(0))))
        for name, impl in K.IMPLS.items():
            r["ours_" + name] = t_ms(lambda: ours(X, dz, x, dw, N, Kd, T, impl))
        ref = (dz.float().t() @ x.float())
        torch.mm(dz.t(), x, out=wb)
        r["bf16_out_rel_err"] = float((wb.float() - ref).norm() / ref.norm())
        fl = 2.0 * T * N * Kd
        best = min((v, k) for k, v in r.items() if k.startswith(("lib", "tn", "ours", "bmm")) and isinstance(v, float))
        r["best"] = best[1]
        r["best_tflops"] = round(fl / best[0] / 1e9, 1)
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
