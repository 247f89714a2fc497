"""Where does the ping-pong GEMM's fused dgrad epilogue (ACT_GRADMUL) differ from fp32 torch?
Prints the relative error per 128-row x 64-column block class and against the impl-2 kernel."""
import sys

import torch

sys.path.insert(0, ".")
from flexflow_amd import _C as C  # noqa: E402


def run(M, N, K, a_k, b_k, impl, act=15):
    torch.manual_seed(9)
    Am = torch.randn(M, K, device="cuda").bfloat16()
    Bn = torch.randn(N, K, device="cuda").bfloat16()
    A = Am if a_k else Am.t().contiguous()
    B = Bn if b_k else Bn.t().contiguous()
    g = torch.rand(M, N, device="cuda").bfloat16() * 1.2 - 0.1
    from flexflow_amd.kernels import act_grad_ref
    ref = (Am.float() @ Bn.float().t()).bfloat16().float() * act_grad_ref(g.float(), act)
    out = torch.full((M, N), 7.0, device="cuda", dtype=torch.bfloat16)
    db = torch.zeros(N, device="cuda")
    ok = C.gemm_dact(A, B, out, g, db, M, N, K, A.shape[-1], B.shape[-1], N, a_k, b_k, act, impl)
    torch.cuda.synchronize()
    d = (out.float() - ref).abs()
    nan = torch.isnan(out.float())
    if nan.any():
        r, c = nan.nonzero(as_tuple=True)
        print(f"  NaN count {int(nan.sum())}: rows%256 {sorted(set((r % 256).tolist()))[:40]} "
              f"cols%256 {sorted(set((c % 256).tolist()))[:40]} row tiles {sorted(set((r // 256).tolist()))}")
    rel = (d.norm() / ref.norm()).item()
    print(f"act={act} impl={impl} M={M} N={N} K={K} a_k={a_k} b_k={b_k} ok={ok} rel={rel:.3e} "
          f"db_rel={((db - ref.sum(0)).norm() / ref.sum(0).norm()).item():.3e}")
    if rel > 1e-2:
        bad = (d > 0.05 * ref.abs().clamp_min(0.5)).float()
        rows = bad.mean(1)
        cols = bad.mean(0)
        print("  bad frac by row%256 (16-row groups):", [round(rows[r::256].mean().item(), 2) for r in range(0, 256, 16)])
        print("  bad frac by col%256 (16-col groups):", [round(cols[c::256].mean().item(), 2) for c in range(0, 256, 16)])
        print("  bad frac by row-tile:", [round(rows[i:i + 256].mean().item(), 2) for i in range(0, M, 256)][:8])
        print("  sample out/ref:", out[0, :8].tolist(), ref[0, :8].tolist())
        print("  out==7 frac:", (out == 7.0).float().mean().item())


for shp in [(512, 1024, 256), (1000, 4096, 1024)]:
    for a_k, b_k in [(True, False)]:
        for impl in (2, 6):
            for act in ((15, 14) if impl == 2 else (15,)):
                run(*shp, a_k, b_k, impl, act)
