"""HIP mixture-of-experts kernels (csrc/kernels/moe.hip) against the fp32 torch formulation of the
same ops (flexflow_amd/ops/misc.py CPU path; reference src/ops/topk.cu, group_by.cu, aggregate.cu,
aggregate_spec.cu): TopK forward / backward, device routing (reference sample order, capacity drop,
out-of-range expert ids), GroupBy and Aggregate / AggregateSpec forward and backward."""
import math

import pytest
import torch

from flexflow_amd import kernels as K
from flexflow_amd.ops.misc import _expert_slots

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,n,k", [(64, 8, 2), (33, 100, 5), (7, 1000, 16)])
def test_topk(dt, rows, n, k):
    torch.manual_seed(0)
    x = torch.randn(rows, n, device=DEV).to(dt)
    v, i = K.topk(x, k)
    rv, ri = torch.topk(x.float(), k, -1, largest=True, sorted=True)
    assert torch.equal(v.float(), rv)
    # indices: they select exactly these values, once each (bf16 rounding makes ties, which torch
    # breaks in its own order; ours takes the lowest index first)
    assert torch.equal(torch.gather(x.float(), -1, i.long()), rv)
    assert all(len(set(r)) == k for r in i.tolist())
    if dt == torch.float32:
        assert torch.equal(i.long(), ri)
    dv = torch.randn(rows, k, device=DEV).to(dt)
    dx = K.topk_bwd(dv, i, x.shape)
    ref = torch.zeros(rows, n, device=DEV).scatter_add_(-1, i.long(), dv.float())
    assert torch.equal(dx.float(), ref.to(dt).float())


@pytest.mark.parametrize("B,k,n,alpha", [(64, 2, 8, 2.0), (300, 1, 5, 1.0), (1000, 2, 64, 0.5)])
def test_route_matches_reference_order(B, k, n, alpha):
    torch.manual_seed(1)
    assign = torch.randint(0, n, (B, k), device=DEV, dtype=torch.int32)
    assign[3, 0] = -1  # out-of-range ids are dropped
    assign[5, k - 1] = n + 2
    cap = int(math.ceil(alpha * k / n * B))
    e, pos, load = K.moe_route(assign, n, cap)
    re_, rpos, rvalid = _expert_slots(assign.cpu(), n, cap)
    assert torch.equal(e.cpu().long(), re_.clamp(0, n - 1))
    assert torch.equal(pos.cpu() >= 0, rvalid)
    assert torch.equal(pos.cpu().long()[rvalid], rpos[rvalid])
    assert torch.equal(load.cpu().long(), torch.bincount(re_.clamp(0, n - 1), minlength=n))


def _routing(assign, n, cap):
    e, pos, valid = _expert_slots(assign.cpu(), n, cap)
    return e.to(DEV), pos.to(DEV), valid.to(DEV)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_groupby_fwd_bwd(dt):
    torch.manual_seed(2)
    B, k, n, D, alpha = 96, 2, 6, 40, 1.0
    cap = int(math.ceil(alpha * k / n * B))
    data = torch.randn(B, D, device=DEV).to(dt)
    assign = torch.randint(0, n, (B, k), device=DEV, dtype=torch.int32)
    e, pos, _ = K.moe_route(assign, n, cap)
    outs = [torch.full((cap, D), 9.0, device=DEV, dtype=dt) for _ in range(n)]
    K.ext().groupby_fwd(data, e, pos, outs, cap, k)
    re_, rpos, rvalid = _routing(assign, n, cap)
    src = torch.arange(B * k, device=DEV) // k
    for j in range(n):
        ref = torch.zeros(cap, D, device=DEV, dtype=dt)
        m = rvalid & (re_ == j)
        ref[rpos[m]] = data[src[m]]
        assert torch.equal(outs[j], ref)
    douts = [torch.randn(cap, D, device=DEV).to(dt) for _ in range(n)]
    douts[1] = None
    dx = torch.empty(B, D, device=DEV, dtype=dt)
    K.ext().groupby_bwd(douts, e, pos, dx, cap, k)
    ref = torch.zeros(B, D, device=DEV)
    for j, d in enumerate(douts):
        if d is None:
            continue
        m = rvalid & (re_ == j)
        ref.index_add_(0, src[m], d[rpos[m]].float())
    tol = 1e-6 if dt == torch.float32 else 1e-2
    assert torch.allclose(dx.float(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("spec", [False, True])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_aggregate_fwd_bwd(spec, dt):
    torch.manual_seed(3)
    B, k, n, D, cap, lam = 80, 2, 5, 24, 30, 0.04
    gate = torch.rand(B, k, device=DEV).to(dt)
    assign = torch.randint(0, n, (B, k), device=DEV, dtype=torch.int32)
    true_assign = assign.clone()
    true_assign[::3, 0] = (true_assign[::3, 0] + 1) % n  # some rows routed wrongly
    exps = [torch.randn(cap, D, device=DEV).to(dt) for _ in range(n)]
    e, pos, load = K.moe_route(assign, n, cap)
    out = torch.empty(B, D, device=DEV, dtype=dt)
    K.ext().aggregate_fwd(None if spec else gate, exps, e, pos, out, cap, k)
    re_, rpos, rvalid = _routing(assign, n, cap)
    stacked = torch.stack([x.float() for x in exps])
    rows = stacked[re_.clamp(0, n - 1), rpos.clamp(0, cap - 1)] * rvalid[:, None]
    w = torch.ones(B * k, device=DEV) if spec else gate.float().reshape(-1)
    ref = (rows * w[:, None]).reshape(B, k, -1).sum(1)
    tol = 1e-5 if dt == torch.float32 else 2e-2
    assert torch.allclose(out.float(), ref, rtol=tol, atol=tol)
    # backward
    dout = torch.randn(B, D, device=DEV).to(dt)
    dexp = [torch.full_like(x, 5.0) for x in exps]
    dgate = None if spec else torch.empty(B, k, device=DEV, dtype=dt)
    dfull = None if spec else torch.empty(B, n, device=DEV, dtype=dt)
    K.ext().aggregate_bwd(dout, None if spec else gate, exps, dexp, e, pos, assign, true_assign, load, lam, dgate,
                          dfull, cap, k)
    dgrow = dout.float().repeat_interleave(k, 0)
    for j in range(n):
        g = torch.zeros(cap, D, device=DEV)
        m = rvalid & (re_ == j)
        g[rpos[m]] = dgrow[m] * w[m][:, None]
        assert torch.allclose(dexp[j].float(), g.to(dt).float(), rtol=tol, atol=tol)
    if not spec:
        rdg = (dgrow * rows).sum(-1).reshape(B, k)
        assert torch.allclose(dgate.float(), rdg, rtol=tol, atol=10 * tol)
        full = torch.zeros(B, n, device=DEV)
        corr = (assign == true_assign).all(-1)
        contrib = (dgrow * rows).sum(-1) * corr.repeat_interleave(k)
        full.view(-1).index_add_(0, (torch.arange(B * k, device=DEV) // k) * n + re_.clamp(0, n - 1),
                                 contrib * rvalid)
        full = full + lam * torch.bincount(re_.clamp(0, n - 1), minlength=n).float()[None, :]
        full = full - full.mean(-1, keepdim=True)
        assert torch.allclose(dfull.float(), full, rtol=tol, atol=10 * tol)


def test_moe_model_step_captures():
    """The MoE example's training step has no host synchronisation any more: it is captured into a
    hipGraph (round 3: 'operation not permitted when stream is capturing')."""
    from flexflow_amd.core import FFConfig, FFModel, SGDOptimizer
    from flexflow_amd.models import build
    cfg = FFConfig(["--hip-graphs"])
    cfg.batch_size = 64
    ff = FFModel(cfg)
    inputs, out, loss, mets, make_batch = build("moe", ff, 64, small=True)
    ff.optimizer = SGDOptimizer(ff, 0.01)
    ff.compile(loss_type=loss, metrics=mets)
    arrs, lab = make_batch(__import__("numpy").random.default_rng(0))
    for t, a in zip(inputs, arrs):
        t.set_tensor(ff, a)
    ff.label_tensor.set_tensor(ff, lab)
    for _ in range(6):
        ff.train_step()
    torch.cuda.synchronize()
    sg = ff._step_graph
    assert sg is not None and not sg.failed and sg.graph is not None
