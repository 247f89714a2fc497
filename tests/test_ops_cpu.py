"""Op-level numerics on CPU: every op's explicit forward/backward against torch autograd (fp32).

Mirrors the reference's tests/align strategy (align_test.py compares each FlexFlow op's output
and gradients with PyTorch), with the PyTorch side computed here rather than from stored files.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from flexflow_amd.core import *  # noqa: F401,F403
from flexflow_amd.ops import OpCtx


def run_layer(build, inputs, seed=0, int_inputs=()):
    torch.manual_seed(seed)
    ff = FFModel(FFConfig([]))
    ts = []
    for i, x in enumerate(inputs):
        dt = DataType.DT_INT32 if i in int_inputs else DataType.DT_FLOAT
        ts.append(ff.create_tensor(list(x.shape), dt))
    out = build(ff, ts)
    outs = out if isinstance(out, list) else [out]
    L = outs[0].owner_layer
    n = len(L.impl.axis_sizes())
    ctx = OpCtx(layer=L, part_coords=(0,) * n, degrees=(1,) * n)
    ws = [torch.randn(w.dims) * 0.3 for w in L.weights]
    ctx.wgrads = [torch.zeros(w.dims) for w in L.weights]
    clones = [x.clone() for x in inputs]
    slot = [next(i for i, t in enumerate(ts) if t is u) for u in L.inputs]
    xs = [clones[i] for i in slot]
    ys = L.impl.forward(ctx, xs, ws)
    dys = [torch.randn(y.shape) if y.is_floating_point() else None for y in ys]
    dslot = L.impl.backward(ctx, dys)
    dxs = [None] * len(inputs)
    for i, d in zip(slot, dslot):
        if d is not None:
            dxs[i] = d if dxs[i] is None else dxs[i] + d
    return L, clones, ws, ys, dys, dxs, ctx.wgrads


def ref_grads(fn, inputs, ws, dys, int_inputs=()):
    xi = [x.clone().requires_grad_(i not in int_inputs and x.is_floating_point()) for i, x in enumerate(inputs)]
    wi = [w.clone().requires_grad_() for w in ws]
    out = fn(xi, wi)
    outs = out if isinstance(out, (list, tuple)) else [out]
    loss = sum((o.float() * d).sum() for o, d in zip(outs, dys) if d is not None)
    req = [t for t in xi + wi if t.requires_grad]
    gs = torch.autograd.grad(loss, req, allow_unused=True)
    it = iter(gs)
    gx = [next(it) if t.requires_grad else None for t in xi]
    gw = [next(it) for _ in wi]
    return outs, gx, gw


def close(a, b, tol=1e-4):
    if a is None or b is None:
        return
    a, b = torch.as_tensor(a).float(), torch.as_tensor(b).float()
    assert a.shape == b.shape, (a.shape, b.shape)
    err = (a - b).abs().max().item()
    scale = max(1.0, b.abs().max().item())
    assert err <= tol * scale, f"max err {err} (scale {scale})"


def check(build, fn, inputs, int_inputs=(), tol=1e-4):
    L, xs, ws, ys, dys, dxs, wg = run_layer(build, inputs, int_inputs=int_inputs)
    outs, gx, gw = ref_grads(fn, inputs, ws, dys, int_inputs)
    for y, o in zip(ys, outs):
        close(y, o, tol)
    for d, g in zip(dxs, gx):
        if d is not None and g is not None:
            close(d, g, tol)
    for d, g in zip(wg, gw):
        close(d, g, tol)
    return L


@pytest.mark.parametrize("act", [ActiMode.AC_MODE_NONE, ActiMode.AC_MODE_RELU, ActiMode.AC_MODE_GELU,
                                 ActiMode.AC_MODE_TANH, ActiMode.AC_MODE_SIGMOID])
def test_linear(act):
    x = torch.randn(4, 5, 12)
    acts = {ActiMode.AC_MODE_NONE: lambda z: z, ActiMode.AC_MODE_RELU: torch.relu, ActiMode.AC_MODE_GELU: F.gelu,
            ActiMode.AC_MODE_TANH: torch.tanh, ActiMode.AC_MODE_SIGMOID: torch.sigmoid}
    check(lambda ff, t: ff.dense(t[0], 7, act), lambda x, w: acts[act](x[0] @ w[0].t() + w[1]), [x])


def test_conv_pool_bn():
    x = torch.randn(2, 3, 9, 9)
    check(lambda ff, t: ff.conv2d(t[0], 4, 3, 3, 2, 2, 1, 1, ActiMode.AC_MODE_RELU),
          lambda x, w: torch.relu(F.conv2d(x[0], w[0], w[1], 2, 1)), [x])
    check(lambda ff, t: ff.pool2d(t[0], 3, 3, 2, 2, 1, 1),
          lambda x, w: F.max_pool2d(F.pad(x[0], (1, 1, 1, 1), value=float("-inf")), 3, 2), [x])
    check(lambda ff, t: ff.pool2d(t[0], 2, 2, 2, 2, 0, 0, PoolType.POOL_AVG),
          lambda x, w: F.avg_pool2d(x[0], 2, 2), [x])
    check(lambda ff, t: ff.batch_norm(t[0], relu=False),
          lambda x, w: F.batch_norm(x[0], None, None, w[0], w[1], training=True), [x], tol=1e-3)


def test_layernorm_softmax():
    x = torch.randn(3, 6, 16)
    check(lambda ff, t: ff.layer_norm(t[0], [-1]),
          lambda x, w: F.layer_norm(x[0], (16,), w[0], w[1]), [x])
    check(lambda ff, t: ff.softmax(t[0], -1), lambda x, w: torch.softmax(x[0], -1), [x])
    check(lambda ff, t: ff.softmax(t[0], 1), lambda x, w: torch.softmax(x[0], 1), [x])


def test_embedding():
    idx = torch.randint(0, 20, (4, 6), dtype=torch.int32)
    check(lambda ff, t: ff.embedding(t[0], 20, 8, AggrMode.AGGR_MODE_NONE),
          lambda x, w: w[0][x[0].long()], [idx], int_inputs=(0,))
    check(lambda ff, t: ff.embedding(t[0], 20, 8, AggrMode.AGGR_MODE_SUM),
          lambda x, w: w[0][x[0].long()].sum(1), [idx], int_inputs=(0,))
    check(lambda ff, t: ff.embedding(t[0], 20, 8, AggrMode.AGGR_MODE_AVG),
          lambda x, w: w[0][x[0].long()].mean(1), [idx], int_inputs=(0,))


def _mha_ref(q, k, v, wqkv, bqkv, wo, bo, H, causal=False):
    B, S, E = q.shape
    D = wqkv.shape[2]
    W = wqkv.reshape(3, H * D, E)
    bb = bqkv.reshape(3, H * D)
    qq = (q @ W[0].t() + bb[0]).view(B, S, H, D).transpose(1, 2)
    kk = (k @ W[1].t() + bb[1]).view(B, S, H, D).transpose(1, 2)
    vv = (v @ W[2].t() + bb[2]).view(B, S, H, D).transpose(1, 2)
    s = qq @ kk.transpose(-1, -2) / math.sqrt(D)
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool).triu(1), float("-inf"))
    o = (torch.softmax(s, -1) @ vv).transpose(1, 2).reshape(B, S, H * D)
    return o @ wo.reshape(wo.shape[0], -1).t() + bo


def test_mha_self_and_cross():
    x = torch.randn(2, 5, 16)
    check(lambda ff, t: ff.multihead_attention(t[0], t[0], t[0], 16, 4),
          lambda x, w: _mha_ref(x[0], x[0], x[0], w[0], w[1], w[2], w[3], 4), [x], tol=2e-4)
    q = torch.randn(2, 5, 16)
    kv = torch.randn(2, 7, 12)

    def ref(x, w):
        H, D = 2, 8
        qq = (x[0] @ w[0].reshape(H * D, -1).t() + w[3].reshape(-1)).view(2, 5, H, D).transpose(1, 2)
        kk = (x[1] @ w[1].reshape(H * D, -1).t() + w[4].reshape(-1)).view(2, 7, H, D).transpose(1, 2)
        vv = (x[2] @ w[2].reshape(H * D, -1).t() + w[5].reshape(-1)).view(2, 7, H, D).transpose(1, 2)
        o = torch.softmax(qq @ kk.transpose(-1, -2) / math.sqrt(D), -1) @ vv
        return o.transpose(1, 2).reshape(2, 5, H * D) @ w[6].reshape(16, -1).t() + w[7]

    check(lambda ff, t: ff.multihead_attention(t[0], t[1], t[2], 16, 2, 8, 8), ref, [q, kv, kv.clone()], tol=2e-4)


def test_elementwise():
    a = torch.rand(3, 4, 5) + 0.5
    b = torch.rand(3, 4, 5) + 0.5
    c = torch.rand(4, 1) + 0.5
    for name, fn in [("add", torch.add), ("subtract", torch.sub), ("multiply", torch.mul), ("divide", torch.div)]:
        check(lambda ff, t, n=name: getattr(ff, n)(t[0], t[1]), lambda x, w, f=fn: f(x[0], x[1]), [a, b])
        check(lambda ff, t, n=name: getattr(ff, n)(t[0], t[1]), lambda x, w, f=fn: f(x[0], x[1]), [a, c])
    check(lambda ff, t: ff.max(t[0], t[1]), lambda x, w: torch.maximum(x[0], x[1]), [a, b])
    check(lambda ff, t: ff.min(t[0], t[1]), lambda x, w: torch.minimum(x[0], x[1]), [a, b])
    un = [("relu", torch.relu), ("sigmoid", torch.sigmoid), ("tanh", torch.tanh), ("elu", F.elu),
          ("gelu", F.gelu), ("exp", torch.exp), ("sin", torch.sin), ("cos", torch.cos), ("rsqrt", torch.rsqrt),
          ("identity", lambda z: z)]
    for name, fn in un:
        check(lambda ff, t, n=name: getattr(ff, n)(t[0]), lambda x, w, f=fn: f(x[0]), [a])
    check(lambda ff, t: ff.pow(t[0], 3.0), lambda x, w: x[0] ** 3, [a])
    check(lambda ff, t: ff.scalar_multiply(t[0], 2.5), lambda x, w: x[0] * 2.5, [a])
    check(lambda ff, t: ff.scalar_add(t[0], 2.5), lambda x, w: x[0] + 2.5, [a])
    check(lambda ff, t: ff.scalar_sub(t[0], 2.5), lambda x, w: x[0] - 2.5, [a])
    check(lambda ff, t: ff.scalar_true_divide(t[0], 2.5), lambda x, w: x[0] / 2.5, [a])


def test_shape_ops():
    a = torch.randn(2, 3, 4, 5)
    check(lambda ff, t: ff.flat(t[0]), lambda x, w: x[0].reshape(2, -1), [a])
    check(lambda ff, t: ff.reshape(t[0], [2, 12, 5]), lambda x, w: x[0].reshape(2, 12, 5), [a])
    check(lambda ff, t: ff.transpose(t[0], [0, 2, 1, 3]), lambda x, w: x[0].permute(0, 2, 1, 3), [a])
    check(lambda ff, t: ff.reverse(t[0], 2), lambda x, w: torch.flip(x[0], [2]), [a])
    b = torch.randn(2, 5, 4, 5)
    check(lambda ff, t: ff.concat([t[0], t[1]], 1), lambda x, w: torch.cat([x[0], x[1]], 1), [a, b])
    check(lambda ff, t: ff.split(t[0], [1, 2], 1), lambda x, w: list(torch.split(x[0], [1, 2], 1)), [a])
    check(lambda ff, t: ff.reduce_sum(t[0], [1, 3]), lambda x, w: x[0].sum((1, 3)), [a])
    check(lambda ff, t: ff.mean(t[0], [2], True), lambda x, w: x[0].mean(2, keepdim=True), [a])
    idx = torch.randint(0, 4, (2, 3, 2, 5))
    check(lambda ff, t: ff.gather(t[0], t[1], 2), lambda x, w: torch.gather(x[0], 2, x[1].long()), [a, idx],
          int_inputs=(1,))


def test_batch_matmul():
    a = torch.randn(3, 4, 6)
    b = torch.randn(3, 6, 5)
    check(lambda ff, t: ff.batch_matmul(t[0], t[1]), lambda x, w: x[0] @ x[1], [a, b])


def test_topk_and_moe_routing():
    x = torch.randn(8, 6)
    L, xs, ws, ys, dys, dxs, wg = run_layer(lambda ff, t: ff.top_k(t[0], 2), [x])
    v, i = torch.topk(x, 2, -1)
    close(torch.sort(ys[0], -1)[0], torch.sort(v, -1)[0])
    # group_by + aggregate_spec compose to a permutation-invariant routing round trip
    ff = FFModel(FFConfig([]))
    d = ff.create_tensor([8, 4])
    a = ff.create_tensor([8, 1], DataType.DT_INT32)
    outs = ff.group_by(d, a, 4, 2.0)
    assert len(outs) == 4 and outs[0].dims == (4, 4)


def test_cast_dropout():
    a = torch.randn(4, 4)
    check(lambda ff, t: ff.dropout(t[0], 0.0, 0), lambda x, w: x[0], [a])
    L, xs, ws, ys, dys, dxs, wg = run_layer(lambda ff, t: ff.dropout(t[0], 0.5, 3), [torch.ones(64, 64)])
    keep = (ys[0] != 0).float().mean().item()
    assert 0.4 < keep < 0.6
    assert torch.allclose(dxs[0], dys[0] * (ys[0] != 0) * 2.0)
