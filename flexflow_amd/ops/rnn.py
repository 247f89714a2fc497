"""LSTM layer (the reference's legacy Legion NMT application, nmt/lstm.cu + nmt/rnn.cu: cuDNN LSTM
over chunks of timesteps with per-chunk GPU placement; there is no LSTM in the reference's FFModel).

Here it is an FFModel op: inputs x [B, L, E], hx [B, H], cx [B, H]; outputs y [B, L, H], hy, cy;
weights W_ih [4H, E], W_hh [4H, H], b [4H] (gate order i, f, g, o, as torch.nn.LSTM with
b = b_ih + b_hh). Parallel axes: the batch only (the recurrence couples time and hidden units);
model parallelism between layers / time chunks — the reference NMT's GPU placement — is the op
placement the strategy search already expresses (per-op device lists).

Execution (compute dtype, fp32 cell state):
  forward : one GEMM for the input projection of all L steps (+ bias), then per step one GEMM
            accumulating h_{t-1}.W_hh^T into that step's gate rows (beta = 1, strided rows) and the
            fused pointwise step kernel (csrc/kernels/rnn.hip), which writes h straight into y[:, t];
  backward: per step (reverse) the pointwise backward kernel (gate gradients overwrite the saved
            gates in place) and one GEMM for dh_{t-1} = dG_t.W_hh; then the weight gradients
            dW_ih = dG^T X, dW_hh = dG^T H_prev, db = colsum(dG) and dx = dG.W_ih as single GEMMs
            over all B*L rows (split-K-friendly shapes instead of L small ones).
"""
from __future__ import annotations

import math

import torch

from .. import kernels as K
from ..type import OperatorType
from .base import OpImpl, WeightSpec, register


@register(OperatorType.OP_LSTM)
class LSTM(OpImpl):
    op_type = OperatorType.OP_LSTM

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        B, L, E = in_dims[0]
        H = int(attrs["hidden_size"])
        dt = in_dtypes[0]
        from ..core.initializers import UniformInitializer, ZeroInitializer
        k = 1.0 / math.sqrt(H)  # torch.nn.LSTM's default U(-1/sqrt(H), 1/sqrt(H))
        init = attrs.get("kernel_init") or UniformInitializer(int(attrs.get("seed", 7)), -k, k)
        ws = [WeightSpec("w_ih", (4 * H, E), dt, init), WeightSpec("w_hh", (4 * H, H), dt, init),
              WeightSpec("bias", (4 * H,), dt, ZeroInitializer())]
        return [(B, L, H), (B, H), (B, H)], [dt, dt, dt], ws

    def axis_kinds(self):
        return ["sample", "none", "none"]

    def supports_axis(self, axis):
        return axis == 0

    def input_maps(self):
        return [(0, None, None), (0, None), (0, None)]

    def output_maps(self):
        return [(0, 1, 2), (0, None), (0, None)]

    def saves_output(self):
        return True  # backward reads y (the h_{t-1} operand of dW_hh)

    def flops(self, in_shapes, out_shapes, w_shapes):
        B, L, E = in_shapes[0]
        H = out_shapes[0][-1]
        return 2.0 * B * L * 4 * H * (E + H) + 10.0 * B * L * H

    def uses_mfma(self):
        return True

    def overwrites_wgrad(self, i):
        return i in (0, 1)  # W_ih / W_hh GEMMs with beta = 0 under wgrad_overwrite

    # ------------------------------------------------------------------ execution
    def forward(self, ctx, xs, ws):
        x, hx, cx = xs
        w_ih, w_hh, b = ws
        B, L, E = x.shape
        H = w_hh.shape[1]
        dev, dt = x.device, x.dtype
        x2 = x.reshape(B * L, E).contiguous()
        G = torch.empty(B * L * 4 * H, device=dev, dtype=dt)
        K.gemm(x2, w_ih, G, B * L, 4 * H, E, True, True, E, E, 4 * H, bias=b)
        y = torch.empty(B, L, H, device=dev, dtype=dt)
        yf = y.view(-1)
        cs = torch.empty(L + 1, B * H, device=dev, dtype=torch.float32)
        cs[0].copy_(cx.reshape(-1))
        hx = hx.reshape(B, H).contiguous().to(dt)
        ldg, ldy = L * 4 * H, L * H
        for t in range(L):
            Gt = G[t * 4 * H:]
            if t == 0:
                K.gemm(hx, w_hh, Gt, B, 4 * H, H, True, True, H, H, ldg, beta=1.0)
            else:
                K.gemm(yf[(t - 1) * H:], w_hh, Gt, B, 4 * H, H, True, True, ldy, H, ldg, beta=1.0)
            K.lstm_fwd_cell(Gt, ldg, cs[t], cs[t + 1], yf[t * H:], ldy, B, H)
        hy = y[:, L - 1].contiguous()
        cy = cs[L].view(B, H).to(dt)
        if ctx.training:
            ctx.saved.update(G=G, cs=cs, x2=x2, y=y, hx=hx, w_ih=w_ih, w_hh=w_hh, shape=(B, L, E, H))
        return [y, hy, cy]

    def backward(self, ctx, douts):
        s = ctx.saved
        B, L, E, H = s["shape"]
        G, cs, x2, y, hx = s["G"], s["cs"], s["x2"], s["y"], s["hx"]
        w_ih, w_hh = s["w_ih"], s["w_hh"]
        dev, dt = G.device, G.dtype
        dy, dhy, dcy = (list(douts) + [None, None, None])[:3]
        dyf = dy.reshape(-1).contiguous() if dy is not None else None
        dc = dcy.reshape(-1).float().clone() if dcy is not None else torch.zeros(B * H, device=dev)
        dh_rec = dhy.reshape(B, H).contiguous().to(dt) if dhy is not None else None
        ldg, ldy = L * 4 * H, L * H
        for t in reversed(range(L)):
            Gt = G[t * 4 * H:]
            K.lstm_bwd_cell(Gt, ldg, cs[t + 1], cs[t], dyf[t * H:] if dyf is not None else None, ldy, dh_rec, dc,
                            Gt, B, H)
            nxt = torch.empty(B, H, device=dev, dtype=dt)
            K.gemm(Gt, w_hh, nxt, B, H, 4 * H, True, False, ldg, H, H)
            dh_rec = nxt
        dG2 = G.view(B * L, 4 * H)
        wb = 0.0 if ctx.extra.get("wgrad_overwrite") else 1.0
        if ctx.wgrads and ctx.wgrads[0] is not None:
            K.gemm(dG2, x2, ctx.wgrads[0].view(4 * H, E), 4 * H, E, B * L, False, False, 4 * H, E, E, beta=wb)
        if len(ctx.wgrads) > 1 and ctx.wgrads[1] is not None:
            hprev = torch.empty(B, L, H, device=dev, dtype=dt)
            hprev[:, 0].copy_(hx)
            if L > 1:
                hprev[:, 1:].copy_(y[:, :L - 1])
            K.gemm(dG2, hprev.view(B * L, H), ctx.wgrads[1].view(4 * H, H), 4 * H, H, B * L, False, False, 4 * H, H, H,
                   beta=wb)
        if len(ctx.wgrads) > 2 and ctx.wgrads[2] is not None:
            K.bias_grad(dG2, ctx.wgrads[2].view(-1))
        dx = None
        if ctx.extra.get("need_dx0", True):
            dx = torch.empty(B * L, E, device=dev, dtype=dt)
            K.gemm(dG2, w_ih, dx, B * L, E, 4 * H, True, False, 4 * H, E, E)
            dx = dx.view(B, L, E)
        ctx.saved.clear()
        return [dx, dh_rec, dc.view(B, H).to(dt)]
