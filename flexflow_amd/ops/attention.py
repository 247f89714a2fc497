"""Multi-head attention (reference src/ops/attention.cc / attention.cu, cuDNN MHA; the reference HIP
build compiles it to a no-op, attention.cpp:33-43).

Semantics follow the reference API: `kdim`/`vdim` are per-head projection sizes, output size is
`embed_dim`. Parallel axes: batch (sample), sequence (query side only; kept at 1), and a *heads*
axis (parameter parallelism): each part owns H/deg heads — its slice of the Q/K/V and output
projections — and emits a partial sum of the output projection (reduced on the consumer edge).

GPU path (bf16): for self-attention ONE fused QKV GEMM ([T,E] x [3*H*D,E]^T) whose output is read
in place by the flash-attention kernel through strides (no permute copies), then the output
projection GEMM; the backward mirrors it (flash bwd writes dQ/dK/dV straight into the fused
[T, 3, H, D] gradient buffer that feeds one dgrad and one split-K wgrad GEMM).
"""
from __future__ import annotations

import math
import os

import torch

from .. import kernels as K
from ..type import OperatorType
from .base import OpImpl, WeightSpec, register


def _pad_heads(t, st, B, S, H, d, Dp):
    """[B, S, H, Dp] zero-padded copy of the strided per-head view (batch, head, row strides st)."""
    out = torch.zeros(B, S, H, Dp, device=t.device, dtype=t.dtype)
    out[..., :d].copy_(t.as_strided((B, H, S, d), (st[0], st[1], st[2], 1)).permute(0, 2, 1, 3))
    return out


def _attn_ref(q, k, v, scale, causal):
    s = torch.einsum("bhqd,bhkd->bhqk", q, k) * scale
    if causal:
        Sq, Sk = s.shape[-2:]
        s = s.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    return torch.einsum("bhqk,bhkd->bhqd", torch.softmax(s, -1), v)


@register(OperatorType.OP_MULTIHEAD_ATTENTION)
class MultiHeadAttention(OpImpl):
    op_type = OperatorType.OP_MULTIHEAD_ATTENTION

    @classmethod
    def infer(cls, attrs, in_dims, in_dtypes):
        q, k, v = in_dims
        H = attrs["num_heads"]
        E = attrs["embed_dim"]
        kd = attrs.get("kdim") or E // H
        vd = attrs.get("vdim") or E // H
        attrs["kdim"], attrs["vdim"] = kd, vd
        dt = in_dtypes[0]
        kinit = attrs.get("kernel_init")
        from ..core.initializers import ZeroInitializer
        ws = []
        if attrs.get("self_attn") and kd == vd and q[-1] == k[-1] == v[-1]:
            attrs["fused_qkv"] = True
            ws.append(WeightSpec("qkv_weight", (3, H, kd, q[-1]), dt, kinit))
            if attrs.get("bias", True):
                ws.append(WeightSpec("qkv_bias", (3, H, kd), dt, ZeroInitializer()))
        else:
            attrs["fused_qkv"] = False
            ws += [WeightSpec("q_weight", (H, kd, q[-1]), dt, kinit), WeightSpec("k_weight", (H, kd, k[-1]), dt, kinit),
                   WeightSpec("v_weight", (H, vd, v[-1]), dt, kinit)]
            if attrs.get("bias", True):
                ws += [WeightSpec("q_bias", (H, kd), dt, ZeroInitializer()),
                       WeightSpec("k_bias", (H, kd), dt, ZeroInitializer()),
                       WeightSpec("v_bias", (H, vd), dt, ZeroInitializer())]
        ws.append(WeightSpec("o_weight", (E, H, vd), dt, kinit))
        if attrs.get("bias", True):
            ws.append(WeightSpec("o_bias", (E,), dt, ZeroInitializer()))
        return [tuple(q[:-1]) + (E,)], [dt], ws

    # axes: 0 batch, 1 seq, 2 embed, 3 heads
    H_AXIS = 3

    def extra_axis_sizes(self):
        return [self.attrs["num_heads"]]

    def axis_kinds(self):
        return ["sample", "none", "none", "parameter"]

    def supports_axis(self, axis):
        return axis in (0, 3)

    def input_maps(self):
        return [(0, 1, None), (0, None, None), (0, None, None)]

    def weight_maps(self):
        out = []
        for w in self.layer.weights:
            n = w.short_name
            if n == "qkv_weight":
                out.append((None, 3, None, None))
            elif n == "qkv_bias":
                out.append((None, 3, None))
            elif n in ("q_weight", "k_weight", "v_weight"):
                out.append((3, None, None))
            elif n in ("q_bias", "k_bias", "v_bias"):
                out.append((3, None))
            elif n == "o_weight":
                out.append((None, 3, None))
            else:  # o_bias
                out.append((None,))
        return out

    def _w(self, ws):
        return {w.short_name: t for w, t in zip(self.layer.weights, ws)}

    def forward(self, ctx, xs, ws):
        q_in, k_in, v_in = xs
        W = self._w(ws)
        B, Sq, _ = q_in.shape
        Sk = k_in.shape[1]
        kd, vd = self.attrs["kdim"], self.attrs["vdim"]
        Hl = W["o_weight"].shape[1]
        E = W["o_weight"].shape[0]
        scale = 1.0 / math.sqrt(kd)
        causal = bool(self.attrs.get("causal", False))
        bo = W.get("o_bias")
        if bo is not None and ctx.degree(self.H_AXIS) > 1 and ctx.coord(self.H_AXIS) != 0:
            bo = None
        fused = self.attrs["fused_qkv"] and (q_in is k_in is v_in or (q_in.data_ptr() == k_in.data_ptr() == v_in.data_ptr()))
        s = ctx.saved if ctx.training else {}
        if fused:
            x2 = q_in.reshape(B * Sq, -1)
            wq = W["qkv_weight"].reshape(3 * Hl * kd, -1)
            bq = W["qkv_bias"].reshape(-1) if "qkv_bias" in W else None
            qkv, _ = K.linear_fwd(x2, wq, bq, K.ACT_NONE, False)  # [T, 3, Hl, D]
            st = [Sq * 3 * Hl * kd, kd, 3 * Hl * kd]
            qv, kv, vv = qkv.view(-1), qkv.view(-1)[Hl * kd:], qkv.view(-1)[2 * Hl * kd:]
            qs = ks = vs = st
            s.update(x2=x2, wqkv=wq, qkv=qkv)
            if ctx.training and ctx.extra.get("need_dx0", True):  # TN dgrad (kernels.weight_t)
                s["wqkv_t"] = K.weight_t(ctx.extra.setdefault("wt_store_qkv", {}), wq)
        else:
            outs = []
            for name, t, d in (("q", q_in, kd), ("k", k_in, kd), ("v", v_in, vd)):
                x2 = t.reshape(-1, t.shape[-1])
                w2 = W[f"{name}_weight"].reshape(Hl * d, -1)
                b2 = W[f"{name}_bias"].reshape(-1) if f"{name}_bias" in W else None
                y, _ = K.linear_fwd(x2, w2, b2, K.ACT_NONE, False)
                outs.append(y)
                s[f"x_{name}"], s[f"w_{name}"] = x2, w2
            qv, kv, vv = outs
            qs = [Sq * Hl * kd, kd, Hl * kd]
            ks = [Sk * Hl * kd, kd, Hl * kd]
            vs = [Sk * Hl * vd, vd, Hl * vd]
            s.update(q=qv, k=kv, v=vv)
        o = torch.empty(B, Sq, Hl, vd, device=q_in.device, dtype=q_in.dtype)
        os_ = [Sq * Hl * vd, vd, Hl * vd]
        if K.attn_supported(q_in, kd) and kd == vd:
            lse = K.flash_attn_fwd(qv, qs, kv, ks, vv, vs, o, os_, B, Hl, Sq, Sk, kd, scale, causal)
            s["lse"] = lse
        elif K.attn_padded_dim(q_in, kd, vd):
            # head dims the MFMA kernels have no instance for (e.g. 16, 32, 80, 96): zero-pad Q, K,
            # V to the next instance (64 / 128). Zero columns add nothing to Q.K^T and give zero
            # output columns, so the softmax and the sliced output are exact; the scale stays
            # 1/sqrt(kd)
            Dp = K.attn_padded_dim(q_in, kd, vd)
            pq, pk, pv = (_pad_heads(t, st, Bq, S_, Hl, kd, Dp) for t, st, Bq, S_ in
                          ((qv, qs, B, Sq), (kv, ks, B, Sk), (vv, vs, B, Sk)))
            po = torch.empty(B, Sq, Hl, Dp, device=q_in.device, dtype=q_in.dtype)
            pst = [Sq * Hl * Dp, Dp, Hl * Dp]
            kst = [Sk * Hl * Dp, Dp, Hl * Dp]
            lse = K.flash_attn_fwd(pq, pst, pk, kst, pv, kst, po, pst, B, Hl, Sq, Sk, Dp, scale, causal)
            o.copy_(po[..., :vd])
            s.update(lse=lse, pad=(Dp, pq, pk, pv, po))
        elif K.attn_f32_supported(q_in) and os.environ.get("FF_ATTN_REF_FALLBACK") != "1":
            # --dtype fp32 on the device: f32 MFMA GEMMs + causal mask + row softmax, our kernels
            s["P"] = K.attn_f32_fwd(qv, qs, kv, ks, vv, vs, o.view(-1), os_, B, Hl, Sq, Sk, kd, vd, scale, causal)
        else:
            if K.native(q_in) and q_in.dtype == torch.bfloat16 and os.environ.get("FF_ATTN_REF_FALLBACK") != "1":
                raise NotImplementedError(
                    f"{self.layer.name}: no MFMA attention kernel for head dims q/k {kd}, v {vd} (supported: equal "
                    "q/k/v head dims up to 128; FF_ATTN_REF_FALLBACK=1 runs the fp32 PyTorch reference instead)")
            q4 = qv.as_strided((B, Hl, Sq, kd), (qs[0], qs[1], qs[2], 1)).float()
            k4 = kv.as_strided((B, Hl, Sk, kd), (ks[0], ks[1], ks[2], 1)).float()
            v4 = vv.as_strided((B, Hl, Sk, vd), (vs[0], vs[1], vs[2], 1)).float()
            o.copy_(_attn_ref(q4, k4, v4, scale, causal).permute(0, 2, 1, 3))
        o2 = o.view(B * Sq, Hl * vd)
        wo = W["o_weight"].reshape(E, Hl * vd)
        if ctx.training:
            s["wo_t"] = K.weight_t(ctx.extra.setdefault("wt_store_o", {}), wo)
        y, _ = K.linear_fwd(o2, wo, bo, K.ACT_NONE, False)
        if ctx.training:
            s.update(o=o, wo=wo, has_bo=bo is not None, shape=(B, Sq, Sk, Hl, kd, vd, E), fused=fused,
                     qs=qs, ks=ks, vs=vs, os=os_, scale=scale, causal=causal)
        return [y.view(B, Sq, E)]

    def overwrites_wgrad(self, i):
        return not self.layer.weights[i].short_name.endswith("bias")  # projection GEMMs use dw_beta = wb

    def _grad_index(self):
        return {w.short_name: i for i, w in enumerate(self.layer.weights)}

    def backward(self, ctx, douts):
        s = ctx.saved
        B, Sq, Sk, Hl, kd, vd, E = s["shape"]
        gi = self._grad_index()
        gw = lambda n: (ctx.wgrads[gi[n]] if (ctx.wgrads and n in gi) else None)  # noqa: E731
        dy2 = douts[0].reshape(B * Sq, E).contiguous()
        o = s["o"]
        o2 = o.view(B * Sq, Hl * vd)
        dwo = gw("o_weight")
        dbo = gw("o_bias") if (s["has_bo"] and not ctx.extra.get("bias_grad_fused")) else None
        wb = 0.0 if ctx.extra.get("wgrad_overwrite") else 1.0
        do2 = K.linear_bwd(dy2, o2, s["wo"], None, K.ACT_NONE,
                           dwo.view(E, Hl * vd) if dwo is not None else None, dbo, dw_beta=wb, wt=s.get("wo_t"))
        do = do2.view(B, Sq, Hl, vd)
        scale, causal = s["scale"], s["causal"]
        qs, ks, vs, os_ = s["qs"], s["ks"], s["vs"], s["os"]
        fused = s["fused"]
        bias_done = False
        if fused:
            qkv = s["qkv"]
            qv, kv, vv = qkv.view(-1), qkv.view(-1)[Hl * kd:], qkv.view(-1)[2 * Hl * kd:]
            dqkv = torch.empty_like(qkv)
            dq, dk, dv = dqkv.view(-1), dqkv.view(-1)[Hl * kd:], dqkv.view(-1)[2 * Hl * kd:]
        else:
            qv, kv, vv = s["q"], s["k"], s["v"]
            dq, dk, dv = torch.empty_like(qv), torch.empty_like(kv), torch.empty_like(vv)
        if "pad" in s:
            Dp, pq, pk, pv, po = s["pad"]
            pdo = torch.zeros_like(po)
            pdo[..., :vd] = do
            pdq, pdk, pdv = torch.empty_like(pq), torch.empty_like(pk), torch.empty_like(pv)
            pst = [Sq * Hl * Dp, Dp, Hl * Dp]
            kst = [Sk * Hl * Dp, Dp, Hl * Dp]
            K.flash_attn_bwd(pq, pst, pk, kst, pv, kst, po, pst, pdo, pst, s["lse"], pdq, pst, pdk, kst, pdv, kst,
                             B, Hl, Sq, Sk, Dp, scale, causal)
            for g, st, pg, S_, d in ((dq, qs, pdq, Sq, kd), (dk, ks, pdk, Sk, kd), (dv, vs, pdv, Sk, vd)):
                g.as_strided((B, Hl, S_, d), (st[0], st[1], st[2], 1)).copy_(pg[..., :d].permute(0, 2, 1, 3))
        elif "lse" in s:
            # fused projection: the kernel can add the QKV bias gradient (column sums of dq / dk / dv)
            # itself, sparing linear_bwd a pass over dqkv (bias_act_bwd + fold)
            dbq = gw("qkv_bias") if (fused and os.environ.get("FF_ATTN_BIAS_FUSION", "1") == "1") else None
            if dbq is not None and dbq.dtype == torch.float32 and dbq.is_contiguous():
                bias_done = K.flash_attn_bwd(qv, qs, kv, ks, vv, vs, o, os_, do, os_, s["lse"], dq, qs, dk, ks, dv, vs,
                                             B, Hl, Sq, Sk, kd, scale, causal, dbias=dbq.view(-1))
            else:
                K.flash_attn_bwd(qv, qs, kv, ks, vv, vs, o, os_, do, os_, s["lse"], dq, qs, dk, ks, dv, vs,
                                 B, Hl, Sq, Sk, kd, scale, causal)
        elif "P" in s:
            K.attn_f32_bwd(qv, qs, kv, ks, vv, vs, do.contiguous().view(-1), os_, s["P"], dq.view(-1), dk.view(-1),
                           dv.view(-1), B, Hl, Sq, Sk, kd, vd, scale)
        else:
            q4 = qv.as_strided((B, Hl, Sq, kd), (qs[0], qs[1], qs[2], 1)).detach().float().requires_grad_()
            k4 = kv.as_strided((B, Hl, Sk, kd), (ks[0], ks[1], ks[2], 1)).detach().float().requires_grad_()
            v4 = vv.as_strided((B, Hl, Sk, vd), (vs[0], vs[1], vs[2], 1)).detach().float().requires_grad_()
            with torch.enable_grad():
                out = _attn_ref(q4, k4, v4, scale, causal)
            g4 = do.permute(0, 2, 1, 3).float()
            gq, gk, gv = torch.autograd.grad(out, (q4, k4, v4), g4)
            dq.as_strided((B, Hl, Sq, kd), (qs[0], qs[1], qs[2], 1)).copy_(gq)
            dk.as_strided((B, Hl, Sk, kd), (ks[0], ks[1], ks[2], 1)).copy_(gk)
            dv.as_strided((B, Hl, Sk, vd), (vs[0], vs[1], vs[2], 1)).copy_(gv)
        if fused:
            dw = gw("qkv_weight")
            db = None if bias_done else gw("qkv_bias")
            acc = (ctx.extra.get("dx_accum") or {}).get(0)
            dx2 = K.linear_bwd(dqkv, s["x2"], s["wqkv"], None, K.ACT_NONE,
                               dw.view(3 * Hl * kd, -1) if dw is not None else None,
                               db.view(-1) if db is not None else None, dw_beta=wb,
                               dx_out=acc.view(B * Sq, -1) if acc is not None else None, wt=s.get("wqkv_t"))
            dx = acc if acc is not None else dx2.view(B, Sq, -1)
            ctx.saved.clear()
            return [dx, None, None]  # all three inputs are the same tensor: gradient once
        grads = []
        accs = ctx.extra.get("dx_accum") or {}
        for slot, (name, g, d, S_) in enumerate((("q", dq, kd, Sq), ("k", dk, kd, Sk), ("v", dv, vd, Sk))):
            acc = accs.get(slot)
            dw = gw(f"{name}_weight")
            db = gw(f"{name}_bias")
            x2 = s[f"x_{name}"]
            dx2 = K.linear_bwd(g.view(B * S_, Hl * d), x2, s[f"w_{name}"], None, K.ACT_NONE,
                               dw.view(Hl * d, -1) if dw is not None else None,
                               db.view(-1) if db is not None else None, dw_beta=wb,
                               dx_out=acc.view(B * S_, -1) if acc is not None else None)
            grads.append(acc if acc is not None else dx2.view(B, S_, -1))
        ctx.saved.clear()
        return grads

    def accumulates_dx(self):
        return True

    def accum_may_alias_douts(self):
        return True  # dy is consumed by the output projection before the QKV dgrad writes

    def flops(self, in_shapes, out_shapes, w_shapes):
        B, Sq, Eq = in_shapes[0]
        Sk = in_shapes[1][1]
        kd, vd = self.attrs["kdim"], self.attrs["vdim"]
        Hl = w_shapes[-2][1] if len(w_shapes[-1]) == 1 else w_shapes[-1][1]
        E = self.attrs["embed_dim"]
        proj = 2.0 * B * (Sq * Hl * kd * Eq + Sk * Hl * kd * Eq + Sk * Hl * vd * Eq + Sq * Hl * vd * E)
        att = 2.0 * B * Hl * Sq * Sk * (kd + vd)
        return proj + att

    def uses_mfma(self):
        return True
