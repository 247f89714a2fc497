"""HuggingFace model import through torch.export (PyTorchModel(is_hf_model=True)).

Reference: python/flexflow/torch/model.py:2408-2607 traces HuggingFace models with
`transformers.utils.fx.symbolic_trace` and maps the fx graph to FFModel calls. That tracer is gone
from transformers 5.x, so here the model is exported with `torch.export` (ATen-level graph with the
shapes of the given batch / sequence lengths) and the graph is mapped directly:

* Every node that depends only on parameters, buffers and literals — position buckets, the
  relative-position-bias lookup, causal masks — is evaluated once at import (constant folding)
  and enters the FFModel as a constant tensor. Consequently a learned table used only there (T5's
  relative_attention_bias) is frozen at its import-time value.
* Inputs whose name contains "mask" (attention_mask) are folded as all-ones: batches are taken
  to be unpadded. A padded batch needs its mask as a separate additive-bias input (not mapped).
* linear / embedding become dense / embedding layers whose weights are the torch parameters
  (copied in at compile); tied weights (T5's shared embedding and lm_head) become separate FF
  weights initialised from the same values.
* T5 / LLaMA RMS norm (x * rsqrt(mean(x^2) + eps) * w) becomes one rms_norm op; the remaining
  arithmetic (add / mul / pow / tanh ...) maps 1:1; scaled_dot_product_attention becomes
  batch_matmul -> (+ bias) -> softmax -> batch_matmul.

The builders are resolved lazily from the graph outputs, so folded or replaced sub-graphs emit
no dead FF layers.
"""
from __future__ import annotations

import math
from typing import Dict, List

import numpy as np
import torch

from ..type import AggrMode, DataType

aten = torch.ops.aten

_IDENTITY = {aten.contiguous.default, aten.clone.default, aten.alias.default, aten.detach.default,
             aten.to.dtype, aten.to.dtype_layout, aten.to.device, aten.lift_fresh_copy.default,
             aten._to_copy.default}
_SKIP = {aten._assert_tensor_metadata.default}


def _example_inputs(model, input_names, batch_size, seq_length):
    if isinstance(seq_length, (list, tuple)):
        enc_len, dec_len = seq_length[0], seq_length[-1]
    else:
        enc_len = dec_len = seq_length or 16
    vocab = int(getattr(getattr(model, "config", None), "vocab_size", 100) or 100)
    g = torch.Generator().manual_seed(0)
    out = {}
    for name in input_names:
        n = dec_len if name.startswith("decoder") else enc_len
        if "mask" in name:
            out[name] = torch.ones(batch_size, n, dtype=torch.long)
        else:
            out[name] = torch.randint(1, vocab, (batch_size, n), generator=g, dtype=torch.long)
    return out


class ExportImporter:
    def __init__(self, model, input_names, batch_size=1, seq_length=None):
        self.model = model
        self.input_names = list(input_names or ["input_ids"])
        self.batch_size = batch_size
        self.seq_length = seq_length
        self.ep = None

    def export(self):
        import inspect
        kw = _example_inputs(self.model, self.input_names, self.batch_size, self.seq_length)
        params = inspect.signature(self.model.forward).parameters
        if "use_cache" in params:
            kw["use_cache"] = False
        if "return_dict" in params:
            kw["return_dict"] = True
        was_training = self.model.training
        self.model.eval()
        try:
            self.ep = torch.export.export(self.model, (), kw, strict=False)
        finally:
            self.model.train(was_training)
        return self.ep

    # ------------------------------------------------------------------ graph -> FFModel
    def to_ff(self, ffmodel, input_tensors) -> list:
        ep = self.ep if self.ep is not None else self.export()
        sig = ep.graph_signature
        state = dict(ep.state_dict)
        consts = dict(getattr(ep, "constants", {}) or {})
        user_inputs = list(sig.user_inputs)
        ff_inputs = dict(zip(self.input_names, input_tensors))
        const: Dict[str, object] = {}
        params = set()
        node_of = {}
        for n in ep.graph.nodes:
            node_of[n.name] = n
            if n.op != "placeholder":
                continue
            if n.name in sig.inputs_to_parameters:
                const[n.name] = state[sig.inputs_to_parameters[n.name]].detach()
                params.add(n.name)
            elif n.name in sig.inputs_to_buffers:
                fqn = sig.inputs_to_buffers[n.name]
                const[n.name] = (state[fqn] if fqn in state else consts[fqn]).detach()
            elif n.name in getattr(sig, "inputs_to_lifted_tensor_constants", {}):
                const[n.name] = consts[sig.inputs_to_lifted_tensor_constants[n.name]].detach()
            elif n.name in user_inputs and "mask" in n.name:  # folded: unpadded batches (module doc)
                const[n.name] = torch.ones(n.meta["val"].shape, dtype=n.meta["val"].dtype)
        # constant folding, in graph order
        for n in ep.graph.nodes:
            if n.op != "call_function" or n.target in _SKIP:
                continue
            if all(a.name in const for a in n.all_input_nodes):
                args = torch.fx.node.map_arg(n.args, lambda a: const[a.name])
                kwargs = torch.fx.node.map_arg(n.kwargs, lambda a: const[a.name])
                with torch.no_grad():
                    v = n.target(*args, **kwargs)
                const[n.name] = v.detach() if isinstance(v, torch.Tensor) else v
        self._ff, self._const, self._params, self._node_of = ffmodel, const, params, node_of
        self._env: Dict[str, object] = dict(ff_inputs)
        self._copies: List = []
        out_node = next(n for n in ep.graph.nodes if n.op == "output")
        outs = out_node.args[0]
        outs = list(outs) if isinstance(outs, (list, tuple)) else [outs]
        first = next(o for o in outs if isinstance(o, torch.fx.Node))
        result = [self._ff_of(first)]
        for w, arr in self._copies:  # applied at compile (FFModel._pending_weights)
            w.set_weights(ffmodel, arr)
        return result

    # lazily build the FF tensor of a dynamic node
    def _val(self, a):
        if isinstance(a, torch.fx.Node):
            return self._const[a.name] if a.name in self._const else self._ff_of(a)
        return a

    def _is_const(self, a):
        return not isinstance(a, torch.fx.Node) or a.name in self._const

    def _shape(self, n):
        return tuple(int(s) for s in n.meta["val"].shape)

    def _const_tensor(self, value, name):
        v = value.float().numpy() if isinstance(value, torch.Tensor) else np.asarray(value, np.float32)
        if v.ndim == 0:
            return float(v)
        t = self._ff.create_tensor(list(v.shape), DataType.DT_FLOAT, create_grad=False, name=name)
        t.set_tensor(self._ff, v.astype(np.float32))
        return t

    def _ff_of(self, n):
        if n.name in self._env:
            return self._env[n.name]
        if n.op == "placeholder":
            raise NotImplementedError(f"model input {n.name} was not given an FF tensor")
        t = self._build(n)
        self._env[n.name] = t
        return t

    def _rms_match(self, w_node, x_node):
        """x_node = mul(h, rsqrt(add(mean(pow(h, 2), [-1], True), eps))) [through to() casts]."""
        def strip(m):
            while isinstance(m, torch.fx.Node) and m.op == "call_function" and m.target in _IDENTITY:
                m = m.args[0]
            return m
        x_node = strip(x_node)
        if not (isinstance(x_node, torch.fx.Node) and x_node.target == aten.mul.Tensor):
            return None
        for h, r in (x_node.args, x_node.args[::-1]):
            r = strip(r)
            if not (isinstance(r, torch.fx.Node) and r.target == aten.rsqrt.default):
                continue
            ad = strip(r.args[0])
            if not (isinstance(ad, torch.fx.Node) and ad.target in (aten.add.Tensor, aten.add.Scalar)):
                continue
            mean, eps = ad.args[0], ad.args[1]
            if isinstance(eps, torch.fx.Node):
                if eps.name not in self._const:
                    continue
                eps = float(self._const[eps.name])
            mean = strip(mean)
            if not (isinstance(mean, torch.fx.Node) and mean.target == aten.mean.dim):
                continue
            pw = strip(mean.args[0])
            if not (isinstance(pw, torch.fx.Node) and pw.target == aten.pow.Tensor_Scalar and pw.args[1] == 2):
                continue
            if strip(pw.args[0]) is not strip(h):
                continue
            return strip(h), float(eps)
        return None

    def _build(self, n):
        ff, tgt, a = self._ff, n.target, n.args
        name = n.name
        if tgt in _IDENTITY:
            return self._val(a[0])
        if tgt == aten.linear.default:
            W = self._const[a[1].name]
            b = a[2] if len(a) > 2 else None
            y = ff.dense(self._val(a[0]), int(W.shape[0]), use_bias=b is not None, name=name)
            L = ff.layers[-1]
            self._copies.append((L.weights[0], W.float().numpy()))
            if b is not None:
                self._copies.append((L.weights[1], self._const[b.name].float().numpy()))
            return y
        if tgt == aten.embedding.default:
            W = self._const[a[0].name]
            y = ff.embedding(self._val(a[1]), int(W.shape[0]), int(W.shape[1]), AggrMode.AGGR_MODE_NONE, name=name)
            self._copies.append((ff.layers[-1].weights[0], W.float().numpy()))
            return y
        if tgt in (aten.mul.Tensor, aten.mul.Scalar):
            x, y = a[0], a[1]
            # RMS norm: mul(weight_param, normalized(h)) (either operand order)
            for w_, x_ in ((x, y), (y, x)):
                if isinstance(w_, torch.fx.Node) and w_.name in self._params and self._const[w_.name].dim() == 1:
                    m = self._rms_match(w_, x_)
                    if m is not None:
                        h, eps = m
                        out = ff.rms_norm(self._val(h), eps, name=name)
                        self._copies.append((ff.layers[-1].weights[0], self._const[w_.name].float().numpy()))
                        return out
            return self._binary("mul", x, y, name)
        if tgt in (aten.add.Tensor, aten.add.Scalar):
            if len(a) > 2 and a[2] != 1:
                raise NotImplementedError("add with alpha")
            return self._binary("add", a[0], a[1], name)
        if tgt in (aten.sub.Tensor, aten.sub.Scalar):
            return self._binary("sub", a[0], a[1], name)
        if tgt in (aten.div.Tensor, aten.div.Scalar):
            return self._binary("div", a[0], a[1], name)
        if tgt == aten.rsub.Scalar:  # s - x
            return ff.scalar_add(ff.scalar_multiply(self._val(a[0]), -1.0, inplace=False), float(a[1]), inplace=False,
                                 name=name)
        if tgt == aten.pow.Tensor_Scalar:
            return ff.pow(self._val(a[0]), float(a[1]), name=name)
        if tgt == aten.mean.dim:
            x = self._val(a[0])
            dims = [d % len(x.dims) for d in a[1]]
            return ff.mean(x, dims, bool(a[2]) if len(a) > 2 else False, name=name)
        if tgt == aten.rsqrt.default:
            return ff.rsqrt(self._val(a[0]), name=name)
        if tgt == aten.tanh.default:
            return ff.tanh(self._val(a[0]), name=name)
        if tgt == aten.relu.default:
            return ff.relu(self._val(a[0]), inplace=False, name=name)
        if tgt == aten.gelu.default:
            return ff.gelu(self._val(a[0]), inplace=False, name=name)
        if tgt == aten.exp.default:
            return ff.exp(self._val(a[0]), name=name)
        if tgt == aten.sigmoid.default:
            return ff.sigmoid(self._val(a[0]), name=name)
        if tgt == aten.neg.default:
            return ff.scalar_multiply(self._val(a[0]), -1.0, inplace=False, name=name)
        if tgt in (aten.softmax.int, aten._softmax.default):
            x = self._val(a[0])
            return ff.softmax(x, int(a[1]) % len(x.dims), name=name)
        if tgt == aten.dropout.default:
            p = float(a[1])
            return ff.dropout(self._val(a[0]), p, name=name) if p > 0 else self._val(a[0])
        if tgt == aten.transpose.int:
            x = self._val(a[0])
            perm = list(range(len(x.dims)))
            d0, d1 = a[1] % len(perm), a[2] % len(perm)
            perm[d0], perm[d1] = perm[d1], perm[d0]
            return ff.transpose(x, perm, name=name)
        if tgt == aten.permute.default:
            return ff.transpose(self._val(a[0]), [int(d) for d in a[1]], name=name)
        if tgt in (aten.view.default, aten.reshape.default, aten._unsafe_view.default, aten.unsqueeze.default,
                   aten.squeeze.dim, aten.flatten.using_ints):
            x = self._val(a[0])
            shape = list(self._shape(n))
            return x if tuple(x.dims) == tuple(shape) else ff.reshape(x, shape, name=name)
        if tgt == aten.expand.default:
            x = self._val(a[0])
            if tuple(x.dims) == self._shape(n):
                return x
            raise NotImplementedError("expand of a model-dependent tensor")
        if tgt == aten.scaled_dot_product_attention.default:
            return self._sdpa(n)
        raise NotImplementedError(f"torch.export import: no mapping for {tgt}")

    def _binary(self, kind, x, y, name):
        ff = self._ff
        if self._is_const(x) and self._is_const(y):
            raise AssertionError("constant binary op reached the builder")
        if self._is_const(y) or self._is_const(x):
            c, t, rev = (self._val(y), self._val(x), False) if self._is_const(y) else (self._val(x), self._val(y), True)
            if isinstance(c, torch.Tensor) and c.numel() == 1:
                c = float(c.reshape(()))
            if not isinstance(c, torch.Tensor) and not isinstance(c, np.ndarray) and not hasattr(c, "dims"):
                c = float(c)
                if kind == "mul":
                    return ff.scalar_multiply(t, c, inplace=False, name=name)
                if kind == "add":
                    return ff.scalar_add(t, c, inplace=False, name=name)
                if kind == "sub":
                    if rev:  # c - t
                        return ff.scalar_add(ff.scalar_multiply(t, -1.0, inplace=False), c, inplace=False, name=name)
                    return ff.scalar_sub(t, c, inplace=False, name=name)
                if kind == "div" and not rev:
                    return ff.scalar_true_divide(t, c, inplace=False, name=name)
                raise NotImplementedError("scalar / tensor")
            ct = self._const_tensor(c, name + "_const")
            x_, y_ = (ct, t) if rev else (t, ct)
        else:
            x_, y_ = self._val(x), self._val(y)
        fn = {"mul": ff.multiply, "add": ff.add, "sub": ff.subtract, "div": ff.divide}[kind]
        return fn(x_, y_, name=name)

    def _sdpa(self, n):
        ff = self._ff
        a, kw = list(n.args), dict(n.kwargs)
        names = ["query", "key", "value", "attn_mask", "dropout_p", "is_causal", "scale"]
        args = dict(zip(names, a))
        args.update(kw)
        if args.get("is_causal"):
            raise NotImplementedError("sdpa is_causal=True (causal masks arrive as attn_mask constants)")
        q, k, v = (self._val(args[x]) for x in ("query", "key", "value"))
        D = q.dims[-1]
        scale = args.get("scale")
        scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
        perm = list(range(len(k.dims)))
        perm[-1], perm[-2] = perm[-2], perm[-1]
        s = ff.batch_matmul(q, ff.transpose(k, perm))
        if scale != 1.0:
            s = ff.scalar_multiply(s, scale, inplace=False)
        m = args.get("attn_mask")
        if m is not None:
            if self._is_const(m):
                mv = self._val(m)
                if mv.dtype == torch.bool:
                    mv = torch.zeros(mv.shape).masked_fill(~mv, -1e9)
                s = ff.add(s, self._const_tensor(mv, n.name + "_mask"))
            else:
                s = ff.add(s, self._val(m))
        p = ff.softmax(s, len(s.dims) - 1)
        dp = float(args.get("dropout_p") or 0.0)
        if dp > 0:
            p = ff.dropout(p, dp)
        return ff.batch_matmul(p, v, name=n.name)
