"""torch.fx frontend: PyTorch nn.Module -> `.ff` text IR -> FFModel (reference
python/flexflow/torch/model.py: PyTorchModel.torch_to_ff / torch_to_string / torch_to_file /
file_to_ff).

The `.ff` format is the reference's, one node per line:
    name; in_1,in_2,; out_1,; OP_TYPE; arg; arg; ...
(IR_DELIMITER "; ", in/out lists comma-terminated, OP_TYPE = flexflow_amd.type.OpType member name),
so files exported by either implementation load in the other for the shared op set.

Design: a single table maps each fx target (module class, function, or method name) to an encoder
(fx node -> OP_TYPE + string args) and each OP_TYPE to a builder (FFModel, inputs, args -> output).
Direct conversion (torch_to_ff) simply round-trips through the same strings, so the file path and
the in-memory path cannot drift apart. Shapes that the IR leaves symbolic (view(-1, n), flatten,
adaptive pooling) are resolved against the FFModel tensor dims at build time. Python values
(tensor.size(), getitem on shapes / split outputs) flow through the same environment as tensors.

`copy_weights(ffmodel)` (after compile) loads the torch module's parameters into the FFModel, so
a converted model reproduces the torch forward pass exactly (tests/test_torch_frontend_cpu.py).
"""
from __future__ import annotations

import math
import operator
from typing import Callable, Dict, List, Optional

import numpy as np

from ..type import ActiMode, AggrMode, DataType, OpType, PoolType

IR_DELIMITER = "; "
INOUT_NODE_DELIMITER = ","


def _fmt_list(v):
    return "[" + ",".join(str(int(x)) for x in v) + "]"


def _parse_list(s):
    s = s.strip()
    if s in ("", "[]"):
        return []
    return [int(x) for x in s.strip("[]").split(",") if x.strip() != ""]


class IRNode:
    def __init__(self, name, innodes, outnodes, op_type: OpType, args: List[str]):
        self.name, self.innodes, self.outnodes, self.op_type, self.args = name, innodes, outnodes, op_type, args

    def to_string(self):
        if self.op_type == OpType.ATTRIBUTE:
            return IR_DELIMITER.join([self.name, self.op_type.name] + self.args)
        ins = "".join(f"{n}{INOUT_NODE_DELIMITER}" for n in self.innodes)
        outs = "".join(f"{n}{INOUT_NODE_DELIMITER}" for n in self.outnodes)
        return IR_DELIMITER.join([self.name, ins, outs, self.op_type.name] + [str(a) for a in self.args])

    @staticmethod
    def from_string(line: str) -> "IRNode":
        items = [i.strip() for i in line.strip().split(";")]
        if len(items) >= 2 and items[1] == OpType.ATTRIBUTE.name:
            return IRNode(items[0], [], [], OpType.ATTRIBUTE, items[2:])
        ins = [n.strip() for n in items[1].split(INOUT_NODE_DELIMITER) if n.strip()]
        outs = [n.strip() for n in items[2].split(INOUT_NODE_DELIMITER) if n.strip()]
        return IRNode(items[0], ins, outs, OpType[items[3]], items[4:])


# --------------------------------------------------------------------------- encoders (fx -> IR)
def _acti_of(m):
    return str(ActiMode.AC_MODE_NONE.value)


def _enc_module(m, node) -> (OpType, List[str]):
    import torch.nn as nn
    if isinstance(m, nn.Linear):
        return OpType.LINEAR, [m.out_features, ActiMode.AC_MODE_NONE.value, int(m.bias is not None)]
    if isinstance(m, nn.Conv2d):
        kh, kw = m.kernel_size
        sh, sw = m.stride
        if isinstance(m.padding, str):
            raise NotImplementedError("string padding on Conv2d")
        ph, pw = m.padding
        return OpType.CONV2D, [m.out_channels, kh, kw, sh, sw, ph, pw, ActiMode.AC_MODE_NONE.value, m.groups,
                               int(m.bias is not None)]
    if isinstance(m, (nn.MaxPool2d, nn.AvgPool2d)):
        k = m.kernel_size if isinstance(m.kernel_size, tuple) else (m.kernel_size, m.kernel_size)
        st = m.stride if m.stride is not None else k
        st = st if isinstance(st, tuple) else (st, st)
        p = m.padding if isinstance(m.padding, tuple) else (m.padding, m.padding)
        pt = PoolType.POOL_MAX if isinstance(m, nn.MaxPool2d) else PoolType.POOL_AVG
        return OpType.POOL2D, [k[0], k[1], st[0], st[1], p[0], p[1], pt.value, ActiMode.AC_MODE_NONE.value]
    if isinstance(m, (nn.AdaptiveAvgPool2d, nn.AdaptiveMaxPool2d)):
        o = m.output_size if isinstance(m.output_size, tuple) else (m.output_size, m.output_size)
        pt = PoolType.POOL_AVG if isinstance(m, nn.AdaptiveAvgPool2d) else PoolType.POOL_MAX
        return OpType.POOL2D, ["adaptive", o[0], o[1], pt.value]
    if isinstance(m, nn.BatchNorm2d):
        return OpType.BATCH_NORM, []
    if isinstance(m, nn.LayerNorm):
        return OpType.LAYER_NORM, [len(m.normalized_shape), m.eps, int(m.elementwise_affine)]
    if isinstance(m, nn.Embedding):
        return OpType.EMBEDDING, [m.num_embeddings, m.embedding_dim]
    if isinstance(m, nn.Softmax):
        return OpType.SOFTMAX, [m.dim if m.dim is not None else -1]
    if isinstance(m, nn.Dropout):
        return OpType.DROPOUT, [m.p]
    if isinstance(m, nn.Flatten):
        return OpType.FLAT, [m.start_dim, m.end_dim]
    if isinstance(m, nn.MultiheadAttention):
        if not m.batch_first:
            raise NotImplementedError("MultiheadAttention(batch_first=False)")
        return OpType.MULTIHEAD_ATTENTION, [m.embed_dim, m.num_heads, int(m.in_proj_bias is not None)]
    simple = {nn.ReLU: OpType.RELU, nn.GELU: OpType.GELU, nn.Sigmoid: OpType.SIGMOID, nn.Tanh: OpType.TANH,
              nn.ELU: OpType.ELU, nn.Identity: OpType.IDENTITY}
    for cls, op in simple.items():
        if isinstance(m, cls):
            return op, []
    raise NotImplementedError(f"unsupported module {type(m).__name__}")


def _fn_key(target):
    if isinstance(target, str):
        return target
    return getattr(target, "__name__", str(target))


_BINARY = {"add": OpType.ADD, "sub": OpType.SUBTRACT, "mul": OpType.MULTIPLY, "truediv": OpType.DIVIDE,
           "div": OpType.DIVIDE, "iadd": OpType.ADD, "isub": OpType.SUBTRACT, "imul": OpType.MULTIPLY}
_SCALAR = {"add": OpType.SCALAR_ADD, "sub": OpType.SCALAR_SUB, "mul": OpType.SCALAR_MULTIPLY,
           "truediv": OpType.SCALAR_TRUEDIV, "div": OpType.SCALAR_TRUEDIV, "floordiv": OpType.SCALAR_FLOORDIV,
           "iadd": OpType.SCALAR_ADD, "isub": OpType.SCALAR_SUB, "imul": OpType.SCALAR_MULTIPLY}
_UNARY = {"relu": OpType.RELU, "gelu": OpType.GELU, "tanh": OpType.TANH, "sigmoid": OpType.SIGMOID,
          "exp": OpType.EXP, "rsqrt": OpType.RSQRT, "sin": OpType.SIN, "cos": OpType.COS, "elu": OpType.ELU,
          "contiguous": OpType.CONTIGUOUS, "float": OpType.FLOAT}


def _is_node(a):
    return hasattr(a, "op") and hasattr(a, "name") and hasattr(a, "users")


def _enc_function(node):
    """call_function / call_method -> (OpType, innode names, args)."""
    key = _fn_key(node.target)
    a = list(node.args)
    kw = dict(node.kwargs)
    ins = [x.name for x in a if _is_node(x)]
    if key in _BINARY and len(a) == 2:
        l, r = a
        if _is_node(l) and _is_node(r):
            return _BINARY[key], ins, []
        scalar = r if _is_node(l) else l
        if key in ("sub", "isub", "truediv", "div") and not _is_node(l):
            raise NotImplementedError(f"scalar {key} with the tensor on the right")
        return _SCALAR[key], ins, [float(scalar)]
    if key == "floordiv" and not _is_node(a[1]):
        return OpType.SCALAR_FLOORDIV, ins, [float(a[1])]
    if key in ("cat", "concat"):
        ts = a[0]
        return OpType.CONCAT, [t.name for t in ts], [kw.get("dim", a[1] if len(a) > 1 else 0)]
    if key == "split":
        size = kw.get("split_size_or_sections", a[1])
        dim = kw.get("dim", a[2] if len(a) > 2 else 0)
        sizes = size if isinstance(size, (list, tuple)) else [size]
        return OpType.SPLIT, ins, [_fmt_list(sizes), dim, int(isinstance(size, (list, tuple)))]
    if key == "flatten":
        return OpType.FLAT, ins, [kw.get("start_dim", a[1] if len(a) > 1 else 0),
                                  kw.get("end_dim", a[2] if len(a) > 2 else -1)]
    if key in _UNARY:
        return _UNARY[key], ins, []
    if key == "softmax":
        return OpType.SOFTMAX, ins, [kw.get("dim", a[1] if len(a) > 1 else -1)]
    if key == "dropout":
        return OpType.DROPOUT, ins, [kw.get("p", a[1] if len(a) > 1 else 0.5)]
    if key == "getitem":
        return OpType.GETITEM, ins, [a[1] if isinstance(a[1], int) else repr(a[1])]
    if key in ("matmul", "bmm"):
        return OpType.BATCH_MATMUL, ins, []
    if key == "transpose":
        return OpType.TRANSPOSE, ins, [a[1], a[2]]
    if key == "permute":
        perm = a[1:] if not isinstance(a[1], (list, tuple)) else a[1]
        return OpType.PERMUTE, ins, [_fmt_list(perm)]
    if key in ("view", "reshape"):
        shp = a[1:] if not isinstance(a[1], (list, tuple)) else a[1]
        if any(_is_node(s) for s in shp):
            return OpType.VIEW, ins, ["dynamic"] + [s.name if _is_node(s) else int(s) for s in shp]
        return OpType.RESHAPE if key == "reshape" else OpType.VIEW, ins, [_fmt_list(shp)]
    if key == "unsqueeze":
        return OpType.UNSQUEEZE, ins, [a[1]]
    if key in ("to", "type_as"):
        return OpType.TO if key == "to" else OpType.TYPE_AS, ins[:1], []
    if key == "pow":
        return OpType.POW, ins, [float(a[1])]
    if key == "mean":
        dims = kw.get("dim", a[1] if len(a) > 1 else None)
        dims = [dims] if isinstance(dims, int) else list(dims)
        return OpType.MEAN, ins, [_fmt_list(dims), int(kw.get("keepdim", a[2] if len(a) > 2 else False))]
    if key == "sum":
        dims = kw.get("dim", a[1] if len(a) > 1 else None)
        dims = [dims] if isinstance(dims, int) else list(dims)
        return OpType.REDUCE_SUM, ins, [_fmt_list(dims), int(kw.get("keepdim", a[2] if len(a) > 2 else False))]
    if key == "size":
        return OpType.GETATTR, ins, ["size"] + ([a[1]] if len(a) > 1 else [])
    if key == "getattr" and a[1] in ("shape",):
        return OpType.GETATTR, ins, ["size"]
    if key == "expand":
        return OpType.EXPAND, ins, [_fmt_list(a[1:] if not isinstance(a[1], (list, tuple)) else a[1])]
    if key == "layer_norm":
        shp = a[1]
        return OpType.LAYER_NORM, ins[:1], [len(shp), kw.get("eps", 1e-5), 0]
    raise NotImplementedError(f"unsupported function/method {key}")


# --------------------------------------------------------------------------- builders (IR -> FF)
def _axis(ax, nd):
    return ax + nd if ax < 0 else ax


def _build(ff, node: IRNode, ins: list, name: str):
    op, a = node.op_type, node.args
    x = ins[0] if ins else None
    nd = len(x.dims) if x is not None and hasattr(x, "dims") else 0
    if op == OpType.LINEAR:
        return ff.dense(x, int(a[0]), ActiMode(int(a[1])), bool(int(a[2])), name=name)
    if op == OpType.CONV2D:
        v = [int(t) for t in a]
        return ff.conv2d(x, v[0], v[1], v[2], v[3], v[4], v[5], v[6], ActiMode(v[7]), v[8], bool(v[9]), name=name)
    if op == OpType.POOL2D:
        if a[0] == "adaptive":
            oh, ow, pt = int(a[1]), int(a[2]), PoolType(int(a[3]))
            h, w = x.dims[2], x.dims[3]
            if h % oh or w % ow:
                raise NotImplementedError("adaptive pooling with a non-divisible output size")
            kh, kw = h // oh, w // ow
            return ff.pool2d(x, kh, kw, kh, kw, 0, 0, pt, name=name)
        v = [int(t) for t in a]
        return ff.pool2d(x, v[0], v[1], v[2], v[3], v[4], v[5], PoolType(v[6]), ActiMode(v[7]), name=name)
    if op == OpType.BATCH_NORM:
        return ff.batch_norm(x, relu=False, name=name)
    if op == OpType.LAYER_NORM:
        n = int(a[0])
        return ff.layer_norm(x, list(range(nd - n, nd)), bool(int(a[2])), float(a[1]), name=name)
    if op == OpType.EMBEDDING:
        return ff.embedding(x, int(a[0]), int(a[1]), AggrMode.AGGR_MODE_NONE, name=name)
    if op == OpType.SOFTMAX:
        return ff.softmax(x, _axis(int(a[0]), nd), name=name)
    if op == OpType.DROPOUT:
        return ff.dropout(x, float(a[0]), 0, name=name)
    if op == OpType.FLAT:
        s, e = _axis(int(a[0]), nd), _axis(int(a[1]), nd)
        if s == 1 and e == nd - 1:
            return ff.flat(x, name=name)
        shp = list(x.dims[:s]) + [int(np.prod(x.dims[s:e + 1]))] + list(x.dims[e + 1:])
        return ff.reshape(x, shp, name=name)
    if op == OpType.MULTIHEAD_ATTENTION:
        E, H, bias = int(a[0]), int(a[1]), bool(int(a[2]))
        q, k, v = (ins + [ins[0]] * 3)[:3]
        # torch returns (attn_output, attn_weights); the weights are not materialised
        return (ff.multihead_attention(q, k, v, E, H, E // H, E // H, 0.0, bias, name=name), None)
    unary = {OpType.RELU: ff.relu, OpType.GELU: ff.gelu, OpType.SIGMOID: ff.sigmoid, OpType.TANH: ff.tanh,
             OpType.ELU: ff.elu, OpType.EXP: ff.exp, OpType.RSQRT: ff.rsqrt, OpType.SIN: ff.sin, OpType.COS: ff.cos}
    if op in unary:
        return unary[op](x, name=name)
    if op in (OpType.IDENTITY, OpType.CONTIGUOUS, OpType.FLOAT, OpType.TO, OpType.TYPE_AS):
        return x
    binary = {OpType.ADD: ff.add, OpType.SUBTRACT: ff.subtract, OpType.MULTIPLY: ff.multiply,
              OpType.DIVIDE: ff.divide}
    if op in binary:
        return binary[op](ins[0], ins[1], name=name)
    scalar = {OpType.SCALAR_ADD: ff.scalar_add, OpType.SCALAR_SUB: ff.scalar_sub,
              OpType.SCALAR_MULTIPLY: ff.scalar_multiply, OpType.SCALAR_TRUEDIV: ff.scalar_true_divide,
              OpType.SCALAR_FLOORDIV: ff.scalar_floor_divide}
    if op in scalar:
        return scalar[op](x, float(a[0]), name=name)
    if op == OpType.CONCAT:
        return ff.concat(ins, _axis(int(a[0]), nd), name=name)
    if op == OpType.SPLIT:
        sizes, dim, explicit = _parse_list(a[0]), _axis(int(a[1]), nd), int(a[2])
        if not explicit:
            step = sizes[0]
            n = x.dims[dim]
            sizes = [min(step, n - i) for i in range(0, n, step)]
        return ff.split(x, sizes, dim, name=name)
    if op == OpType.GETITEM:
        idx = int(a[0])
        return x[idx]
    if op == OpType.GETATTR:
        if a[0] == "size":
            return tuple(x.dims) if len(a) == 1 else x.dims[_axis(int(a[1]), nd)]
        raise NotImplementedError(a[0])
    if op == OpType.BATCH_MATMUL:
        return ff.batch_matmul(ins[0], ins[1], name=name)
    if op == OpType.TRANSPOSE:
        d0, d1 = _axis(int(a[0]), nd), _axis(int(a[1]), nd)
        perm = list(range(nd))
        perm[d0], perm[d1] = perm[d1], perm[d0]
        return ff.transpose(x, perm, name=name)
    if op == OpType.PERMUTE:
        return ff.transpose(x, _parse_list(a[0]), name=name)
    if op in (OpType.RESHAPE, OpType.VIEW):
        if a and a[0] == "dynamic":  # sizes computed in the graph (x.shape[0], x.size(1), ...)
            extra = iter(ins[1:])
            shp = [int(v) if v.lstrip("-").isdigit() else int(next(extra)) for v in a[1:]]
        else:
            shp = _parse_list(a[0])
        total = int(np.prod(x.dims))
        if -1 in shp:
            k = int(np.prod([s for s in shp if s != -1]))
            shp[shp.index(-1)] = total // k
        return ff.reshape(x, shp, name=name)
    if op == OpType.UNSQUEEZE:
        d = int(a[0])
        d = d + nd + 1 if d < 0 else d
        return ff.reshape(x, list(x.dims[:d]) + [1] + list(x.dims[d:]), name=name)
    if op == OpType.POW:
        return ff.pow(x, float(a[0]), name=name)
    if op in (OpType.MEAN, OpType.REDUCE_SUM):
        dims = [_axis(d, nd) for d in _parse_list(a[0])]
        keep = bool(int(a[1]))
        if op == OpType.MEAN:
            return ff.mean(x, dims, keep, name=name)
        return ff.reduce_sum(x, dims, keep, name=name)
    raise NotImplementedError(f"no builder for {op.name}")


class PyTorchModel:
    """reference PyTorchModel (python/flexflow/torch/model.py:2408-2607)."""

    def __init__(self, model, is_hf_model=False, input_names=None, batch_size=1, seq_length=None):
        import torch
        assert isinstance(model, torch.nn.Module)
        self.model = model
        self.is_hf_model = is_hf_model
        self.input_names = input_names
        self.batch_size = batch_size
        self.seq_length = seq_length
        self._ff_of_module: Dict[str, object] = {}

    # ------------------------------------------------------------------ tracing
    def _trace(self) -> List[IRNode]:
        import torch
        if self.is_hf_model:
            from transformers.utils.fx import symbolic_trace as hf_trace
            kw = dict(input_names=self.input_names, batch_size=self.batch_size)
            if self.seq_length is not None:
                kw["sequence_length"] = self.seq_length
            traced = hf_trace(self.model, **kw)
        else:
            traced = torch.fx.symbolic_trace(self.model)
        modules = dict(self.model.named_modules())
        nodes: List[IRNode] = []
        self._module_of_node: Dict[str, str] = {}
        for n in traced.graph.nodes:
            outs = [u.name for u in n.users]
            if n.op == "placeholder":
                nodes.append(IRNode(n.name, [], outs, OpType.INPUT, []))
            elif n.op == "output":
                res = n.args[0]
                res = list(res) if isinstance(res, (list, tuple)) else [res]
                nodes.append(IRNode(n.name, [r.name for r in res if _is_node(r)], [], OpType.OUTPUT, []))
            elif n.op == "call_module":
                m = modules[n.target]
                op, args = _enc_module(m, n)
                ins = [x.name for x in n.args if _is_node(x)]
                if op == OpType.MULTIHEAD_ATTENTION:
                    ins = ins[:3]
                nodes.append(IRNode(n.name, ins, outs, op, [str(v) for v in args]))
                self._module_of_node[n.name] = n.target
            elif n.op in ("call_function", "call_method"):
                op, ins, args = _enc_function(n)
                nodes.append(IRNode(n.name, ins, outs, op, [str(v) for v in args]))
            elif n.op == "get_attr":
                raise NotImplementedError(f"direct parameter access ({n.target}) is not supported")
            else:
                raise NotImplementedError(n.op)
        return nodes

    def torch_to_string(self) -> List[str]:
        return [n.to_string() for n in self._trace()]

    def torch_to_file(self, filename):
        with open(filename, "w") as f:
            for line in self.torch_to_string():
                f.write(line + "\n")

    def _hf_fx_available(self):
        try:
            from transformers.utils.fx import symbolic_trace  # noqa: F401
            return True
        except ImportError:  # transformers >= 5 dropped its fx tracer
            return False

    def torch_to_ff(self, ffmodel, input_tensors, verbose=False):
        if self.is_hf_model and not self._hf_fx_available():
            from .export import ExportImporter
            imp = ExportImporter(self.model, self.input_names, self.batch_size, self.seq_length)
            return imp.to_ff(ffmodel, input_tensors)
        nodes = self._trace()
        outs, built = PyTorchModel._build_nodes(nodes, ffmodel, input_tensors, verbose)
        self._ff_of_module = {self._module_of_node[k]: v for k, v in built.items() if k in self._module_of_node}
        return outs

    @staticmethod
    def file_to_ff(filename, ffmodel, input_tensors, verbose=False):
        with open(filename) as f:
            lines = [ln for ln in f.read().splitlines() if ln.strip()]
        return PyTorchModel.string_to_ff(lines, ffmodel, input_tensors, verbose)

    @staticmethod
    def string_to_ff(lines, ffmodel, input_tensors, verbose=False):
        nodes = [IRNode.from_string(ln) for ln in lines]
        return PyTorchModel._build_nodes(nodes, ffmodel, input_tensors, verbose)[0]

    @staticmethod
    def _build_nodes(nodes, ffmodel, input_tensors, verbose):
        env: Dict[str, object] = {}
        built: Dict[str, object] = {}
        it = iter(input_tensors)
        outputs = []
        for nd in nodes:
            if nd.op_type == OpType.INPUT:
                env[nd.name] = next(it)
                continue
            if nd.op_type == OpType.OUTPUT:
                outputs = [env[i] for i in nd.innodes]
                continue
            ins = [env[i] for i in nd.innodes]
            n_layers = len(ffmodel.layers)
            out = _build(ffmodel, nd, ins, nd.name)
            env[nd.name] = out
            if len(ffmodel.layers) > n_layers:
                built[nd.name] = ffmodel.layers[-1]
            if verbose:
                print(nd.to_string())
        return outputs, built

    # ------------------------------------------------------------------ weights
    def copy_weights(self, ffmodel):
        """Load the torch parameters into the compiled FFModel (layers created by torch_to_ff)."""
        import torch.nn as nn
        modules = dict(self.model.named_modules())
        for mname, L in self._ff_of_module.items():
            m = modules[mname]
            vals = []
            if isinstance(m, (nn.Linear, nn.Conv2d)):
                vals = [m.weight] + ([m.bias] if m.bias is not None else [])
            elif isinstance(m, nn.Embedding):
                vals = [m.weight]
            elif isinstance(m, nn.LayerNorm) and m.elementwise_affine:
                vals = [m.weight, m.bias]
            elif isinstance(m, nn.BatchNorm2d):
                vals = [m.weight, m.bias]
            elif isinstance(m, nn.MultiheadAttention):
                vals = [m.in_proj_weight]
                if m.in_proj_bias is not None:
                    vals.append(m.in_proj_bias)
                vals.append(m.out_proj.weight)
                if m.out_proj.bias is not None:
                    vals.append(m.out_proj.bias)
            for w, v in zip(L.weights, vals):
                w.set_weights(ffmodel, v.detach().cpu().float().numpy().reshape(w.dims))
