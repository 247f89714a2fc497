"""torch.nn.Module -> ONNX without the onnx package (torch.onnx.export needs it, and it is not in
this image). The reference's ONNX examples start from `torch.onnx.export(model, input,
"x.onnx")` (examples/python/onnx/*_pt.py); `export_torch` plays that role: the module is traced
with torch.fx and every node is emitted as the ONNX operator the torch exporter would produce
(opset 11): Linear -> Gemm(transB=1), Conv2d -> Conv, BatchNorm2d -> BatchNormalization,
pooling, activations, Flatten / view, residual Add, Concat, Dropout, Softmax.

The first input is named "input.1" (the torch exporter's name, which the reference examples feed:
`onnx_model.apply(ffmodel, {"input.1": input1})`). `export_params=False` leaves the weights out,
like the reference's exports, so FFModel initialises them.
"""
from __future__ import annotations

import operator
from typing import Dict, List, Optional

import numpy as np

from .proto import make_model_bytes


def _pair(v):
    return list(v) if isinstance(v, (tuple, list)) else [v, v]


class _TorchExporter:
    def __init__(self, export_params: bool):
        self.nodes = []
        self.inits: Dict[str, np.ndarray] = {}
        self.export_params = export_params
        self.weight_inputs: Dict[str, list] = {}
        self.k = 0

    def out(self, base):
        self.k += 1
        return f"{base}_{self.k}"

    def emit(self, op, ins, attrs=None, base=None):
        o = self.out(base or op)
        self.nodes.append((op, list(ins), [o], attrs or {}))
        return o

    def param(self, name, t):
        if t is None:
            return None
        if self.export_params:
            self.inits[name] = t.detach().cpu().float().numpy()
        else:  # declared as a shaped graph input (as torch.onnx.export does), values left out
            self.weight_inputs[name] = list(t.shape)
        return name

    def const(self, base, arr):
        nm = self.out(base)
        self.inits[nm] = np.asarray(arr)
        return nm

    # ------------------------------------------------------------------ modules
    def module(self, name, m, xs):
        import torch.nn as nn
        x = xs[0]
        if isinstance(m, nn.Linear):
            ins = [x, self.param(f"{name}.weight", m.weight)]
            if m.bias is not None:
                ins.append(self.param(f"{name}.bias", m.bias))
            return self.emit("Gemm", ins, {"transB": 1, "alpha": 1.0, "beta": 1.0})
        if isinstance(m, nn.Conv2d):
            if any(d != 1 for d in _pair(m.dilation)):
                raise NotImplementedError("export_torch: dilated Conv2d")
            if isinstance(m.padding, str):
                raise NotImplementedError("export_torch: string padding")
            ph, pw = _pair(m.padding)
            ins = [x, self.param(f"{name}.weight", m.weight)]
            if m.bias is not None:
                ins.append(self.param(f"{name}.bias", m.bias))
            return self.emit("Conv", ins, {"kernel_shape": _pair(m.kernel_size), "strides": _pair(m.stride),
                                           "pads": [ph, pw, ph, pw], "group": int(m.groups),
                                           "dilations": [1, 1]})
        if isinstance(m, nn.BatchNorm2d):
            ins = [x, self.param(f"{name}.weight", m.weight), self.param(f"{name}.bias", m.bias),
                   self.param(f"{name}.running_mean", m.running_mean), self.param(f"{name}.running_var", m.running_var)]
            return self.emit("BatchNormalization", ins, {"epsilon": float(m.eps), "momentum": 1.0 - float(m.momentum)})
        if isinstance(m, (nn.MaxPool2d, nn.AvgPool2d)):
            if getattr(m, "ceil_mode", False):
                raise NotImplementedError("export_torch: ceil_mode pooling")
            ph, pw = _pair(m.padding)
            op = "MaxPool" if isinstance(m, nn.MaxPool2d) else "AveragePool"
            attrs = {"kernel_shape": _pair(m.kernel_size), "strides": _pair(m.stride or m.kernel_size),
                     "pads": [ph, pw, ph, pw]}
            if op == "AveragePool":
                attrs["count_include_pad"] = int(bool(m.count_include_pad))
            return self.emit(op, [x], attrs)
        if isinstance(m, nn.AdaptiveAvgPool2d):
            if tuple(_pair(m.output_size)) != (1, 1):
                raise NotImplementedError("export_torch: AdaptiveAvgPool2d to a size other than 1x1")
            return self.emit("GlobalAveragePool", [x])
        if isinstance(m, (nn.ReLU, nn.Sigmoid, nn.Tanh)):
            return self.emit({nn.ReLU: "Relu", nn.Sigmoid: "Sigmoid", nn.Tanh: "Tanh"}[type(m)], [x])
        if isinstance(m, nn.Softmax):
            return self.emit("Softmax", [x], {"axis": int(m.dim if m.dim is not None else 1)})
        if isinstance(m, nn.Dropout):
            return self.emit("Dropout", [x], {"ratio": float(m.p)})
        if isinstance(m, nn.Flatten):
            if m.end_dim != -1:
                raise NotImplementedError("export_torch: Flatten with end_dim")
            return self.emit("Flatten", [x], {"axis": int(m.start_dim)})
        if isinstance(m, nn.Identity):
            return self.emit("Identity", [x])
        raise NotImplementedError(f"export_torch: module {type(m).__name__}")

    # ------------------------------------------------------------------ functions / methods
    def function(self, target, args, kwargs, env, shape_of):
        import torch
        import torch.nn.functional as F

        def v(a):
            return env[a.name] if hasattr(a, "name") and a.name in env else a

        name = getattr(target, "__name__", str(target))
        if target in (operator.add, operator.iadd, torch.add) or name in ("add", "add_"):
            return self.emit("Add", [v(args[0]), v(args[1])])
        if target in (operator.mul, operator.imul, torch.mul) or name in ("mul", "mul_"):
            return self.emit("Mul", [v(args[0]), v(args[1])])
        if target in (operator.sub, torch.sub) or name == "sub":
            return self.emit("Sub", [v(args[0]), v(args[1])])
        if target in (F.relu, torch.relu) or name in ("relu", "relu_"):
            return self.emit("Relu", [v(args[0])])
        if target in (torch.sigmoid,) or name == "sigmoid":
            return self.emit("Sigmoid", [v(args[0])])
        if target in (torch.tanh,) or name == "tanh":
            return self.emit("Tanh", [v(args[0])])
        if target in (F.softmax, torch.softmax) or name == "softmax":
            dim = kwargs.get("dim", args[1] if len(args) > 1 else -1)
            return self.emit("Softmax", [v(args[0])], {"axis": int(dim)})
        if target is torch.flatten or name == "flatten":
            start = int(kwargs.get("start_dim", args[1] if len(args) > 1 else 0))
            return self.emit("Flatten", [v(args[0])], {"axis": start})
        if target is torch.cat or name in ("cat", "concat"):
            dim = int(kwargs.get("dim", args[1] if len(args) > 1 else 0))
            return self.emit("Concat", [v(a) for a in args[0]], {"axis": dim})
        if name in ("view", "reshape"):
            dims = args[1:] if not isinstance(args[1], (tuple, list)) else args[1]
            shp = [int(d) if isinstance(d, int) else -1 for d in dims]
            return self.emit("Reshape", [v(args[0]), self.const("shape", np.asarray(shp, np.int64))])
        if target in (F.max_pool2d,):
            k = _pair(args[1] if len(args) > 1 else kwargs["kernel_size"])
            s = _pair(kwargs.get("stride", args[2] if len(args) > 2 else k) or k)
            return self.emit("MaxPool", [v(args[0])], {"kernel_shape": k, "strides": s, "pads": [0, 0, 0, 0]})
        if target in (F.dropout,):
            return self.emit("Dropout", [v(args[0])], {"ratio": float(kwargs.get("p", 0.5))})
        raise NotImplementedError(f"export_torch: function {name}")


def export_torch(model, example_input, path: Optional[str] = None, export_params: bool = True,
                 input_names: Optional[List[str]] = None) -> bytes:
    """Serialize `model` (traced with torch.fx at `example_input`'s shapes) as ONNX opset 11."""
    import torch
    import torch.fx as fx
    xs = list(example_input) if isinstance(example_input, (tuple, list)) else [example_input]
    names = list(input_names or ["input.1"] + [f"input.{i + 2}" for i in range(len(xs) - 1)])
    gm = fx.symbolic_trace(model)
    modules = dict(gm.named_modules())
    ex = _TorchExporter(export_params)
    env: Dict[str, str] = {}
    shapes: Dict[str, list] = {}
    # shapes of every node, from one real forward (for the declared graph output)
    from torch.fx.passes.shape_prop import ShapeProp
    ShapeProp(gm).propagate(*[x.detach() for x in xs])
    ins = {}
    k = 0
    outputs = {}
    for n in gm.graph.nodes:
        if n.op == "placeholder":
            env[n.name] = names[k]
            ins[names[k]] = list(xs[k].shape)
            k += 1
        elif n.op == "call_module":
            env[n.name] = ex.module(n.target, modules[n.target], [env[a.name] for a in n.args if hasattr(a, "name")])
        elif n.op in ("call_function", "call_method"):
            tgt = n.target if n.op == "call_function" else _Method(n.target)
            env[n.name] = ex.function(tgt, n.args, n.kwargs, env, shapes)
        elif n.op == "output":
            res = n.args[0]
            res = list(res) if isinstance(res, (tuple, list)) else [res]
            for r in res:
                tm = r.meta.get("tensor_meta")
                outputs[env[r.name]] = list(tm.shape) if tm is not None else []
        else:
            raise NotImplementedError(f"export_torch: fx op {n.op} ({n.target})")
    ins.update(ex.weight_inputs)
    data = make_model_bytes(ex.nodes, ins, outputs, ex.inits, opset=11, name=type(model).__name__)
    if path:
        with open(path, "wb") as f:
            f.write(data)
    return data


class _Method:
    """A call_method target, named like the function it mirrors."""

    def __init__(self, name):
        self.__name__ = name

    def __eq__(self, other):
        return False

    __hash__ = object.__hash__
