"""ONNX frontend (reference python/flexflow/onnx/model.py: ONNXModel(filename).apply(ffmodel,
input_dict) and ONNXModelKeras).

The `onnx` package is not installed in this image. The converter therefore works on any object
with the ModelProto shape — `.graph.node[*].{op_type,input,output,attribute}`,
`.graph.initializer[*].{name,dims}` and `.graph.input` — which is what `onnx.load()` returns; a
file path is accepted only when `onnx` is importable (a clear ImportError otherwise). Attributes
are read through `onnx.helper.get_attribute_value` when available and through the AttributeProto
fields (f, i, s, ints, floats) otherwise, so hand-built graphs (tests) and real models take the
same path.

Weights named by initializers become the FFModel layer weights; `load_initializers(ffmodel)` copies
their values after compile when the initializers carry data (numpy arrays or TensorProtos).
"""
from __future__ import annotations

from typing import Dict

import numpy as np

from ..type import ActiMode, DataType, PoolType


def _attr_value(a):
    try:
        from onnx import helper  # type: ignore
        return helper.get_attribute_value(a)
    except Exception:  # noqa: BLE001 - duck-typed AttributeProto
        for f in ("ints", "floats"):
            v = getattr(a, f, None)
            if v:
                return list(v)
        for f in ("i", "f", "s", "t"):
            v = getattr(a, f, None)
            if v is not None:
                return v
        return None


def _attrs(node) -> Dict[str, object]:
    return {a.name: _attr_value(a) for a in getattr(node, "attribute", [])}


def _init_array(t):
    if isinstance(t, np.ndarray):
        return t
    try:
        from onnx import numpy_helper  # type: ignore
        return numpy_helper.to_array(t)
    except Exception:  # noqa: BLE001
        return np.asarray(getattr(t, "array", None)) if getattr(t, "array", None) is not None else None


class ONNXModel:
    def __init__(self, filename_or_model):
        if isinstance(filename_or_model, (str, bytes, bytearray)):
            try:
                import onnx  # type: ignore
                filename_or_model = onnx.load(filename_or_model) if isinstance(filename_or_model, str) else \
                    onnx.load_from_string(bytes(filename_or_model))
            except ImportError:  # no onnx package: our protobuf reader (flexflow_amd/onnx/proto.py)
                from .proto import load_model
                filename_or_model = load_model(filename_or_model)
        self.model = filename_or_model
        g = self.model.graph
        self.inits = {t.name: t for t in getattr(g, "initializer", [])}
        self.opset = max([int(getattr(o, "version", 0) or 0) for o in getattr(self.model, "opset_import", [])
                          if getattr(o, "domain", "") in ("", "ai.onnx")] or [13])
        self.symbol_table: Dict[str, object] = {}
        self._layer_weights = {}  # ff layer -> [initializer names]

    def _dims(self, name):
        if name in self.inits:
            return tuple(int(d) for d in self.inits[name].dims)
        for vi in getattr(self.model.graph, "input", []):  # weight passed as a graph input
            if getattr(vi, "name", None) == name and getattr(vi, "shape", None):
                return tuple(int(d) for d in vi.shape)
        raise KeyError(f"no initializer or shaped graph input named {name}")

    # ------------------------------------------------------------------ handlers
    def handleAdd(self, ff, n):
        return ff.add(self.symbol_table[n.input[0]], self.symbol_table[n.input[1]], name=n.name or None)

    def handleSub(self, ff, n):
        return ff.subtract(self.symbol_table[n.input[0]], self.symbol_table[n.input[1]], name=n.name or None)

    def handleMul(self, ff, n):
        return ff.multiply(self.symbol_table[n.input[0]], self.symbol_table[n.input[1]], name=n.name or None)

    def handleConcat(self, ff, n):
        ax = int(_attrs(n).get("axis", 1))
        ts = [self.symbol_table[i] for i in n.input]
        return ff.concat(ts, ax if ax >= 0 else len(ts[0].dims) + ax, name=n.name or None)

    def handleSplit(self, ff, n):
        at = _attrs(n)
        x = self.symbol_table[n.input[0]]
        ax = int(at.get("axis", 0))
        sizes = list(at.get("split", [])) or [x.dims[ax] // len(n.output)] * len(n.output)
        return ff.split(x, sizes, ax, name=n.name or None)

    def _pool(self, ff, n, pt):
        at = _attrs(n)
        k = list(at["kernel_shape"])
        s = list(at.get("strides", [1, 1]))
        p = list(at.get("pads", [0, 0, 0, 0]))
        x = self.symbol_table[n.input[0]]
        auto = at.get("auto_pad", b"NOTSET")
        auto = auto.decode() if isinstance(auto, bytes) else str(auto)
        if auto in ("SAME_UPPER", "SAME_LOWER"):
            p = []
            for d, (kk, ss) in enumerate(zip(k, s)):
                size = x.dims[2 + d]
                tot = max((-(-size // ss) - 1) * ss + kk - size, 0)
                lo = tot // 2 if auto == "SAME_UPPER" else tot - tot // 2
                p.append((lo, tot - lo))
            p = [p[0][0], p[1][0], p[0][1], p[1][1]]
        elif auto == "VALID":
            p = [0, 0, 0, 0]
        if int(at.get("ceil_mode", 0)):
            raise NotImplementedError(f"{n.op_type}: ceil_mode=1 is not supported (floor output sizes only)")
        if any(int(d) != 1 for d in at.get("dilations", [1, 1])):
            raise NotImplementedError(f"{n.op_type}: dilations != 1 are not supported")
        if p[0] != p[2] or p[1] != p[3]:
            raise NotImplementedError(f"{n.op_type}: asymmetric padding {p} is not supported")
        kw = {}
        if pt == PoolType.POOL_AVG:  # ONNX default excludes the padding from the divisor
            kw["count_include_pad"] = bool(int(at.get("count_include_pad", 0)))
        return ff.pool2d(x, k[0], k[1], s[0], s[1], p[0], p[1], pt, name=n.name or None, **kw)

    def handleMaxPool(self, ff, n):
        return self._pool(ff, n, PoolType.POOL_MAX)

    def handleAveragePool(self, ff, n):
        return self._pool(ff, n, PoolType.POOL_AVG)

    def handleGlobalAveragePool(self, ff, n):
        x = self.symbol_table[n.input[0]]
        h, w = x.dims[2], x.dims[3]
        return ff.pool2d(x, h, w, 1, 1, 0, 0, PoolType.POOL_AVG, name=n.name or None)

    def handleBatchNormalization(self, ff, n):
        out = ff.batch_norm(self.symbol_table[n.input[0]], relu=False, name=n.name or None)
        self._layer_weights[ff.get_last_layer().name] = (list(ff.get_last_layer().weights), list(n.input[1:3]))
        return out

    def handleConv(self, ff, n):
        at = _attrs(n)
        x = self.symbol_table[n.input[0]]
        wd = self._dims(n.input[1])
        k = list(at.get("kernel_shape", wd[2:]))
        s = list(at.get("strides", [1, 1]))
        p = list(at.get("pads", [0, 0, 0, 0]))
        g = int(at.get("group", 1))
        out = ff.conv2d(x, wd[0], k[0], k[1], s[0], s[1], p[0], p[1], ActiMode.AC_MODE_NONE, g, len(n.input) > 2,
                        name=n.name or None)
        self._layer_weights[ff.get_last_layer().name] = (list(ff.get_last_layer().weights), list(n.input[1:]))
        return out

    def handleDropout(self, ff, n):
        rate = float(_attrs(n).get("ratio", 0.5))
        return ff.dropout(self.symbol_table[n.input[0]], rate, 0, name=n.name or None)

    def handleFlatten(self, ff, n):
        return ff.flat(self.symbol_table[n.input[0]], name=n.name or None)

    def handleGemm(self, ff, n):
        at = _attrs(n)
        wd = self._dims(n.input[1])
        trans_b = int(at.get("transB", 0))
        out_dim = wd[0] if trans_b else wd[1]
        out = ff.dense(self.symbol_table[n.input[0]], out_dim, ActiMode.AC_MODE_NONE, len(n.input) > 2,
                       name=n.name or None)
        self._layer_weights[ff.get_last_layer().name] = (list(ff.get_last_layer().weights), list(n.input[1:]) + ([] if trans_b else ["__T__"]))
        return out

    handleDense = handleGemm

    def handleMatMul(self, ff, n):
        if n.input[1] in self.inits:
            wd = self._dims(n.input[1])
            out = ff.dense(self.symbol_table[n.input[0]], wd[1], ActiMode.AC_MODE_NONE, False, name=n.name or None)
            self._layer_weights[ff.get_last_layer().name] = (list(ff.get_last_layer().weights), [n.input[1], "__T__"])
            return out
        return ff.batch_matmul(self.symbol_table[n.input[0]], self.symbol_table[n.input[1]], name=n.name or None)

    def handleRelu(self, ff, n):
        return ff.relu(self.symbol_table[n.input[0]], name=n.name or None)

    def handleSigmoid(self, ff, n):
        return ff.sigmoid(self.symbol_table[n.input[0]], name=n.name or None)

    def handleTanh(self, ff, n):
        return ff.tanh(self.symbol_table[n.input[0]], name=n.name or None)

    def handleSoftmax(self, ff, n):
        x = self.symbol_table[n.input[0]]
        at = _attrs(n)
        ax = int(at.get("axis", -1 if self.opset >= 13 else 1))
        ax = ax if ax >= 0 else len(x.dims) + ax
        if self.opset < 13 and ax != len(x.dims) - 1:
            # opset < 13: softmax over the flattened trailing dims [ax:] (one 2-D row per prefix)
            lead = [int(d) for d in x.dims[:ax]]
            flat = ff.reshape(x, lead + [int(np.prod(x.dims[ax:]))])
            return ff.reshape(ff.softmax(flat, len(lead), name=n.name or None), list(x.dims))
        return ff.softmax(x, ax, name=n.name or None)

    def handleSqrt(self, ff, n):
        return ff.pow(self.symbol_table[n.input[0]], 0.5, name=n.name or None)

    def handleReciprocal(self, ff, n):
        return ff.pow(self.symbol_table[n.input[0]], -1.0, name=n.name or None)

    def handleExp(self, ff, n):
        return ff.exp(self.symbol_table[n.input[0]], name=n.name or None)

    def handleReshape(self, ff, n):
        x = self.symbol_table[n.input[0]]
        shape = self.symbol_table.get(n.input[1])
        if shape is None and n.input[1] in self.inits:
            shape = _init_array(self.inits[n.input[1]])
        shp = [int(v) for v in np.asarray(shape).reshape(-1)]
        shp = [x.dims[i] if v == 0 else v for i, v in enumerate(shp)]
        if -1 in shp:
            k = int(np.prod([v for v in shp if v != -1]))
            shp[shp.index(-1)] = int(np.prod(x.dims)) // k
        return ff.reshape(x, shp, name=n.name or None)

    def handleTranspose(self, ff, n):
        perm = list(_attrs(n)["perm"])
        return ff.transpose(self.symbol_table[n.input[0]], perm, name=n.name or None)

    def handleCast(self, ff, n):
        return self.symbol_table[n.input[0]]

    def handleIdentity(self, ff, n):
        return self.symbol_table[n.input[0]]

    def handleUnsqueeze(self, ff, n):
        x = self.symbol_table[n.input[0]]
        axes = list(_attrs(n).get("axes", []))
        dims = list(x.dims)
        for a in sorted(axes):
            dims.insert(a, 1)
        return ff.reshape(x, dims, name=n.name or None)

    def handleConstant(self, ff, n):
        v = _attrs(n).get("value")
        return _init_array(v)

    def handlePad(self, ff, n):
        raise NotImplementedError("Pad: fold the padding into the following Conv/Pool (as the reference)")

    # ------------------------------------------------------------------ driver
    def apply(self, ffmodel, input_dict):
        """input_dict: graph-input name -> FFModel tensor. Returns the output tensor."""
        self.symbol_table = dict(input_dict)
        out = None
        for n in self.model.graph.node:
            h = getattr(self, "handle" + n.op_type, None)
            if h is None:
                raise NotImplementedError(f"ONNX op {n.op_type} is not supported")
            res = h(ffmodel, n)
            if isinstance(res, (list, tuple)):
                for name, r in zip(n.output, res):
                    self.symbol_table[name] = r
            else:
                self.symbol_table[n.output[0]] = res
            out = res
        return out

    def load_initializers(self, ffmodel):
        """Copy initializer values into the compiled model's weights (when the graph carries them)."""
        # weight Parameters are kept (not layer names): graph substitutions at compile may replace
        # the layer (e.g. Conv+Relu fusion) but the fused layer shares the same Parameters
        for lname, (weights, names) in self._layer_weights.items():
            transpose = "__T__" in names
            vals = [_init_array(self.inits[nm]) for nm in names if nm != "__T__" and nm in self.inits]
            for i, (w, v) in enumerate(zip(weights, vals)):
                if v is None:
                    continue
                if transpose and i == 0:
                    v = v.T
                w.set_weights(ffmodel, np.ascontiguousarray(v, dtype=np.float32).reshape(w.dims))


class ONNXModelKeras(ONNXModel):
    """Models exported by keras2onnx (reference ONNXModelKeras, python/flexflow/onnx/model.py):
    a Dense layer arrives as MatMul(x, W[in, out]) followed by Add(., b); the pair becomes one
    dense layer with bias (weights transposed into our [out, in] layout)."""

    def __init__(self, filename_or_model, ffconfig=None, ffmodel=None):
        super().__init__(filename_or_model)
        self.ffconfig, self.ffmodel = ffconfig, ffmodel

    def _dense_pairs(self):
        nodes = list(self.model.graph.node)
        users = {}
        for n in nodes:
            for i in n.input:
                users.setdefault(i, []).append(n)
        pairs = {}
        for n in nodes:
            if n.op_type != "MatMul" or n.input[1] not in self.inits or len(self._dims(n.input[1])) != 2:
                continue
            us = users.get(n.output[0], [])
            if len(us) != 1 or us[0].op_type != "Add":
                continue
            add = us[0]
            other = add.input[1] if add.input[0] == n.output[0] else add.input[0]
            if other in self.inits and tuple(self._dims(other)) == (self._dims(n.input[1])[1],):
                pairs[id(n)] = (add, other)
        return pairs

    def apply(self, ffmodel, input_dict):
        pairs = self._dense_pairs()
        skip = {id(a) for a, _ in pairs.values()}
        self.symbol_table = dict(input_dict)
        out = None
        for n in self.model.graph.node:
            if id(n) in skip:
                continue
            if id(n) in pairs:
                add, bias = pairs[id(n)]
                wd = self._dims(n.input[1])
                res = ffmodel.dense(self.symbol_table[n.input[0]], wd[1], ActiMode.AC_MODE_NONE, True,
                                    name=n.name or None)
                L = ffmodel.get_last_layer()
                self._layer_weights[L.name] = (list(L.weights), [n.input[1], bias, "__T__"])
                self.symbol_table[add.output[0]] = res
                out = res
                continue
            h = getattr(self, "handle" + n.op_type, None)
            if h is None:
                raise NotImplementedError(f"ONNX op {n.op_type} is not supported")
            res = h(ffmodel, n)
            if isinstance(res, (list, tuple)):
                for name, r in zip(n.output, res):
                    self.symbol_table[name] = r
            else:
                self.symbol_table[n.output[0]] = res
            out = res
        return out
