"""Keras graph -> ONNX, in keras2onnx's conventions (the converter the reference's keras_exp runs
on tf.keras models, python/flexflow/keras_exp/models/model.py: `keras2onnx.convert_keras`).

Without TensorFlow in the image, keras_exp models are written with our keras layers
(flexflow_amd.keras.layers); this exporter walks that graph — nested models inlined — and emits
the ONNX a keras2onnx export of the same model would hold: Dense -> MatMul(x, W[in, out]) + Add(b)
(+ activation node), Conv2D -> Conv (+ activation), pooling, Flatten, Concat, elementwise merges,
Dropout, Reshape, BatchNormalization, Softmax. Weights are drawn from each layer's initializer
(Glorot-uniform kernels, zero biases), as a freshly built tf.keras model would carry them.
Graph inputs are named "input_<key>" (the reference's keying of its input dict).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

from ..keras import layers as KL
from ..onnx.proto import make_model_bytes
from ..type import ActiMode


class _Exporter:
    def __init__(self, seed=0):
        self.nodes: List[Tuple] = []
        self.inits: Dict[str, np.ndarray] = {}
        self.rng = np.random.default_rng(seed)
        self.n = 0

    def name(self, base):
        self.n += 1
        return f"{base}_{self.n}"

    def init(self, base, arr):
        nm = self.name(base)
        self.inits[nm] = np.ascontiguousarray(arr)
        return nm

    def glorot(self, shape, fan_in, fan_out):
        lim = np.sqrt(6.0 / (fan_in + fan_out))
        return self.rng.uniform(-lim, lim, shape).astype(np.float32)

    def node(self, op, ins, attrs=None, base=None):
        out = self.name(base or op.lower())
        self.nodes.append((op, list(ins), [out], attrs or {}))
        return out

    def act(self, x, act):
        if isinstance(act, ActiMode):
            act = {ActiMode.AC_MODE_NONE: None, ActiMode.AC_MODE_RELU: "relu", ActiMode.AC_MODE_SIGMOID: "sigmoid",
                   ActiMode.AC_MODE_TANH: "tanh", ActiMode.AC_MODE_GELU: "gelu"}[act]
        a = {None: None, "linear": None, "relu": "Relu", "sigmoid": "Sigmoid", "tanh": "Tanh",
             "softmax": "Softmax"}.get(act, act)
        if a is None:
            return x
        if a not in ("Relu", "Sigmoid", "Tanh", "Softmax"):
            raise NotImplementedError(f"keras_exp export: activation {act!r}")
        return self.node(a, [x], {"axis": -1} if a == "Softmax" else None)

    # ---------------------------------------------------------------- layers
    def layer(self, L, xs, in_shapes):
        if isinstance(L, KL.Dense):
            fin = in_shapes[0][-1]
            w = self.init("kernel", self.glorot((fin, L.units), fin, L.units))
            y = self.node("MatMul", [xs[0], w])
            if getattr(L, "use_bias", True):
                y = self.node("Add", [y, self.init("bias", np.zeros(L.units, np.float32))])
            return [self.act(y, "softmax" if L.softmax else L.activation)]
        if isinstance(L, KL.Activation):
            return [self.act(xs[0], L.activation)]
        if isinstance(L, KL.Conv2D):
            cin = in_shapes[0][0]
            if L.groups != 1:
                raise NotImplementedError("keras_exp export: grouped Conv2D")
            kh, kw = L.kernel
            w = self.init("kernel", self.glorot((L.filters, cin, kh, kw), cin * kh * kw, L.filters * kh * kw))
            ins = [xs[0], w]
            if getattr(L, "use_bias", True):
                ins.append(self.init("bias", np.zeros(L.filters, np.float32)))
            ph, pw = L.pads
            y = self.node("Conv", ins, {"kernel_shape": [kh, kw], "strides": list(L.strides),
                                        "pads": [ph, pw, ph, pw]})
            return [self.act(y, L.activation)]
        if isinstance(L, KL.Pooling2D):
            op = "MaxPool" if isinstance(L, KL.MaxPooling2D) else "AveragePool"
            ph, pw = L.pads
            return [self.node(op, [xs[0]], {"kernel_shape": list(L.pool), "strides": list(L.strides),
                                            "pads": [ph, pw, ph, pw]})]
        if isinstance(L, KL.Flatten):
            return [self.node("Flatten", [xs[0]], {"axis": 1})]
        if isinstance(L, KL.Concatenate):
            ax = L.axis if L.axis >= 0 else len(in_shapes[0]) + 1 + L.axis
            return [self.node("Concat", xs, {"axis": int(ax)})]
        if isinstance(L, (KL.Add, KL.Subtract, KL.Multiply)):
            op = {KL.Add: "Add", KL.Subtract: "Sub", KL.Multiply: "Mul"}[type(L)]
            y = xs[0]
            for x in xs[1:]:
                y = self.node(op, [y, x])
            return [y]
        if isinstance(L, KL.Dropout):
            return [self.node("Dropout", [xs[0]], {"ratio": float(L.rate)})]
        if isinstance(L, KL.Reshape):
            shp = self.init("shape", np.asarray([-1] + list(L.target_shape), np.int64))
            return [self.node("Reshape", [xs[0], shp])]
        if isinstance(L, KL.BatchNormalization):
            c = in_shapes[0][0]
            ins = [xs[0], self.init("gamma", np.ones(c, np.float32)), self.init("beta", np.zeros(c, np.float32)),
                   self.init("mean", np.zeros(c, np.float32)), self.init("var", np.ones(c, np.float32))]
            return [self.node("BatchNormalization", ins, {"epsilon": 1e-3})]
        raise NotImplementedError(f"keras_exp export: layer {type(L).__name__}")


def export_keras_model(model, input_keys, batch_size, seed=0, opset=13) -> bytes:
    """ONNX bytes of a flexflow_amd.keras functional model (nested models inlined)."""
    from ..keras.models import Model as KModel
    ex = _Exporter(seed)
    env: Dict[int, str] = {}
    shapes: Dict[int, tuple] = {}
    inputs = {}
    for key, t in zip(input_keys, model._inputs):
        nm = f"input_{key}"
        env[id(t)] = nm
        shapes[id(t)] = t.shape
        inputs[nm] = [batch_size] + list(t.shape)

    def run(m, bindings):
        def val(t):
            if id(t) in bindings:
                return bindings[id(t)]
            L = t.layer
            call = next(ci for ci, outs in enumerate(L.outbound) if any(o is t for o in outs))
            xs = [val(x) for x in L.inbound[call]]
            in_shapes = [x.shape for x in L.inbound[call]]
            if isinstance(L, KModel):
                outs = run(L, {id(a): v for a, v in zip(L._inputs, xs)})
            else:
                outs = ex.layer(L, xs, in_shapes)
            for o, v in zip(L.outbound[call], outs):
                bindings[id(o)] = v
            return bindings[id(t)]
        return [val(o) for o in m._outputs]

    outs = run(model, env)
    final = {o: [batch_size] + list(t.shape) for o, t in zip(outs, model._outputs)}
    return make_model_bytes(ex.nodes, inputs, final, ex.inits, opset=opset, name=model.name)
