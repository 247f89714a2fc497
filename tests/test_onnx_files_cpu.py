"""Real .onnx files through ONNXModel without the `onnx` package: our protobuf reader
(flexflow_amd/onnx/proto.py) on the reference's own fixtures (triton/src/test/data/*.onnx, read as
data only). Expected values come from a torch fp32 evaluation of each op's ONNX semantics; the
reference's fixtures hold no expected outputs, so agreement with onnxruntime is parity-unpinned.
Fixtures whose attributes this frontend does not implement must raise NotImplementedError."""
import glob
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from flexflow_amd.core import FFConfig, FFModel, SGDOptimizer
from flexflow_amd.onnx import ONNXModel
from flexflow_amd.onnx.proto import input_shapes, load_model
from flexflow_amd.type import DataType, LossType, MetricsType

DATA = "/root/reference/triton/src/test/data"
FILES = sorted(glob.glob(os.path.join(DATA, "*.onnx")))
pytestmark = pytest.mark.skipif(not FILES, reason="reference ONNX fixtures not mounted")

UNSUPPORTED = {"avg_pool_ceil", "max_pool_ceil", "max_pool_dilations", "avg_pool_autopad"}


def _attr(node, name, default=None):
    for a in node.attribute:
        if a.name == name:
            if a.ints:
                return a.ints
            return a.i if a.i is not None else (a.f if a.f is not None else a.s)
    return default


def _expected(name, node, opset, ins, inits):
    x = [torch.from_numpy(v) for v in ins]
    op = node.op_type
    if op in ("Add", "Sub", "Mul"):
        return {"Add": x[0] + x[1], "Sub": x[0] - x[1], "Mul": x[0] * x[1]}[op]
    if op == "Tanh":
        return torch.tanh(x[0])
    if op == "Sqrt":
        return torch.sqrt(x[0])
    if op == "Reciprocal":
        return 1.0 / x[0]
    if op in ("Identity", "Cast"):
        return x[0]
    if op == "Softmax":
        ax = _attr(node, "axis", -1 if opset >= 13 else 1)
        ax = ax % x[0].dim()
        if opset < 13:
            lead = x[0].shape[:ax]
            return torch.softmax(x[0].reshape(*lead, -1), -1).reshape(x[0].shape)
        return torch.softmax(x[0], ax)
    if op == "Conv":
        w = torch.from_numpy(inits[node.input[1]])
        b = torch.from_numpy(inits[node.input[2]]) if len(node.input) > 2 else None
        p = _attr(node, "pads", [0, 0, 0, 0])
        return F.conv2d(x[0], w, b, tuple(_attr(node, "strides", [1, 1])), (p[0], p[1]))
    if op in ("MaxPool", "AveragePool"):
        k = tuple(_attr(node, "kernel_shape"))
        s = tuple(_attr(node, "strides", [1, 1]))
        p = _attr(node, "pads", [0, 0, 0, 0])
        auto = _attr(node, "auto_pad", None)
        if op == "MaxPool":
            if auto:  # SAME_UPPER, symmetric here
                tot = [max((-(-d // st) - 1) * st + kk - d, 0) for d, kk, st in zip(x[0].shape[2:], k, s)]
                p = [t // 2 for t in tot]
                xp = F.pad(x[0], (p[1], p[1], p[0], p[0]), value=float("-inf"))
                return F.max_pool2d(xp, k, s)
            return F.max_pool2d(x[0], k, s, (p[0], p[1]))
        cip = bool(_attr(node, "count_include_pad", 0))
        return F.avg_pool2d(x[0], k, s, (p[0], p[1]), count_include_pad=cip)
    raise AssertionError(op)


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(p)[:-5] for p in FILES])
def test_reference_onnx_fixture(path):
    name = os.path.basename(path)[:-5]
    model = load_model(path)
    node = model.graph.node[0]
    shapes = input_shapes(model)
    cfg = FFConfig(["--no-hip-graphs"])
    first = list(shapes.values())[0]
    cfg.batch_size = int(first[0])
    ff = FFModel(cfg)
    rng = np.random.default_rng(0)
    tensors, arrays = {}, []
    for nm, shp in shapes.items():
        tensors[nm] = ff.create_tensor([int(d) for d in shp], DataType.DT_FLOAT)
        a = rng.uniform(0.5, 2.0, [int(d) for d in shp]).astype(np.float32)  # > 0 for sqrt / reciprocal
        arrays.append(a)
    om = ONNXModel(path)
    assert om.model.graph.node[0].op_type == node.op_type
    if name in UNSUPPORTED:
        with pytest.raises(NotImplementedError):
            om.apply(ff, tensors)
        return
    out = om.apply(ff, tensors)
    inits = {t.name: t.array for t in model.graph.initializer}
    ref = _expected(name, node, om.opset, arrays, inits).numpy()
    # output shape per the ONNX spec of the node's attributes; the value-info the file declares
    # agrees except in max_pool_autopad / max_pool_order, whose declared [1,1,2,2] / [1,1,3,3] do
    # not follow from their attributes (no strides / no pads given)
    assert list(out.dims) == list(ref.shape), (out.dims, ref.shape)
    if name not in ("max_pool_autopad", "max_pool_order"):
        assert list(out.dims) == [int(d) for d in model.graph.output[0].shape]
    ff.optimizer = SGDOptimizer(ff, 0.0)
    ff.compile(loss_type=LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, metrics=[MetricsType.METRICS_MEAN_SQUARED_ERROR])
    om.load_initializers(ff)
    for (nm, t), a in zip(tensors.items(), arrays):
        t.set_tensor(ff, a)
    ff.forward()
    got = np.asarray(out.get_tensor(ff))
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)
