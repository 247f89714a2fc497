"""ONNX frontend on a ModelProto-shaped graph (the `onnx` package is not installed in this image:
parity with real onnx.load() output is unpinned; the graph objects below have its field layout)."""
from types import SimpleNamespace as NS

import numpy as np
import torch

from flexflow_amd.core import FFConfig, FFModel, SGDOptimizer
from flexflow_amd.onnx import ONNXModel
from flexflow_amd.type import DataType, LossType, MetricsType


def A(name, **kw):
    return NS(name=name, **kw)


def node(op, ins, outs, name="", attrs=()):
    return NS(op_type=op, input=list(ins), output=list(outs), name=name, attribute=list(attrs))


def test_onnx_cnn_mlp_parity():
    rng = np.random.default_rng(0)
    w_conv = rng.standard_normal((4, 3, 3, 3)).astype(np.float32) * 0.2
    b_conv = rng.standard_normal(4).astype(np.float32) * 0.1
    w_fc = rng.standard_normal((10, 4 * 4 * 4)).astype(np.float32) * 0.1
    b_fc = rng.standard_normal(10).astype(np.float32) * 0.1
    inits = [NS(name="wc", dims=w_conv.shape, array=w_conv), NS(name="bc", dims=b_conv.shape, array=b_conv),
             NS(name="wf", dims=w_fc.shape, array=w_fc), NS(name="bf", dims=b_fc.shape, array=b_fc)]
    nodes = [
        node("Conv", ["x", "wc", "bc"], ["c"], "conv", [A("kernel_shape", ints=[3, 3]), A("strides", ints=[1, 1]),
                                                       A("pads", ints=[1, 1, 1, 1])]),
        node("Relu", ["c"], ["r"], "relu"),
        node("MaxPool", ["r"], ["p"], "pool", [A("kernel_shape", ints=[2, 2]), A("strides", ints=[2, 2])]),
        node("Flatten", ["p"], ["f"], "flat"),
        node("Gemm", ["f", "wf", "bf"], ["g"], "fc", [A("transB", i=1)]),
        node("Softmax", ["g"], ["y"], "sm", [A("axis", i=-1)]),
    ]
    model = NS(graph=NS(node=nodes, initializer=inits, input=[NS(name="x")]))
    cfg = FFConfig(["--no-hip-graphs"])
    cfg.batch_size = 2
    ff = FFModel(cfg)
    x = ff.create_tensor([2, 3, 8, 8], DataType.DT_FLOAT)
    om = ONNXModel(model)
    out = om.apply(ff, {"x": x})
    ff.optimizer = SGDOptimizer(ff, 0.01)
    ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
    om.load_initializers(ff)
    inp = rng.standard_normal((2, 3, 8, 8)).astype(np.float32)
    x.set_tensor(ff, inp)
    ff.forward()
    got = np.asarray(out.get_tensor(ff))
    t = torch.nn.functional.conv2d(torch.from_numpy(inp), torch.from_numpy(w_conv), torch.from_numpy(b_conv), 1, 1)
    t = torch.nn.functional.max_pool2d(torch.relu(t), 2, 2).flatten(1)
    ref = torch.softmax(t @ torch.from_numpy(w_fc).t() + torch.from_numpy(b_fc), -1).numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)


def test_export_torch_roundtrip_matches_torch():
    """flexflow_amd.onnx.export.export_torch (torch.onnx.export's role; the onnx package is not
    installed) -> our ONNX reader -> FFModel reproduces the torch forward: conv/bn/pool/residual
    add/global pool/flatten/gemm/softmax, with and without exported parameters."""
    import torch
    import torch.nn as nn
    from flexflow_amd.core import FFConfig, FFModel, SGDOptimizer
    from flexflow_amd.onnx import ONNXModel
    from flexflow_amd.onnx.export import export_torch
    from flexflow_amd.type import DataType, LossType, MetricsType

    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.c1 = nn.Conv2d(3, 8, 3, padding=1)
            self.bn = nn.BatchNorm2d(8)
            self.p = nn.MaxPool2d(2, 2)
            self.c2 = nn.Conv2d(8, 8, 3, padding=1)
            self.gap = nn.AdaptiveAvgPool2d(1)
            self.fc = nn.Linear(8, 5)

        def forward(self, x):
            y = self.p(torch.relu(self.bn(self.c1(x))))
            y = y + self.c2(y)
            return torch.softmax(self.fc(torch.flatten(self.gap(y), 1)), dim=1)

    torch.manual_seed(0)
    m = Net().eval()
    x = torch.randn(4, 3, 16, 16)
    om = ONNXModel(export_torch(m, x))
    assert [n.op_type for n in om.model.graph.node] == ["Conv", "BatchNormalization", "Relu", "MaxPool", "Conv", "Add",
                                                        "GlobalAveragePool", "Flatten", "Gemm", "Softmax"]
    ff = FFModel(FFConfig(["--device", "cpu"]))
    ff.config.batch_size = 4
    t = ff.create_tensor([4, 3, 16, 16], DataType.DT_FLOAT)
    out = om.apply(ff, {"input.1": t})
    ff.optimizer = SGDOptimizer(ff, 0.0)
    ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
    om.load_initializers(ff)
    t.set_tensor(ff, x.numpy())
    ff.executor.forward(training=False)
    np.testing.assert_allclose(np.asarray(out.get_tensor(ff)), m(x).detach().numpy(), rtol=1e-4, atol=1e-5)
    # export_params=False: weights are shaped graph inputs, no initializers (FFModel initialises)
    om2 = ONNXModel(export_torch(m, x, export_params=False))
    assert not om2.inits and {"fc.weight", "c1.weight"} <= {vi.name for vi in om2.model.graph.input}
