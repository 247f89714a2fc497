"""torch.fx frontend (reference python/flexflow/torch/model.py + examples/python/pytorch/*):
.ff IR round trip and forward-pass parity with the source nn.Module after copy_weights."""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from flexflow_amd.core import FFConfig, FFModel, SGDOptimizer
from flexflow_amd.torch import PyTorchModel
from flexflow_amd.type import DataType, LossType, MetricsType


class MLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.linear1 = nn.Linear(32, 64)
        self.linear2 = nn.Linear(64, 64)
        self.linear3 = nn.Linear(64, 10)
        self.relu = nn.ReLU()
        self.softmax = nn.Softmax(dim=-1)

    def forward(self, x):
        y = self.relu(self.linear1(x))
        y = self.relu(self.linear2(y)) + y * 0.5
        return self.softmax(self.linear3(y))


class CNN(nn.Module):
    def __init__(self):
        super().__init__()
        self.c1 = nn.Conv2d(3, 8, 3, 1, 1)
        self.c2 = nn.Conv2d(3, 8, 5, 1, 2)
        self.c3 = nn.Conv2d(16, 16, 3, 2, 1)
        self.pool = nn.MaxPool2d(2, 2)
        self.gap = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(16, 10)

    def forward(self, x):
        t = torch.cat([F.relu(self.c1(x)), torch.tanh(self.c2(x))], dim=1)
        t = self.pool(t)
        t = F.relu(self.c3(t))
        t = self.gap(t)
        t = torch.flatten(t, 1)
        return self.fc(t)


class Block(nn.Module):
    def __init__(self, e=32, h=4):
        super().__init__()
        self.attn = nn.MultiheadAttention(e, h, batch_first=True)
        self.ln1 = nn.LayerNorm(e)
        self.ff1 = nn.Linear(e, 64)
        self.ff2 = nn.Linear(64, e)
        self.ln2 = nn.LayerNorm(e)

    def forward(self, x):
        a = self.attn(x, x, x)[0]
        x = self.ln1(x + a)
        f = self.ff2(F.gelu(self.ff1(x)))
        y = self.ln2(x + f)
        return y.permute(0, 2, 1).reshape(x.shape[0], -1)


def _convert(module, in_shape, via_file=None, loss=LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE):
    cfg = FFConfig(["--no-hip-graphs"])
    cfg.batch_size = in_shape[0]
    ff = FFModel(cfg)
    x = ff.create_tensor(list(in_shape), DataType.DT_FLOAT)
    pm = PyTorchModel(module)
    if via_file:
        pm.torch_to_file(via_file)
        outs = PyTorchModel.file_to_ff(via_file, ff, [x])
        pm.torch_to_ff(FFModel(cfg), [FFModel(cfg).create_tensor(list(in_shape), DataType.DT_FLOAT)])
    else:
        outs = pm.torch_to_ff(ff, [x])
    ff.optimizer = SGDOptimizer(ff, 0.01)
    ff.compile(loss_type=loss, metrics=[MetricsType.METRICS_MEAN_SQUARED_ERROR])
    return ff, pm, x, outs[0]


@pytest.mark.parametrize("cls,shape", [(MLP, (4, 32)), (CNN, (2, 3, 16, 16)), (Block, (2, 8, 32))])
def test_forward_parity(cls, shape):
    torch.manual_seed(0)
    m = cls().eval()
    ff, pm, x, out = _convert(m, shape)
    pm.copy_weights(ff)
    inp = torch.randn(*shape)
    x.set_tensor(ff, inp.numpy())
    ff.forward()
    got = np.asarray(out.get_tensor(ff))
    ref = m(inp).detach().numpy()
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4)


def test_ff_file_round_trip(tmp_path):
    m = MLP()
    p = tmp_path / "mlp.ff"
    lines = PyTorchModel(m).torch_to_string()
    assert lines[0].split("; ")[3] == "INPUT" and any("; LINEAR; 64; " in ln for ln in lines)
    ff, pm, x, out = _convert(m, (4, 32), via_file=str(p))
    assert p.read_text().splitlines() == lines
    kinds = [L.op_type.name for L in ff.layers]
    assert kinds.count("OP_LINEAR") == 3 and "OP_SOFTMAX" in kinds
    # the loaded model trains
    x.set_tensor(ff, np.random.default_rng(0).standard_normal((4, 32)).astype(np.float32))
    ff.label_tensor.set_tensor(ff, np.zeros((4, 10), np.float32))
    ff.forward(); ff.zero_gradients(); ff.backward(); ff.update()
    assert np.isfinite(ff.get_perf_metrics().get_loss())
