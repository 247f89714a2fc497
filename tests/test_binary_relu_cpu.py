"""Residual add + ReLU fused into one element-wise pass (Executor._plan_binary_relu): the plan
fires on ResNet's bottleneck blocks and training matches the unfused executor."""
import numpy as np

from flexflow_amd.core import FFConfig, FFModel, SGDOptimizer
from flexflow_amd.models import build


def _run(monkeypatch, fused):
    if fused:
        monkeypatch.delenv("FF_NO_BINARY_RELU", raising=False)
    else:
        monkeypatch.setenv("FF_NO_BINARY_RELU", "1")
    cfg = FFConfig(["--device", "cpu"])
    cfg.batch_size = 4
    ff = FFModel(cfg)
    inputs, out, loss, mets, make_batch = build("resnet50", ff, 4, small=True)
    ff.optimizer = SGDOptimizer(ff, 0.01)
    ff.compile(loss_type=loss, metrics=mets)
    n = sum(1 for L in ff.layers if ff.executor.ctx[L.name].extra.get("fused_relu"))
    rng = np.random.default_rng(0)
    losses = []
    for _ in range(2):
        arrs, lab = make_batch(rng)
        for t, a in zip(inputs, arrs):
            t.set_tensor(ff, a)
        ff.label_tensor.set_tensor(ff, lab)
        ff.reset_metrics()
        ff.forward()
        ff.zero_gradients()
        ff.backward()
        ff.update()
        losses.append(ff.get_perf_metrics().get_loss())
    return n, np.array(losses)


def test_binary_relu_fusion_matches_unfused(monkeypatch):
    n1, l1 = _run(monkeypatch, True)
    n0, l0 = _run(monkeypatch, False)
    assert n1 > 0 and n0 == 0
    np.testing.assert_allclose(l1, l0, rtol=1e-5)
