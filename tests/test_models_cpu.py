"""Every model of the zoo (reference examples/cpp/*, examples/python/native/*) builds, compiles,
and trains a step on CPU with finite loss; the loss goes down over a few SGD steps on a fixed batch
for the small classifiers."""
import numpy as np
import pytest

from flexflow_amd.core import FFConfig, FFModel, SGDOptimizer
from flexflow_amd.models import MODELS, build


def _run(name, steps=2, batch=2, lr=0.01):
    cfg = FFConfig(["--no-hip-graphs"])
    cfg.batch_size = batch
    ff = FFModel(cfg)
    inputs, out, loss, mets, make_batch = build(name, ff, batch, small=True)
    ff.optimizer = SGDOptimizer(ff, lr)
    ff.compile(loss_type=loss, metrics=mets)
    rng = np.random.default_rng(0)
    arrs, lab = make_batch(rng)
    for t, a in zip(inputs, arrs):
        t.set_tensor(ff, a)
    ff.label_tensor.set_tensor(ff, lab)
    losses = []
    for _ in range(steps):
        ff.reset_metrics()
        ff.forward()
        ff.zero_gradients()
        ff.backward()
        ff.update()
        losses.append(ff.get_perf_metrics().get_loss())
    return losses


@pytest.mark.parametrize("name", [m for m in MODELS if m not in ("inception_v3", "resnext50", "resnet50")])
def test_model_trains(name):
    losses = _run(name)
    assert all(np.isfinite(losses)), losses


@pytest.mark.parametrize("name", ["resnet50", "resnext50", "inception_v3"])
def test_big_cnn_builds_and_steps(name):
    losses = _run(name, steps=1, batch=1)
    assert np.isfinite(losses[0])


@pytest.mark.parametrize("name", ["mnist_mlp", "alexnet"])
def test_loss_decreases(name):
    losses = _run(name, steps=5, batch=4, lr=0.05)
    assert losses[-1] < losses[0], losses
