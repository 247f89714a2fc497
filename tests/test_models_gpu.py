"""Every model of the zoo (reference examples/cpp/*) trains on the MI355X at its full size in bf16
through the HIP kernels (hipGraph-captured steps), and the bf16 run tracks an fp32 run of the same
weights and batch (small sizes, first-step loss)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(name, dtype, steps, batch, small, graphs=True, lr=1e-3, seed=0):
    import torch
    from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel
    from flexflow_amd.models import build
    flags = ["--dtype", dtype, "--seed", str(seed)]
    if not graphs:
        flags.append("--no-hip-graphs")
    cfg = FFConfig(flags)
    cfg.batch_size = batch
    ff = FFModel(cfg)
    inputs, out, loss, mets, make_batch = build(name, ff, batch, small=small)
    ff.optimizer = AdamOptimizer(ff, lr)
    ff.compile(loss_type=loss, metrics=mets)
    arrs, lab = make_batch(np.random.default_rng(seed))
    for t, a in zip(inputs, arrs):
        t.set_tensor(ff, a)
    ff.label_tensor.set_tensor(ff, lab)
    losses = []
    for _ in range(steps):
        ff.reset_metrics()
        ff.train_step()
        losses.append(ff.get_perf_metrics().get_loss())
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return losses


@pytest.mark.parametrize("name,batch", [("alexnet", 8), ("resnet50", 4), ("resnext50", 2), ("inception_v3", 2),
                                        ("dlrm", 64), ("xdl", 64), ("candle_uno", 32), ("mlp_unify", 16),
                                        ("mnist_mlp", 32), ("transformer", 4), ("moe", 32)])
def test_zoo_model_trains_bf16(name, batch):
    # 5 steps: three eager warm-up steps, then the captured hipGraph is created and replayed
    losses = _run(name, "bf16", steps=5, batch=batch, small=False)
    assert all(np.isfinite(losses)), losses


@pytest.mark.parametrize("name", ["alexnet", "dlrm", "transformer", "mlp_unify", "moe"])
def test_zoo_bf16_tracks_fp32(name):
    a = _run(name, "bf16", steps=1, batch=8, small=True, graphs=False)
    b = _run(name, "fp32", steps=1, batch=8, small=True, graphs=False)
    np.testing.assert_allclose(a[0], b[0], rtol=5e-2, atol=1e-2)
