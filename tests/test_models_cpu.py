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


def test_bias_grad_fusion_into_layernorm_matches_unfused(monkeypatch):
    """The out-projection and FFN2 bias gradients summed inside the following LayerNorm's backward
    (executor._plan_bias_grad_fusion) train exactly like the separate column-reduction pass."""
    import numpy as np
    from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexflow_amd.models.bert import BertConfig, build_bert

    def run(fused):
        if fused:
            monkeypatch.delenv("FF_NO_BIAS_FUSION", raising=False)
        else:
            monkeypatch.setenv("FF_NO_BIAS_FUSION", "1")
        cfg = FFConfig(["--device", "cpu"])
        bc = BertConfig.tiny(16)
        cfg.batch_size = 2
        ff = FFModel(cfg)
        ids, pos, _ = build_bert(ff, 2, bc)
        ff.optimizer = AdamOptimizer(ff, 1e-3)
        ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
        n = sum(1 for c in ff.executor.ctx.values() if c.extra.get("bias_grad_fused"))
        rng = np.random.default_rng(0)
        ids.set_tensor(ff, rng.integers(0, bc.vocab, (2, 16), dtype=np.int32))
        pos.set_tensor(ff, np.tile(np.arange(16, dtype=np.int32), (2, 1)))
        ff.label_tensor.set_tensor(ff, rng.integers(0, bc.vocab, (2, 16, 1), dtype=np.int32))
        for _ in range(2):
            ff.train_step()
        ws = {f"{L.name}.{i}": np.asarray(w.get_weights(ff)) for L in ff.layers for i, w in enumerate(L.weights)}
        return n, ws

    n1, a = run(True)
    n0, b = run(False)
    assert n0 == 0 and n1 == 2 * BertConfig.tiny(16).layers  # out-proj + FFN2 of every layer
    for k in a:
        np.testing.assert_allclose(a[k], b[k], rtol=1e-5, atol=1e-6, err_msg=k)


def test_dact_fusion_into_consumer_dgrad_matches_unfused(monkeypatch):
    """FFN2's dgrad GEMM applying FFN1's GELU' and summing FFN1's bias gradient
    (executor._plan_dact_fusion -> kernels.gemm_dact) trains like the separate bias_act_bwd pass."""
    import numpy as np
    from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexflow_amd.models.bert import BertConfig, build_bert

    def run(fused):
        if fused:
            monkeypatch.delenv("FF_NO_DACT_FUSION", raising=False)
        else:
            monkeypatch.setenv("FF_NO_DACT_FUSION", "1")
        cfg = FFConfig(["--device", "cpu"])
        bc = BertConfig.tiny(16)
        cfg.batch_size = 2
        ff = FFModel(cfg)
        ids, pos, _ = build_bert(ff, 2, bc)
        ff.optimizer = AdamOptimizer(ff, 1e-3)
        ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
        n = sum(1 for c in ff.executor.ctx.values() if c.extra.get("dact_fused"))
        rng = np.random.default_rng(0)
        ids.set_tensor(ff, rng.integers(0, bc.vocab, (2, 16), dtype=np.int32))
        pos.set_tensor(ff, np.tile(np.arange(16, dtype=np.int32), (2, 1)))
        ff.label_tensor.set_tensor(ff, rng.integers(0, bc.vocab, (2, 16, 1), dtype=np.int32))
        for _ in range(2):
            ff.train_step()
        ws = {f"{L.name}.{i}": np.asarray(w.get_weights(ff)) for L in ff.layers for i, w in enumerate(L.weights)}
        return n, ws

    n1, a = run(True)
    n0, b = run(False)
    assert n0 == 0 and n1 == BertConfig.tiny(16).layers  # FFN1 of every layer (the MLM transform feeds a LayerNorm)
    for k in a:
        np.testing.assert_allclose(a[k], b[k], rtol=1e-5, atol=1e-6, err_msg=k)


def test_partial_gradient_zeroing_matches_full(monkeypatch):
    """Arenas lay out accumulated gradients first and zero_gradients() clears only that prefix (the
    overwritten GEMM gradients need no clearing): training matches zeroing the whole arena."""
    import numpy as np
    from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexflow_amd.models.bert import BertConfig, build_bert

    def run(full):
        if full:
            monkeypatch.setenv("FF_ZERO_ALL_GRADS", "1")
        else:
            monkeypatch.delenv("FF_ZERO_ALL_GRADS", raising=False)
        cfg = FFConfig(["--device", "cpu"])
        bc = BertConfig.tiny(16)
        cfg.batch_size = 2
        ff = FFModel(cfg)
        ids, pos, _ = build_bert(ff, 2, bc)
        ff.optimizer = AdamOptimizer(ff, 1e-3)
        ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
        ars = [a for a in ff.executor.arenas.values() if a.size]
        rng = np.random.default_rng(0)
        for _ in range(3):
            ids.set_tensor(ff, rng.integers(0, bc.vocab, (2, 16), dtype=np.int32))
            pos.set_tensor(ff, np.tile(np.arange(16, dtype=np.int32), (2, 1)))
            ff.label_tensor.set_tensor(ff, rng.integers(0, bc.vocab, (2, 16, 1), dtype=np.int32))
            ff.train_step()
        return ars, {f"{L.name}.{i}": np.asarray(w.get_weights(ff)) for L in ff.layers for i, w in enumerate(L.weights)}

    ars, a = run(False)
    assert all(0 < ar.acc_end < ar.size for ar in ars)  # a real prefix: GEMM weights are not cleared
    _, b = run(True)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_sparse_embedding_sgd_matches_dense(monkeypatch):
    """Plain SGD updates DLRM's embedding tables only on the rows the step's ids touched (and
    clears just those gradient rows; executor._sparse_update -> kernels.sgd_sparse_rows), exactly
    like the dense update over the whole table."""
    def run(sparse):
        if sparse:
            monkeypatch.delenv("FF_SPARSE_EMB", raising=False)
        else:
            monkeypatch.setenv("FF_SPARSE_EMB", "0")
        cfg = FFConfig(["--no-hip-graphs"])
        cfg.batch_size = 4
        ff = FFModel(cfg)
        inputs, out, loss, mets, make_batch = build("dlrm", ff, 4, small=True)
        ff.optimizer = SGDOptimizer(ff, 0.05)
        ff.compile(loss_type=loss, metrics=mets)
        n = sum(len(v) for v in ff.executor._sparse_plan(ff.optimizer).values())
        rng = np.random.default_rng(0)
        for _ in range(3):  # a new batch (new rows, repeated ids) every step
            arrs, lab = make_batch(rng)
            for t, a in zip(inputs, arrs):
                t.set_tensor(ff, a)
            ff.label_tensor.set_tensor(ff, lab)
            ff.train_step()
        ws = [np.asarray(w.get_weights(ff)) for L in ff.layers for w in L.weights]  # names carry guids
        return n, ws

    n1, a = run(True)
    n0, b = run(False)
    assert n1 > 0 and n0 == 0 and len(a) == len(b)
    for k, (x, y) in enumerate(zip(a, b)):
        np.testing.assert_allclose(x, y, rtol=1e-6, atol=1e-7, err_msg=str(k))


def test_sparse_embedding_sgd_two_backwards_then_update(monkeypatch):
    """forward/backward twice (different ids), then one update: rows touched only by the first
    backward must move exactly as with the dense update (the row-sparse plan falls back to dense
    when more than one backward ran since the last update)."""
    def run(sparse):
        if sparse:
            monkeypatch.delenv("FF_SPARSE_EMB", raising=False)
        else:
            monkeypatch.setenv("FF_SPARSE_EMB", "0")
        cfg = FFConfig(["--no-hip-graphs"])
        cfg.batch_size = 4
        ff = FFModel(cfg)
        inputs, out, loss, mets, make_batch = build("dlrm", ff, 4, small=True)
        ff.optimizer = SGDOptimizer(ff, 0.05)
        ff.compile(loss_type=loss, metrics=mets)
        rng = np.random.default_rng(1)
        for step in range(2):
            ff.zero_gradients()
            for _ in range(2):
                arrs, lab = make_batch(rng)
                for t, a in zip(inputs, arrs):
                    t.set_tensor(ff, a)
                ff.label_tensor.set_tensor(ff, lab)
                ff.forward()
                ff.backward()
            ff.update()
        return [np.asarray(w.get_weights(ff)) for L in ff.layers for w in L.weights]

    a, b = run(True), run(False)
    for k, (x, y) in enumerate(zip(a, b)):
        np.testing.assert_allclose(x, y, rtol=1e-6, atol=1e-7, err_msg=str(k))


def test_sparse_plan_follows_momentum_change():
    cfg = FFConfig(["--no-hip-graphs"])
    cfg.batch_size = 4
    ff = FFModel(cfg)
    _, _, loss, mets, _ = build("dlrm", ff, 4, small=True)
    ff.optimizer = SGDOptimizer(ff, 0.05)
    ff.compile(loss_type=loss, metrics=mets)
    assert ff.executor._sparse_plan(ff.optimizer)
    ff.optimizer.momentum = 0.9
    assert not ff.executor._sparse_plan(ff.optimizer)


def test_bert_padded_vocab_matches_unpadded():
    """BertConfig.pad_vocab_multiple: the MLM decoder is padded (1000 -> 1024 columns) with a
    -1e9 bias on the padded logits and the real rows initialised as in the unpadded model, so the
    losses of three Adam steps equal the unpadded model's (bench.py pads 30522 -> 30528)."""
    import numpy as np

    from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexflow_amd.models.bert import BertConfig, build_bert

    def run(pad):
        cfg = FFConfig(["--dtype", "fp32"])
        cfg.batch_size = 2
        ff = FFModel(cfg)
        bc = BertConfig(hidden=64, heads=2, layers=1, ffn=128, vocab=1000, max_pos=32, seq=32)
        bc.pad_vocab_multiple = pad
        ids, pos, out = build_bert(ff, 2, bc)
        ff.optimizer = AdamOptimizer(ff, 1e-3)
        ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
        rng = np.random.default_rng(0)
        ids.set_tensor(ff, rng.integers(0, 1000, (2, 32), dtype=np.int32))
        pos.set_tensor(ff, np.tile(np.arange(32, dtype=np.int32), (2, 1)))
        ff.label_tensor.set_tensor(ff, rng.integers(0, 1000, (2, 32, 1), dtype=np.int32))
        losses = []
        for _ in range(3):
            ff.reset_metrics()
            ff.forward()
            ff.zero_gradients()
            ff.backward()
            ff.update()
            losses.append(ff.get_perf_metrics().get_loss())
        return losses, out

    ref, _ = run(0)
    pad, out = run(64)
    assert out.dims[-1] == 1024
    np.testing.assert_allclose(pad, ref, rtol=1e-5)
