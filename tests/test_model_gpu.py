"""Whole-model numerics on the GPU (bf16 HIP kernels) against the CPU fp32 path of the same
framework with identical deterministic initialisation."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(device_dtype, steps=2):
    from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexflow_amd.models.bert import BertConfig, build_bert
    import flexflow_amd.runtime.executor as ex
    flags = ["--dtype", device_dtype, "--no-hip-graphs"]
    cfg = FFConfig(flags)
    bc = BertConfig(hidden=128, heads=2, layers=2, ffn=256, vocab=1000, max_pos=64, seq=64)
    B = 4
    cfg.batch_size = B
    ff = FFModel(cfg)
    ids, pos, out = build_bert(ff, B, bc)
    ff.optimizer = AdamOptimizer(ff, 1e-3)
    ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
    rng = np.random.default_rng(0)
    ids.set_tensor(ff, rng.integers(0, bc.vocab, (B, bc.seq), dtype=np.int32))
    pos.set_tensor(ff, np.tile(np.arange(bc.seq, dtype=np.int32), (B, 1)))
    ff.label_tensor.set_tensor(ff, rng.integers(0, bc.vocab, (B, bc.seq, 1), dtype=np.int32))
    losses = []
    for _ in range(steps):
        ff.reset_metrics()
        ff.forward()
        ff.zero_gradients()
        ff.backward()
        ff.update()
        losses.append(ff.get_perf_metrics().get_loss())
    w = ff.get_layer_by_name("l1_ffn1").weights[0].get_weights(ff)
    return np.array(losses), w, ff


def test_bert_bf16_gpu_matches_fp32(monkeypatch):
    l_gpu, w_gpu, ff = _run("bf16")
    assert ff.executor.device.type == "cuda"
    # CPU fp32 reference of the same model and init
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    l_cpu, w_cpu, _ = _run("fp32")
    assert np.allclose(l_gpu, l_cpu, rtol=2e-2), (l_gpu, l_cpu)
    assert np.abs(w_gpu - w_cpu).max() < 5e-3


@pytest.mark.parametrize("head_dim", [16, 32, 80, 96])
def test_attention_padded_head_dims_match_fp32(head_dim, monkeypatch):
    """Head dims without their own MFMA instance run zero-padded on the 64 / 128 kernels (no fp32
    fallback): outputs and the first update match the CPU fp32 path."""
    from flexflow_amd.core import DataType, FFConfig, FFModel, LossType, SGDOptimizer

    def run(dtype):
        cfg = FFConfig(["--dtype", dtype, "--no-hip-graphs"])
        B, S, H = 2, 48, 4
        E = H * head_dim
        cfg.batch_size = B
        ff = FFModel(cfg)
        x = ff.create_tensor([B, S, E], DataType.DT_FLOAT, name="x")
        a = ff.multihead_attention(x, x, x, E, H, name="mha")
        ff.dense(a, 8, name="head")
        ff.optimizer = SGDOptimizer(ff, 0.1)
        ff.compile(loss_type=LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE)
        rng = np.random.default_rng(head_dim)
        x.set_tensor(ff, rng.standard_normal((B, S, E)).astype(np.float32))
        ff.label_tensor.set_tensor(ff, rng.standard_normal((B, S, 8)).astype(np.float32))
        ff.forward()
        out = np.asarray(ff._get_tensor_value(ff.output_tensor()), dtype=np.float32)
        ff.zero_gradients()
        ff.backward()
        ff.update()
        w = ff.get_layer_by_name("mha").weights[0].get_weights(ff)
        return out, np.asarray(w), ff

    o_gpu, w_gpu, ff = run("bf16")
    assert ff.executor.device.type == "cuda"
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    o_cpu, w_cpu, _ = run("fp32")
    assert np.abs(o_gpu - o_cpu).max() < 3e-2 * max(1.0, np.abs(o_cpu).max())
    assert np.abs(w_gpu - w_cpu).max() < 5e-3
