"""HuggingFace import through torch.export (flexflow_amd/torch/export.py; the reference traced HF
models with transformers.utils.fx, gone in transformers 5): an MT5 built from a config (random
init, no download) becomes an FFModel whose logits equal the torch model's, and it trains."""
import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")

from flexflow_amd.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer  # noqa: E402
from flexflow_amd.torch.model import PyTorchModel  # noqa: E402
from flexflow_amd.type import DataType, OperatorType  # noqa: E402

B, S, T, V = 2, 12, 10, 256


def _mt5():
    torch.manual_seed(0)
    cfg = transformers.MT5Config(vocab_size=V, d_model=64, d_kv=16, d_ff=128, num_layers=2, num_decoder_layers=2,
                                 num_heads=4, relative_attention_num_buckets=8, dropout_rate=0.0)
    return transformers.MT5ForConditionalGeneration(cfg)


def _import(model):
    fc = FFConfig(["--device", "cpu"])
    fc.batch_size = B
    ff = FFModel(fc)
    ins = [ff.create_tensor([B, S], DataType.DT_INT64), ff.create_tensor([B, S], DataType.DT_INT64),
           ff.create_tensor([B, T], DataType.DT_INT64)]
    hf = PyTorchModel(model, is_hf_model=True, input_names=["input_ids", "attention_mask", "decoder_input_ids"],
                      batch_size=B, seq_length=(S, T))
    outs = hf.torch_to_ff(ff, ins)
    return ff, ins, outs


def test_mt5_logits_match_torch():
    m = _mt5()
    ff, ins, outs = _import(m)
    kinds = {L.op_type for L in ff.layers}
    assert OperatorType.OP_RMS_NORM in kinds and OperatorType.OP_BATCHMATMUL in kinds
    ff.optimizer = SGDOptimizer(ff, 0.01)
    ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
    rng = np.random.default_rng(0)
    ids, dec = rng.integers(1, V, (B, S)), rng.integers(1, V, (B, T))
    ins[0].set_tensor(ff, ids.astype(np.int64))
    ins[1].set_tensor(ff, np.ones((B, S), np.int64))
    ins[2].set_tensor(ff, dec.astype(np.int64))
    ff.forward()
    got = np.asarray(outs[0].get_tensor(ff))
    with torch.no_grad():
        ref = m.eval()(input_ids=torch.tensor(ids), attention_mask=torch.ones(B, S, dtype=torch.long),
                       decoder_input_ids=torch.tensor(dec), use_cache=False).logits.numpy()
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max())


def test_mt5_trains():
    ff, ins, outs = _import(_mt5())
    ff.optimizer = SGDOptimizer(ff, 0.05)
    ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
    rng = np.random.default_rng(1)
    src = rng.integers(1, V, (B, S))
    tgt = src[:, :T]  # copy task
    dec = np.concatenate([np.zeros((B, 1), np.int64), tgt[:, :-1]], 1)
    ins[0].set_tensor(ff, src.astype(np.int64))
    ins[1].set_tensor(ff, np.ones((B, S), np.int64))
    ins[2].set_tensor(ff, dec.astype(np.int64))
    ff.label_tensor.set_tensor(ff, tgt.reshape(B, T, 1).astype(np.int32))
    losses = []
    for _ in range(4):
        ff.reset_metrics()
        ff.train_step()
        losses.append(ff.get_perf_metrics().get_loss())
    assert np.all(np.isfinite(losses)) and losses[-1] < losses[0], losses
