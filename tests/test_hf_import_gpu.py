"""The HuggingFace import path on the GPU: an MT5 imported through torch.export runs on the HIP
kernels in bf16 (RMS norm, dense, batched matmuls, softmax) close to the fp32 torch model, and
trains."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
transformers = pytest.importorskip("transformers")

from flexflow_amd.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer  # noqa: E402
from flexflow_amd.torch.model import PyTorchModel  # noqa: E402
from flexflow_amd.type import DataType  # noqa: E402

B, S, T, V = 4, 16, 12, 512


def test_mt5_bf16_gpu():
    torch.manual_seed(0)
    cfg = transformers.MT5Config(vocab_size=V, d_model=128, d_kv=32, d_ff=256, num_layers=2, num_decoder_layers=2,
                                 num_heads=4, relative_attention_num_buckets=8, dropout_rate=0.0)
    m = transformers.MT5ForConditionalGeneration(cfg)
    fc = FFConfig(["--dtype", "bf16", "--no-hip-graphs"])
    fc.batch_size = B
    ff = FFModel(fc)
    ins = [ff.create_tensor([B, S], DataType.DT_INT64), ff.create_tensor([B, S], DataType.DT_INT64),
           ff.create_tensor([B, T], DataType.DT_INT64)]
    outs = PyTorchModel(m, is_hf_model=True, input_names=["input_ids", "attention_mask", "decoder_input_ids"],
                        batch_size=B, seq_length=(S, T)).torch_to_ff(ff, ins)
    ff.optimizer = SGDOptimizer(ff, 0.05)
    ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
    rng = np.random.default_rng(0)
    src = rng.integers(1, V, (B, S))
    tgt = src[:, :T]
    dec = np.concatenate([np.zeros((B, 1), np.int64), tgt[:, :-1]], 1)
    ins[0].set_tensor(ff, src.astype(np.int64))
    ins[1].set_tensor(ff, np.ones((B, S), np.int64))
    ins[2].set_tensor(ff, dec.astype(np.int64))
    ff.label_tensor.set_tensor(ff, tgt.reshape(B, T, 1).astype(np.int32))
    ff.forward()
    got = np.asarray(outs[0].get_tensor(ff), dtype=np.float32)
    with torch.no_grad():
        ref = m.eval()(input_ids=torch.tensor(src), attention_mask=torch.ones(B, S, dtype=torch.long),
                       decoder_input_ids=torch.tensor(dec), use_cache=False).logits.numpy()
    rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    assert rel < 3e-2, rel
    losses = []
    for _ in range(4):
        ff.reset_metrics()
        ff.train_step()
        losses.append(ff.get_perf_metrics().get_loss())
    assert np.all(np.isfinite(losses)) and losses[-1] < losses[0], losses
