#!/usr/bin/env python3
"""BERT-Large training losses for a few steps (fixed seeds): run under two settings and compare,
e.g. FF_ATTN_BWD=2 (bias gradient summed by the QKV Linear's backward) vs the default (summed
inside the attention backward). usage: bert_loss_check.py [batch=16] [steps=4] [layers=24]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType  # noqa: E402
from flexflow_amd.models.bert import BertConfig, build_bert  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
layers = int(sys.argv[3]) if len(sys.argv) > 3 else 24
torch.manual_seed(0)
cfg = FFConfig(["--dtype", "bf16", "--no-hip-graphs"])
cfg.batch_size = B
ff = FFModel(cfg)
bc = BertConfig.large(512)
bc.layers = layers
ids, pos, _ = build_bert(ff, B, bc)
ff.optimizer = AdamOptimizer(ff, 1e-4)
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
torch.cuda.synchronize()
print("losses", " ".join(f"{v:.6f}" for v in losses))
