"""flexflow_amd.models — the reference's example model zoo (examples/cpp/*, examples/python/native/*)
as FFModel builders, plus a registry used by bench.py / scripts/run_model.py / the tests.

`build(name, ff, batch, small=False)` returns (inputs, output, loss_type, metrics, make_batch) where
make_batch(rng) produces a synthetic batch (numpy arrays for every input and the label) of the
model's shapes — the reference's "synthetic data path" (no dataset files are read).
"""
from __future__ import annotations

from typing import Dict

import numpy as np

from ..type import DataType, LossType, MetricsType
from .bert import BertConfig, build_bert
from .cnn import build_alexnet, build_inception_v3, build_resnet50, build_resnext50
from .misc_models import (MoeConfig, TransformerConfig, build_mlp_unify, build_mnist_mlp, build_moe,
                          build_transformer)
from .recsys import CandleUnoConfig, DLRMConfig, XDLConfig, build_candle_uno, build_dlrm, build_xdl
from .rnn import NMTConfig, build_nmt

SCCE = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY
MSE = LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE
ACC = [MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY]


def _np_dtype(dt):
    return {DataType.DT_INT32: np.int32, DataType.DT_INT64: np.int64}.get(dt, np.float32)


def _rand_input(t, rng, hi=None):
    if t.data_type in (DataType.DT_INT32, DataType.DT_INT64):
        return rng.integers(0, hi or 2, tuple(t.dims)).astype(_np_dtype(t.data_type))
    return rng.standard_normal(tuple(t.dims)).astype(np.float32)


def build(name: str, ff, batch: int, small: bool = False, **kw):
    """Build model `name` into FFModel `ff`. small=True shrinks widths/sizes for CPU tests."""
    name = name.lower()
    hi: Dict[int, int] = {}
    positional = set()
    if name == "alexnet":
        x, out = build_alexnet(ff, batch, image_hw=67 if small else 229)
        inputs, loss, mets, ncls = [x], SCCE, ACC, 10
    elif name in ("resnet", "resnet50"):
        x, out = build_resnet50(ff, batch, image_hw=64 if small else 224, batch_norm=kw.get("batch_norm", False))
        inputs, loss, mets, ncls = [x], SCCE, ACC, 10
    elif name in ("resnext", "resnext50"):
        x, out = build_resnext50(ff, batch, image_hw=64 if small else 224, num_classes=10 if small else 1000,
                                 groups=4 if small else 32)
        inputs, loss, mets, ncls = [x], SCCE, ACC, out.dims[-1]
    elif name in ("inception", "inception_v3", "inceptionv3"):
        x, out = build_inception_v3(ff, batch, image_hw=139 if small else 299)
        inputs, loss, mets, ncls = [x], SCCE, ACC, 10
    elif name == "dlrm":
        cfg = DLRMConfig(embedding_size=[1000] * 4) if small else DLRMConfig(**kw.get("cfg", {}))
        sparse, dense, out = build_dlrm(ff, batch, cfg)
        inputs, loss, mets, ncls = sparse + [dense], MSE, [MetricsType.METRICS_MEAN_SQUARED_ERROR], None
        for t, n in zip(sparse, cfg.embedding_size):
            hi[t.guid] = n
    elif name == "xdl":
        cfg = XDLConfig(embedding_size=[1000] * 4) if small else XDLConfig()
        sparse, out = build_xdl(ff, batch, cfg)
        inputs, loss, mets, ncls = sparse, MSE, [MetricsType.METRICS_MEAN_SQUARED_ERROR], None
        for t, n in zip(sparse, cfg.embedding_size):
            hi[t.guid] = n
    elif name == "candle_uno":
        cfg = CandleUnoConfig(dense_layers=[64] * 2, dense_feature_layers=[64] * 2) if small else CandleUnoConfig()
        inputs, out = build_candle_uno(ff, batch, cfg)
        loss, mets, ncls = MSE, [MetricsType.METRICS_MEAN_SQUARED_ERROR], None
    elif name == "mlp_unify":
        inputs, out = build_mlp_unify(ff, batch, in_dim=64 if small else 1024,
                                      hidden=(128,) * 3 if small else (8192,) * 8)
        loss, mets, ncls = SCCE, ACC, out.dims[-1]
    elif name == "mnist_mlp":
        x, out = build_mnist_mlp(ff, batch)
        inputs, loss, mets, ncls = [x], SCCE, ACC, 10
    elif name == "transformer":
        cfg = TransformerConfig(hidden_size=64, num_heads=4, num_layers=2, sequence_length=16) if small \
            else TransformerConfig()
        x, out = build_transformer(ff, batch, cfg)
        inputs, loss, mets, ncls = [x], MSE, [MetricsType.METRICS_MEAN_SQUARED_ERROR], None
    elif name == "moe":
        cfg = MoeConfig(data_dims=64, hidden_size=32) if small else MoeConfig()
        x, out = build_moe(ff, batch, cfg)
        inputs, loss, mets, ncls = [x], SCCE, ACC, cfg.out_dim
    elif name in ("bert", "bert-large", "bert-base", "bert-tiny"):
        bc = BertConfig.tiny(seq=16) if small or name == "bert-tiny" else \
            (BertConfig.large() if name in ("bert", "bert-large") else BertConfig.base())
        ids, pos, out = build_bert(ff, batch, bc)
        inputs, loss, mets, ncls = [ids, pos], SCCE, ACC, bc.vocab
        hi[ids.guid] = bc.vocab
        positional.add(pos.guid)
    elif name == "nmt":
        nc = NMTConfig.small() if small else NMTConfig()
        src, dst, out = build_nmt(ff, batch, nc)
        inputs, loss, mets, ncls = [src, dst], SCCE, ACC, nc.vocab
        hi[src.guid] = nc.vocab
        hi[dst.guid] = nc.vocab
    else:
        raise KeyError(f"unknown model {name!r}")

    def make_batch(rng):
        arrs = []
        for t in inputs:
            if t.guid in positional:
                arrs.append(np.tile(np.arange(t.dims[1], dtype=np.int32), (t.dims[0], 1)))
            else:
                arrs.append(_rand_input(t, rng, hi.get(t.guid)))
        if loss == SCCE:
            lab_shape = tuple(out.dims[:-1]) + (1,)
            lab = rng.integers(0, ncls, lab_shape).astype(np.int32)
        else:
            lab = rng.standard_normal(tuple(out.dims)).astype(np.float32)
        return arrs, lab

    return inputs, out, loss, mets, make_batch


MODELS = ["alexnet", "resnet50", "resnext50", "inception_v3", "dlrm", "xdl", "candle_uno", "mlp_unify",
          "mnist_mlp", "transformer", "moe", "bert", "nmt"]

__all__ = ["build", "MODELS", "BertConfig", "build_bert", "build_alexnet", "build_resnet50", "build_resnext50",
           "build_inception_v3", "build_dlrm", "build_xdl", "build_candle_uno", "build_mlp_unify", "build_mnist_mlp",
           "build_transformer", "build_moe", "DLRMConfig", "XDLConfig", "CandleUnoConfig", "TransformerConfig",
           "MoeConfig", "NMTConfig", "build_nmt"]
