"""Recommendation / tabular models: DLRM, XDL and CANDLE-Uno — the reference's
examples/cpp/{DLRM,XDL,candle_uno} and examples/python/native/dlrm.py.

MI355X sizing: the reference's DLRM default is 4 tables x 1,000,000 rows x 64 (fp16 tables,
examples/cpp/DLRM/dlrm.cc:26-42, 67-83). With 288 GB of HBM per GPU a table can be 100x that and
still sit on one device, so the search's parameter-parallel option (one table per GPU, the
embedding's `parameter`/vocab axis) is a memory *choice* rather than a necessity; `embedding_dtype`
keeps the reference's half-precision tables (bf16 here).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List

from ..core.initializers import NormInitializer, UniformInitializer
from ..type import ActiMode, AggrMode, DataType


@dataclass
class DLRMConfig:
    """examples/cpp/DLRM/dlrm.cc:26-42 defaults."""
    sparse_feature_size: int = 64
    sigmoid_bot: int = -1
    sigmoid_top: int = -1
    embedding_bag_size: int = 1
    embedding_size: List[int] = field(default_factory=lambda: [1000000] * 4)
    mlp_bot: List[int] = field(default_factory=lambda: [4, 64, 64])
    mlp_top: List[int] = field(default_factory=lambda: [64, 64, 2])
    arch_interaction_op: str = "cat"
    embedding_dtype: DataType = DataType.DT_HALF


def _mlp(ff, t, ln, sigmoid_layer, seed):
    """create_mlp (dlrm.cc:44-65): Glorot-normal-ish weights, no bias."""
    for i in range(len(ln) - 1):
        std = math.sqrt(2.0 / (ln[i + 1] + ln[i]))
        act = ActiMode.AC_MODE_SIGMOID if i == sigmoid_layer else ActiMode.AC_MODE_RELU
        t = ff.dense(t, ln[i + 1], act, use_bias=False, kernel_initializer=NormInitializer(seed + i, 0.0, std))
    return t


def _emb(ff, x, num, dim, dtype, idx):
    rng = math.sqrt(1.0 / num)
    t = ff.embedding(x, num, dim, AggrMode.AGGR_MODE_SUM, dtype=dtype,
                     kernel_initializer=UniformInitializer(1000 + idx, -rng, rng))
    return ff.cast(t, DataType.DT_FLOAT) if dtype != DataType.DT_FLOAT else t


def build_dlrm(ff, batch: int, cfg: DLRMConfig = None):
    """Returns (sparse_inputs, dense_input, output). Loss: MSE (dlrm.cc:168-175)."""
    cfg = cfg or DLRMConfig()
    sparse = [ff.create_tensor([batch, cfg.embedding_bag_size], DataType.DT_INT64) for _ in cfg.embedding_size]
    dense = ff.create_tensor([batch, cfg.mlp_bot[0]], DataType.DT_FLOAT)
    x = _mlp(ff, dense, cfg.mlp_bot, cfg.sigmoid_bot, 1)
    ly = [_emb(ff, s, n, cfg.sparse_feature_size, cfg.embedding_dtype, i)
          for i, (s, n) in enumerate(zip(sparse, cfg.embedding_size))]
    if cfg.arch_interaction_op != "cat":
        raise NotImplementedError("only 'cat' interaction (as the reference, dlrm.cc:84-101)")
    z = ff.concat([x] + ly, -1)
    p = _mlp(ff, z, cfg.mlp_top, len(cfg.mlp_top) - 2, 100)
    return sparse, dense, p


@dataclass
class XDLConfig:
    """examples/cpp/XDL/xdl.cc:24-36 defaults."""
    sparse_feature_size: int = 64
    embedding_bag_size: int = 1
    embedding_size: List[int] = field(default_factory=lambda: [1000000] * 4)
    mlp_top: List[int] = field(default_factory=lambda: [256, 256, 256, 2])


def build_xdl(ff, batch: int, cfg: XDLConfig = None):
    """Embeddings -> concat -> MLP (xdl.cc:115-141). Returns (sparse_inputs, output)."""
    cfg = cfg or XDLConfig()
    sparse = [ff.create_tensor([batch, cfg.embedding_bag_size], DataType.DT_INT64) for _ in cfg.embedding_size]
    ly = [_emb(ff, s, n, cfg.sparse_feature_size, DataType.DT_FLOAT, i)
          for i, (s, n) in enumerate(zip(sparse, cfg.embedding_size))]
    z = ff.concat(ly, -1)
    top = [z.dims[-1]] + list(cfg.mlp_top)
    p = _mlp(ff, z, top, len(top) - 2, 200)
    return sparse, p


@dataclass
class CandleUnoConfig:
    """examples/cpp/candle_uno/candle_uno.cc:24-47 defaults."""
    dense_layers: List[int] = field(default_factory=lambda: [4192] * 4)
    dense_feature_layers: List[int] = field(default_factory=lambda: [4192] * 8)
    feature_shapes: dict = field(default_factory=lambda: {"dose": 1, "cell.rnaseq": 942,
                                                           "drug.descriptors": 5270, "drug.fingerprints": 2048})
    input_features: dict = field(default_factory=lambda: {"dose1": "dose", "dose2": "dose",
                                                           "cell.rnaseq": "cell.rnaseq",
                                                           "drug1.descriptors": "drug.descriptors",
                                                           "drug1.fingerprints": "drug.fingerprints",
                                                           "drug2.descriptors": "drug.descriptors",
                                                           "drug2.fingerprints": "drug.fingerprints"})


def build_candle_uno(ff, batch: int, cfg: CandleUnoConfig = None, share_feature_encoders: bool = False):
    """Per-feature encoders (a dense stack for every cell.* / drug.* input), concat, dense head -> 1
    (candle_uno.cc:89-141; inputs visited in sorted-name order like its std::map). The reference
    builds a separate encoder per input; `share_feature_encoders` ties drug1/drug2 encoders of one
    feature type (the Uno paper's Siamese form). Returns (inputs, output). Loss: MSE."""
    cfg = cfg or CandleUnoConfig()
    inputs, encoded = [], []
    shared = {}
    for name in sorted(cfg.input_features):
        fea = cfg.input_features[name]
        x = ff.create_tensor([batch, cfg.feature_shapes[fea]], DataType.DT_FLOAT)
        inputs.append(x)
        if fea.split(".")[0] not in ("cell", "drug") or "." not in fea:
            encoded.append(x)
            continue
        t = x
        layers = shared.setdefault(fea, []) if share_feature_encoders else []
        for i, d in enumerate(cfg.dense_feature_layers):
            t = ff.dense(t, d, ActiMode.AC_MODE_RELU, use_bias=False,
                         shared_op=layers[i] if i < len(layers) else None)
            if share_feature_encoders and i >= len(layers):
                layers.append(ff.get_last_layer())
        encoded.append(t)
    t = ff.concat(encoded, -1)
    for d in cfg.dense_layers:
        t = ff.dense(t, d, ActiMode.AC_MODE_RELU, use_bias=False)
    t = ff.dense(t, 1, ActiMode.AC_MODE_NONE, use_bias=False)
    return inputs, t
