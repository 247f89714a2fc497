"""MLP_Unify, the attention-encoder Transformer and the mixture-of-experts model — the reference's
examples/cpp/{MLP_Unify,Transformer,mixture_of_experts} and examples/python/native/
{mnist_mlp,multi_head_attention}.py.

The reference's MLP_Unify benchmark runs forward only (examples/cpp/MLP_Unify/mlp.cc:73-77 has
backward/update commented out); ours trains it like every other model.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence

from ..type import ActiMode, DataType


def build_mlp_unify(ff, batch: int, in_dim: int = 1024, hidden: Sequence[int] = (8192,) * 8):
    """Two parallel dense towers over two inputs, summed, softmax (mlp.cc:38-57)."""
    x1 = ff.create_tensor([batch, in_dim], DataType.DT_FLOAT)
    x2 = ff.create_tensor([batch, in_dim], DataType.DT_FLOAT)
    t1, t2 = x1, x2
    for i, h in enumerate(hidden):
        act = ActiMode.AC_MODE_NONE if i + 1 == len(hidden) else ActiMode.AC_MODE_RELU
        t1 = ff.dense(t1, h, act, use_bias=False)
        t2 = ff.dense(t2, h, act, use_bias=False)
    t = ff.softmax(ff.add(t1, t2))
    return [x1, x2], t


def build_mnist_mlp(ff, batch: int, hidden: Sequence[int] = (512, 512), num_classes: int = 10):
    """examples/python/native/mnist_mlp.py: 784 -> 512 -> 512 -> 10 -> softmax."""
    x = ff.create_tensor([batch, 784], DataType.DT_FLOAT)
    t = x
    for h in hidden:
        t = ff.dense(t, h, ActiMode.AC_MODE_RELU)
    t = ff.softmax(ff.dense(t, num_classes))
    return x, t


@dataclass
class TransformerConfig:
    """examples/cpp/Transformer/transformer.cc:78-84 defaults."""
    hidden_size: int = 1024
    embedding_size: int = 1024
    num_heads: int = 16
    num_layers: int = 12
    sequence_length: int = 512


def build_transformer(ff, batch: int, cfg: TransformerConfig = None):
    """Stack of (self-attention -> dense relu -> dense) encoders with no bias, then dense -> 1;
    MSE loss on a [batch, seq, 1] label (transformer.cc:33-45, 134-163)."""
    cfg = cfg or TransformerConfig()
    x = ff.create_tensor([batch, cfg.sequence_length, cfg.hidden_size], DataType.DT_FLOAT)
    t = x
    kd = cfg.hidden_size // cfg.num_heads
    for _ in range(cfg.num_layers):
        t = ff.multihead_attention(t, t, t, cfg.hidden_size, cfg.num_heads, kd, kd)
        t = ff.dense(t, cfg.hidden_size, ActiMode.AC_MODE_RELU, use_bias=False)
        t = ff.dense(t, cfg.hidden_size, ActiMode.AC_MODE_NONE, use_bias=False)
    t = ff.dense(t, 1, ActiMode.AC_MODE_NONE, use_bias=False)
    return x, t


@dataclass
class MoeConfig:
    """examples/cpp/mixture_of_experts/moe.h:30-45 defaults (MNIST-sized)."""
    data_dims: int = 28 * 28
    out_dim: int = 10
    num_exp: int = 5
    num_select: int = 2
    alpha: float = 2.0
    lambda_bal: float = 0.04
    hidden_size: int = 28 * 28
    num_encoder_layers: int = 0
    num_attention_heads: int = 16


def build_moe(ff, batch: int, cfg: MoeConfig = None):
    """moe (gate dense -> top-k -> group_by -> expert denses -> aggregate) -> dense relu
    (moe.cc:150-173); with num_encoder_layers > 0 the create_moe_encoder stack of
    LN(attention + x), LN(moe + x) blocks (moe.cc:100-131) on a [batch, seq, hidden] input."""
    cfg = cfg or MoeConfig()
    if cfg.num_encoder_layers:
        x = ff.create_tensor([batch, cfg.data_dims // cfg.hidden_size or 1, cfg.hidden_size], DataType.DT_FLOAT)
        t = x
        kd = cfg.hidden_size // cfg.num_attention_heads
        for _ in range(cfg.num_encoder_layers):
            a = ff.multihead_attention(t, t, t, cfg.hidden_size, cfg.num_attention_heads, kd, kd)
            t = ff.layer_norm(ff.add(a, t), [-1], True, 1e-5)
            m = ff.moe(t, cfg.num_exp, cfg.num_select, cfg.hidden_size, cfg.alpha, cfg.lambda_bal)
            t = ff.layer_norm(ff.add(m, t), [-1], True, 1e-5)
        t = ff.flat(t)
    else:
        x = ff.create_tensor([batch, cfg.data_dims], DataType.DT_FLOAT)
        t = ff.moe(x, cfg.num_exp, cfg.num_select, cfg.hidden_size, cfg.alpha, cfg.lambda_bal)
    t = ff.dense(t, cfg.out_dim, ActiMode.AC_MODE_RELU)
    t = ff.softmax(t)
    return x, t


def model_names() -> List[str]:
    return ["alexnet", "resnet50", "resnext50", "inception_v3", "dlrm", "xdl", "candle_uno", "mlp_unify",
            "mnist_mlp", "transformer", "moe", "bert"]
