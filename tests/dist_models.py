"""Tiny models + strategies shared by the multi-process (gloo) parallelism tests and the
single-process references they are compared against."""
import json
import os

import numpy as np

from flexflow_amd.core import (ActiMode, AggrMode, DataType, FFConfig, FFModel, LossType, MetricsType,
                               PoolType, SGDOptimizer)
from flexflow_amd.pcg.strategy import OpConfig

B = 8


def build(name, ff):
    rng = np.random.default_rng(7)
    feeds = {}
    if name in ("mlp", "mlp_tp", "mlp_place", "mlp_hybrid"):
        x = ff.create_tensor([B, 16], DataType.DT_FLOAT, name="x")
        t = ff.dense(x, 32, ActiMode.AC_MODE_RELU, name="d1")
        t = ff.dense(t, 24, name="d2")
        t = ff.dense(t, 10, name="d3")
        ff.softmax(t, name="sm")
        feeds[x] = rng.standard_normal((B, 16)).astype(np.float32)
        lab = rng.integers(0, 10, (B, 1)).astype(np.int32)
        loss = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY
    elif name == "parops":
        # explicit parallel ops: hidden activation repartitioned along features, combined back
        x = ff.create_tensor([B, 16], DataType.DT_FLOAT, name="x")
        t = ff.dense(x, 32, ActiMode.AC_MODE_RELU, name="d1")
        t = ff.repartition(t, 1, 2, name="rp")
        t = ff.relu(t, name="r2")
        t = ff.combine(t, 1, name="cb")
        t = ff.dense(t, 10, name="d3")
        ff.softmax(t, name="sm")
        feeds[x] = rng.standard_normal((B, 16)).astype(np.float32)
        lab = rng.integers(0, 10, (B, 1)).astype(np.int32)
        loss = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY
    elif name in ("attn", "attn_tp"):
        x = ff.create_tensor([B, 6, 16], DataType.DT_FLOAT, name="x")
        a = ff.multihead_attention(x, x, x, 16, 4, name="mha")
        t = ff.layer_norm(ff.add(a, x, name="res"), [-1], name="ln")
        t = ff.dense(t, 8, name="d")
        feeds[x] = rng.standard_normal((B, 6, 16)).astype(np.float32)
        lab = rng.standard_normal((B, 6, 8)).astype(np.float32)
        loss = LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE
    elif name in ("cnn", "cnn_attr"):
        x = ff.create_tensor([B, 3, 8, 8], DataType.DT_FLOAT, name="x")
        t = ff.conv2d(x, 4, 3, 3, 1, 1, 1, 1, ActiMode.AC_MODE_RELU, name="c1")
        t = ff.pool2d(t, 2, 2, 2, 2, 0, 0, name="p1")
        t = ff.conv2d(t, 6, 3, 3, 1, 1, 1, 1, name="c2")
        t = ff.flat(t, name="flat")
        t = ff.dense(t, 10, name="fc")
        ff.softmax(t, name="sm")
        feeds[x] = rng.standard_normal((B, 3, 8, 8)).astype(np.float32)
        lab = rng.integers(0, 10, (B, 1)).astype(np.int32)
        loss = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY
    elif name in ("emb", "emb_vocab"):
        ids = ff.create_tensor([B, 3], DataType.DT_INT32, name="ids")
        e = ff.embedding(ids, 40, 12, AggrMode.AGGR_MODE_SUM, name="emb")
        t = ff.dense(e, 5, name="d")
        ff.softmax(t, name="sm")
        feeds[ids] = rng.integers(0, 40, (B, 3)).astype(np.int32)
        lab = rng.integers(0, 5, (B, 1)).astype(np.int32)
        loss = LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY
    else:
        raise KeyError(name)
    return feeds, lab, loss


def strategy(name, ff, world):
    """Hand-written strategies exercising every transfer kind."""
    L = {l.name: l for l in ff.layers}

    def cfg(lname, degs, devs=None):
        n = len(L[lname].impl.axis_sizes())
        d = list(degs) + [1] * (n - len(degs))
        P = int(np.prod(d))
        return OpConfig(tuple(d), tuple(devs if devs is not None else range(P)))

    W = world
    if name == "mlp_tp":
        # column-parallel d1 (out channels), row-parallel d2 (reduction -> partial), dp d3/softmax
        return {"x": cfg("x", [W]), "d1": cfg("d1", [1, W]), "d2": cfg("d2", [1, 1, W]),
                "d3": cfg("d3", [W]), "sm": cfg("sm", [W])}
    if name == "mlp_place":
        # operator placement (inter-op parallelism): each layer on its own device
        return {"x": cfg("x", [1], [0]), "d1": cfg("d1", [1], [0]), "d2": cfg("d2", [1], [1 % W]),
                "d3": cfg("d3", [1], [0]), "sm": cfg("sm", [W])}
    if name == "mlp_hybrid":
        return {"x": cfg("x", [W]), "d1": cfg("d1", [W]), "d2": cfg("d2", [1, W]), "d3": cfg("d3", [1, 1, W]),
                "sm": cfg("sm", [1], [W - 1])}
    if name == "attn_tp":
        return {"x": cfg("x", [W]), "mha": cfg("mha", [1, 1, 1, W]), "res": cfg("res", [W]),
                "ln": cfg("ln", [W, 1]), "d": cfg("d", [1, 1, W])}
    if name == "cnn_attr":
        return {"x": cfg("x", [1, 1, W]), "c1": cfg("c1", [1, 1, W]), "p1": cfg("p1", [1, 1, W]),
                "c2": cfg("c2", [1, W]), "flat": cfg("flat", [W]), "fc": cfg("fc", [1, W]), "sm": cfg("sm", [W])}
    if name == "emb_vocab":
        return {"ids": cfg("ids", [W]), "emb": cfg("emb", [1, 1, W]), "d": cfg("d", [W]), "sm": cfg("sm", [W])}
    return None  # data parallel


def run(name, world, strategy_file=None, steps=2, lr=0.05):
    flags = []
    if strategy_file:
        flags += ["--import-strategy", strategy_file]
    elif world > 1:
        flags += ["--only-data-parallel"]
    if os.environ.get("FF_TEST_DTYPE"):
        flags += ["--dtype", os.environ["FF_TEST_DTYPE"]]
    cfg = FFConfig(flags)
    cfg.batch_size = B
    ff = FFModel(cfg)
    feeds, lab, loss = build(name, ff)
    ff.optimizer = SGDOptimizer(ff, lr)
    ff.compile(loss_type=loss, metrics=[MetricsType.METRICS_ACCURACY])
    for t, v in feeds.items():
        t.set_tensor(ff, v)
    ff.label_tensor.set_tensor(ff, lab)
    for _ in range(steps):
        ff.forward()
        ff.zero_gradients()
        ff.backward()
        ff.update()
    out = {}
    for l in ff.layers:
        for i, w in enumerate(l.weights):
            out[f"{l.name}.{i}"] = w.get_weights(ff)
    out["__output__"] = ff._get_tensor_value(ff.output_tensor())
    return out

