"""Python side of the C API (csrc/capi/flexflow_c.cc -> libflexflow_c.so).

Every C entry point forwards its plain arguments (ints, floats, strings, raw host pointers as
integers) to one function here, so the C layer stays a thin, uniform trampoline and all semantics
live in one place next to the FFModel API they map onto (reference src/c/flexflow_c.cc, 144
functions over the C++ FFModel; this covers the model-building / training / tensor-IO subset).
"""
from __future__ import annotations

import ctypes

import numpy as np

from .config import FFConfig
from .core import AdamOptimizer, FFModel, SGDOptimizer
from .type import ActiMode, AggrMode, CompMode, DataType, LossType, MetricsType, PoolType


def _name(n):
    return n if n else None


# ---------------------------------------------------------------- config
def config_create():
    return FFConfig([])


def config_parse_args(cfg, args):
    cfg.parse_args(list(args))


def config_get(cfg, key):
    return int(getattr(cfg, key))


def config_set_batch_size(cfg, b):
    cfg.batch_size = int(b)


# ---------------------------------------------------------------- model
def model_create(cfg):
    return FFModel(cfg)


def model_compile(m, loss, metrics, comp_mode):
    m.compile(loss_type=LossType(loss), metrics=[MetricsType(x) for x in metrics], comp_mode=CompMode(comp_mode))


def model_call(m, method):
    getattr(m, method)()


def sgd_create(m, lr, momentum, nesterov, wd):
    return SGDOptimizer(m, lr, momentum, bool(nesterov), wd)


def adam_create(m, alpha, b1, b2, wd, eps):
    return AdamOptimizer(m, alpha, b1, b2, wd, eps)


def model_set_optimizer(m, opt):
    m.optimizer = opt


def optimizer_set_lr(opt, lr):
    opt.set_learning_rate(lr)


def model_label_tensor(m):
    return m.label_tensor


def model_perf(m, what):
    pm = m.get_perf_metrics()
    return float(pm.get_accuracy() if what == 0 else pm.get_loss())


# ---------------------------------------------------------------- tensors
def tensor_create(m, dims, dtype, create_grad):
    return m.create_tensor(list(dims), DataType(dtype), bool(create_grad))


def tensor_dims(t):
    return list(int(d) for d in t.dims)


_NP = {DataType.DT_FLOAT: (np.float32, ctypes.c_float), DataType.DT_INT32: (np.int32, ctypes.c_int32),
       DataType.DT_INT64: (np.int64, ctypes.c_int64)}


def tensor_set_data(m, t, addr, n, dtype):
    npdt, cdt = _NP[DataType(dtype)]
    buf = np.ctypeslib.as_array(ctypes.cast(addr, ctypes.POINTER(cdt)), shape=(n,))
    t.set_tensor(m, buf.copy().reshape(t.dims).astype(npdt))


def tensor_get_data(m, t, addr, n):
    v = np.asarray(t.get_tensor(m), dtype=np.float32).reshape(-1)
    if v.size != n:
        raise ValueError(f"buffer has {n} elements, tensor has {v.size}")
    out = np.ctypeslib.as_array(ctypes.cast(addr, ctypes.POINTER(ctypes.c_float)), shape=(n,))
    out[:] = v


# ---------------------------------------------------------------- layers
def add_dense(m, x, out_dim, acti, use_bias, name):
    return m.dense(x, out_dim, ActiMode(acti), bool(use_bias), name=_name(name))


def add_conv2d(m, x, oc, kh, kw, sh, sw, ph, pw, acti, groups, use_bias, name):
    return m.conv2d(x, oc, kh, kw, sh, sw, ph, pw, ActiMode(acti), groups, bool(use_bias), name=_name(name))


def add_pool2d(m, x, kh, kw, sh, sw, ph, pw, pool_type, acti, name):
    return m.pool2d(x, kh, kw, sh, sw, ph, pw, PoolType(pool_type), ActiMode(acti), name=_name(name))


def add_embedding(m, x, num, dim, aggr, name):
    return m.embedding(x, num, dim, AggrMode(aggr), name=_name(name))


def add_layer_norm(m, x, axes, affine, eps, name):
    return m.layer_norm(x, list(axes), bool(affine), eps, name=_name(name))


def add_unary(m, op, x, name):
    return getattr(m, op)(x, name=_name(name))


def add_scalar(m, op, x, s, name):
    return getattr(m, op)(x, s, name=_name(name))


def add_binary(m, op, a, b, name):
    return getattr(m, op)(a, b, name=_name(name))


def add_concat(m, xs, axis, name):
    return m.concat(list(xs), axis, name=_name(name))


def add_softmax(m, x, axis, name):
    return m.softmax(x, axis, name=_name(name))


def add_dropout(m, x, rate, seed, name):
    return m.dropout(x, rate, seed, name=_name(name))


def add_reshape(m, x, shape, name):
    return m.reshape(x, list(shape), name=_name(name))


def add_transpose(m, x, perm, name):
    return m.transpose(x, list(perm), name=_name(name))


def add_batch_norm(m, x, relu, name):
    return m.batch_norm(x, bool(relu), name=_name(name))


def add_mha(m, q, k, v, embed, heads, kdim, vdim, dropout, bias, name):
    return m.multihead_attention(q, k, v, embed, heads, kdim, vdim, dropout, bool(bias), name=_name(name))


def add_embedding_typed(m, x, num, dim, aggr, dtype, name):
    return m.embedding(x, num, dim, AggrMode(aggr), dtype=DataType(dtype), name=_name(name))


def add_split(m, x, sizes, axis, name):
    return m.split(x, list(sizes), axis, name=_name(name))


def add_top_k(m, x, k, sorted_, name):
    return m.top_k(x, k, bool(sorted_), name=_name(name))


def add_group_by(m, data, assign, n, alpha, name):
    return m.group_by(data, assign, n, alpha, name=_name(name))


def add_aggregate(m, xs, n, lambda_bal, spec, name):
    f = m.aggregate_spec if spec else m.aggregate
    return f(list(xs), n, lambda_bal, name=_name(name))


def add_moe(m, x, num_exp, num_select, hidden, alpha, lambda_bal):
    return m.moe(x, num_exp, num_select, hidden, alpha, lambda_bal)


def add_reduce(m, op, x, dims, keepdims, name):
    return getattr(m, op)(x, list(dims), bool(keepdims), name=_name(name))


def add_gather(m, x, index, dim, name):
    return m.gather(x, index, dim, name=_name(name))


def add_cast(m, x, dtype, name):
    return m.cast(x, DataType(dtype), name=_name(name))


def add_rms_norm(m, x, eps, name):
    return m.rms_norm(x, eps, name=_name(name))


def add_reverse(m, x, axis, name):
    return m.reverse(x, axis, name=_name(name))


def model_print_layers(m, idx):
    m.print_layers(idx)


def model_num_layers(m):
    return len(m._non_input_layers())


def model_search_algo(m):
    return str((m.search_report or {}).get("algo") or "")
