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


# ================================================================ reference-complete surface
# (csrc/capi/flexflow_c.h; every name below is called by exactly one C entry point)
def config_parse_default(cfg):
    import sys
    cfg.parse_args(list(sys.argv[1:]))


def config_attr(cfg, key, default):
    return int(getattr(cfg, key, default))


def model_prefetch(m):
    m.prefetch()


def add_binary_named(m, op, a, b, name):
    return getattr(m, op)(a, b, name=_name(name))


def add_reduce_ref(m, op, x, axes, keepdims, name):
    return getattr(m, op)(x, list(axes), bool(keepdims), name=_name(name))


def add_conv2d_init(m, x, oc, kh, kw, sh, sw, ph, pw, acti, groups, use_bias, shared, kinit, binit, name):
    return m.conv2d(x, oc, kh, kw, sh, sw, ph, pw, ActiMode(acti), groups, bool(use_bias), shared_op=shared,
                    kernel_initializer=kinit, bias_initializer=binit, name=_name(name))


def add_dense_init(m, x, out_dim, acti, use_bias, dtype, shared, kinit, binit, reg_type, reg_lambda, name):
    from .type import RegularizerMode
    reg = None
    if int(reg_type) in (RegularizerMode.REG_MODE_L1.value, RegularizerMode.REG_MODE_L2.value) and reg_lambda:
        from .keras.regularizers import L1, L2
        reg = L2(reg_lambda) if int(reg_type) == RegularizerMode.REG_MODE_L2.value else L1(reg_lambda)
    return m.dense(x, out_dim, ActiMode(acti), bool(use_bias), DataType(dtype), shared_op=shared,
                   kernel_initializer=kinit, bias_initializer=binit, kernel_regularizer=reg, name=_name(name))


def add_embedding_init(m, x, num, dim, aggr, shared, kinit, name):
    return m.embedding(x, num, dim, AggrMode(aggr), shared_op=shared, kernel_initializer=kinit, name=_name(name))


def add_mha_init(m, q, k, v, embed, heads, kdim, vdim, dropout, bias, add_bias_kv, add_zero_attn, kinit, name):
    return m.multihead_attention(q, k, v, embed, heads, kdim, vdim, dropout, bool(bias), bool(add_bias_kv),
                                 bool(add_zero_attn), kernel_initializer=kinit, name=_name(name))


def add_batch_matmul(m, a, b, a_seq, b_seq):
    return m.batch_matmul(a, b, None if a_seq < 0 else a_seq, None if b_seq < 0 else b_seq)


def add_pool2d_ref(m, x, kh, kw, sh, sw, ph, pw, pool_type, acti, name):
    return m.pool2d(x, kh, kw, sh, sw, ph, pw, PoolType(pool_type), ActiMode(acti), name=_name(name))


def model_layer(m, i):
    return m.get_layer_by_id(int(i))


def model_last_layer(m):
    return m.get_last_layer()


def model_parameter(m, layer_id):
    """reference FFModel::get_parameter_by_id: the layer_id-th trainable parameter of the model."""
    ps = [w for L in m.layers for w in L.weights]
    return ps[int(layer_id)]


def model_perf_metrics(m):
    return m.get_perf_metrics()


def perf_get(pm, what):
    return float(pm.get_accuracy() if what == 0 else pm.get_loss())


def constant_create(m, dims, value, dtype):
    return m.create_constant(list(dims), float(value), DataType(dtype))


def tensor_map(m, t, op):
    m.map_tensor(t, op) if hasattr(m, "map_tensor") else None


_MAPPED = {}  # id(tensor) -> host numpy buffer of an inline-mapped tensor (raw pointers point into it)


def tensor_inline_map(t, m):
    dt = {DataType.DT_INT32: np.int32, DataType.DT_INT64: np.int64}.get(t.data_type, np.float32)
    if getattr(m, "_compiled", False):
        buf = np.ascontiguousarray(np.asarray(t.get_tensor(m)), dtype=dt).copy()
    else:
        buf = np.ascontiguousarray(t.get_array(m), dtype=dt)
        t._attached = buf  # writes before compile land in the value fed at compile
    _MAPPED[id(t)] = (t, buf)
    t.inline_map(m)


def tensor_inline_unmap(t, m):
    ent = _MAPPED.pop(id(t), None)
    if ent is not None and getattr(m, "_compiled", False) and t.owner_layer is None:
        t.set_tensor(m, ent[1])  # inputs / labels: the host writes become the tensor's value
    t.inline_unmap(m)


def tensor_raw_ptr(t, m, want):
    ent = _MAPPED.get(id(t))
    if ent is None:
        raise RuntimeError("flexflow_tensor_get_raw_ptr_*: call flexflow_tensor_inline_map first")
    buf = ent[1]
    need = np.float32 if want == 0 else np.int32
    if buf.dtype != need:
        raise TypeError(f"tensor is mapped as {buf.dtype}, not {np.dtype(need)}")
    return int(buf.ctypes.data)


def tensor_dims_legion(t):
    return [int(d) for d in reversed(t.dims)]


def tensor_dtype(t):
    return int(t.data_type.value)


def tensor_owner(t):
    if t.owner_layer is None:
        raise ValueError("tensor has no owner op (a model input)")
    return t.owner_layer


def tensor_is_mapped(t):
    return bool(t.is_mapped())


_CT = {DataType.DT_FLOAT: ctypes.c_float, DataType.DT_INT32: ctypes.c_int32, DataType.DT_INT64: ctypes.c_int64,
       DataType.DT_DOUBLE: ctypes.c_double}
_NPT = {DataType.DT_FLOAT: np.float32, DataType.DT_INT32: np.int32, DataType.DT_INT64: np.int64,
        DataType.DT_DOUBLE: np.float64}


def _host_view(addr, n, dtype):
    cdt = _CT[DataType(dtype)]
    return np.ctypeslib.as_array(ctypes.cast(addr, ctypes.POINTER(cdt)), shape=(int(n),))


def tensor_attach(t, m, addr, column_major):
    if column_major:
        raise ValueError("column-major attachment is not supported; pass row-major (C order) data")
    n = int(np.prod(t.dims))
    t.attach_numpy_array(m, None, _host_view(addr, n, t.data_type.value).reshape(t.dims))


def tensor_detach(t, m):
    t.detach_numpy_array()


def tensor_set_dims(t, m, dims, addr, dtype):
    if list(dims) and tuple(int(d) for d in dims) != tuple(t.dims):
        raise ValueError(f"dims {list(dims)} do not match the tensor's {list(t.dims)}")
    n = int(np.prod(t.dims))
    t.set_tensor(m, _host_view(addr, n, dtype).copy().reshape(t.dims).astype(_NPT[DataType(dtype)]))


def tensor_get_into(t, m, addr, dtype, grads):
    v = np.asarray(t.get_gradients(m) if grads else t.get_tensor(m)).reshape(-1)
    out = _host_view(addr, v.size, dtype)
    out[:] = v.astype(_NPT[DataType(dtype)])


def param_set(p, m, dims, addr):
    if list(dims) and tuple(int(d) for d in dims) != tuple(p.dims):
        raise ValueError(f"dims {list(dims)} do not match the parameter's {list(p.dims)}")
    n = int(np.prod(p.dims))
    p.set_weights(m, _host_view(addr, n, DataType.DT_FLOAT.value).copy().reshape(p.dims))


def param_get(p, m, addr):
    v = np.asarray(p.get_weights(m), dtype=np.float32).reshape(-1)
    _host_view(addr, v.size, DataType.DT_FLOAT.value)[:] = v


def model_set_opt(m, opt):
    m.optimizer = opt
    if getattr(m, "_compiled", False) and m.executor is not None:
        m.executor.init_optimizer(opt)


# ---------------------------------------------------------------- initializers
def init_create(kind, seed, a, b):
    from .core import initializers as I
    if kind == "null":
        return None
    if kind == "glorot":
        return I.GlorotUniformInitializer(seed)
    if kind == "zero":
        return I.ZeroInitializer()
    if kind == "uniform":
        return I.UniformInitializer(seed, a, b)
    return I.NormInitializer(seed, a, b)


# ---------------------------------------------------------------- example configs
def net_config_create():
    from .core.netconfig import NetConfig
    return NetConfig()


def dlrm_config_create():
    from .core.netconfig import DLRMConfig
    return DLRMConfig()


def obj_attr(o, key):
    return getattr(o, key)


# ---------------------------------------------------------------- data loader
def dataloader_create(m, t, full, num, dtype):
    from .core.dataloader import SingleDataLoader
    dl = SingleDataLoader.__new__(SingleDataLoader)
    dl.init_from_tensor(m, t, full, num, DataType(dtype))
    return dl


def dataloader_create_ptr(m, t, addr, num, dtype):
    from .core.dataloader import SingleDataLoader
    per = int(np.prod(t.dims[1:])) if len(t.dims) > 1 else 1
    arr = _host_view(addr, int(num) * per, dtype).reshape((int(num),) + tuple(t.dims[1:]))
    dl = SingleDataLoader.__new__(SingleDataLoader)
    dl.init_from_ptr(m, t, arr, num, DataType(dtype))
    return dl


def dataloader_set_num(dl, n):
    dl.num_samples = int(n)


def dataloader_get_num(dl):
    return int(dl.num_samples)


def dataloader_reset(dl):
    dl.reset()


def dataloader_next(dl, m):
    dl.next_batch(m)


# ---------------------------------------------------------------- timing / tracing / ops
def current_time_us(cfg):
    import time
    return time.perf_counter() * 1e6


def trace(cfg, tid, begin):
    (cfg.begin_trace if begin else cfg.end_trace)(int(tid))


def op_count(op, what):
    return len(op.weights if what == 0 else op.inputs if what == 1 else op.outputs)


def op_item(op, what, i):
    return (op.weights if what == 0 else op.inputs if what == 1 else op.outputs)[int(i)]


def op_run(op, m, what):
    (op.init if what == 0 else op.forward)(m)


def model_output_get(m, t, addr, grads):
    tensor_get_into(t, m, addr, DataType.DT_FLOAT.value, grads)
