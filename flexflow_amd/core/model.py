"""FFModel: the layer-graph builder and training API (reference include/flexflow/model.h:326-958,
python flexflow_cffi.py FFModel:887-2305).

`compile()` picks a parallelization strategy — imported from a file, data-parallel
(--only-data-parallel), or searched by the native Unity / MCMC search (flexflow_amd._core) against
the MI355X cost model — then lowers it to a per-rank Executor. The training loop API
(forward / zero_gradients / backward / update / compute_metrics, fit / eval) matches the
reference.
"""
from __future__ import annotations

import math
import os
import sys
import time
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..config import FFConfig
from ..type import (ActiMode, AggrMode, CompMode, DataType, LossType, MetricsType, OperatorType, PoolType,
                    RegularizerMode)
from .layer import Layer, op_class
from .tensor import Parameter, Tensor


class PerfMetrics:
    """reference include/flexflow/metrics_functions.h PerfMetrics."""

    def __init__(self, acc: Optional[np.ndarray] = None, metrics=()):
        a = acc if acc is not None else np.zeros(8)
        self.train_all = int(a[3]) if a[3] > 0 else int(a[7])
        self.train_correct = int(a[1])
        self.loss = float(a[0])
        self.cce_loss = float(a[2])
        self.sparse_cce_loss = float(a[2])
        self.mse_loss = float(a[4])
        self.rmse_loss = float(math.sqrt(a[4] / a[6])) if a[6] > 0 else 0.0
        self.mae_loss = float(a[5])
        self._n_el = float(a[6])
        self._n_rows = float(a[7])
        self.metrics = metrics

    def get_accuracy(self):
        return 100.0 * self.train_correct / self.train_all if self.train_all else 0.0

    def get_loss(self):
        return self.loss / self._n_rows if self._n_rows else 0.0

    def __repr__(self):
        s = [f"loss={self.get_loss():.4f}"]
        if MetricsType.METRICS_ACCURACY in self.metrics:
            s.append(f"accuracy: {self.get_accuracy():.2f}% ({self.train_correct} / {self.train_all})")
        if MetricsType.METRICS_MEAN_SQUARED_ERROR in self.metrics and self._n_el:
            s.append(f"mse: {self.mse_loss / self._n_el:.4f}")
        return "[Metrics] " + " ".join(s)


def _ensure_dist(config: FFConfig):
    if config.world_size > 1 and not dist.is_initialized():
        # FF_DIST_BACKEND=gloo lets several ranks share one GPU (multi-rank rehearsal on a 1-GPU box;
        # RCCL refuses two ranks on one device)
        backend = os.environ.get("FF_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if torch.cuda.is_available():
            torch.cuda.set_device(config.local_rank % torch.cuda.device_count())
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", config.local_rank % torch.cuda.device_count())
        import datetime
        kw["timeout"] = datetime.timedelta(seconds=float(getattr(config, "dist_timeout_s", 1800.0)))
        dist.init_process_group(backend=backend, **kw)
    elif torch.cuda.is_available():
        torch.cuda.set_device(config.local_rank % torch.cuda.device_count())


class FFModel:
    def __init__(self, ffconfig: Optional[FFConfig] = None):
        self.config = ffconfig or FFConfig()
        self.layers: List[Layer] = []
        self.optimizer = None
        self.loss_type = None
        self.metrics = []
        self.comp_mode = CompMode.TRAINING
        self.label_tensor: Optional[Tensor] = None
        self.executor = None
        self.strategy = None
        self.search_report = None
        self._compiled = False
        self._output = None
        self._pending_values = {}
        self._pending_weights = {}  # weight guid -> array set before compile (applied after init)
        self._tensor_remap = {}  # guid -> replacement tensor (graph substitutions at compile)
        self._names = set()
        self.iter_config_seq_length = None
        self._recompile = None
        self._step_graph = None

    # ================================================================== graph building
    def _add(self, op_type, inputs, name=None, **attrs):
        if name is not None:  # layer names key the strategy and executor state: keep them unique
            taken = self._names
            if name in taken:
                k = 1
                while f"{name}_{k}" in taken:
                    k += 1
                name = f"{name}_{k}"
        L = Layer(self, op_type, name, inputs, attrs)
        self._names.add(L.name)
        L.__class__ = op_class(op_type)  # reference per-op layer class (Linear, Conv2D, ...)
        self.layers.append(L)
        return L

    def add_layer(self, op_type, name):
        """reference FFModel.add_layer (flexflow_cffi.py:913): registers the last created op with the
        Python layer list. Layers are registered as they are built here, so this only renames the
        last layer when a name is given."""
        if name and self.layers:
            self.layers[-1].name = name

    def create_tensor(self, dims, data_type=DataType.DT_FLOAT, create_grad=True, name=None):
        L = self._add(OperatorType.OP_INPUT, [], name, dims=tuple(dims), data_type=data_type)
        t = L.outputs[0]
        t.create_grad = create_grad
        return t

    def lstm(self, input, hidden_size, hx=None, cx=None, kernel_initializer=None, name=None):
        """LSTM over input [B, L, E] -> (y [B, L, H], hy [B, H], cy [B, H]); hx / cx default to
        zeros (ops/rnn.py; the reference's LSTM lives in its separate nmt/ application)."""
        B = input.dims[0]
        if hx is None:
            hx = self.create_constant([B, hidden_size], 0.0)
        if cx is None:
            cx = self.create_constant([B, hidden_size], 0.0)
        L = self._add(OperatorType.OP_LSTM, [input, hx, cx], name, hidden_size=int(hidden_size),
                      kernel_init=kernel_initializer)
        return tuple(L.outputs)

    def create_constant(self, dims, value, data_type=DataType.DT_FLOAT):
        t = self.create_tensor(dims, data_type, False)
        self._pending_values[t.guid] = np.full(dims, value, dtype=np.float32 if data_type == DataType.DT_FLOAT else np.int32)
        return t

    def map_tensor(self, tensor, parallel_op=None):
        return tensor

    # ---- element-wise
    def _unary(self, op, x, name=None, **kw):
        return self._add(op, [x], name, **kw).outputs[0]

    def exp(self, x, name=None):
        return self._unary(OperatorType.OP_EXP, x, name)

    def sin(self, x, name=None):
        return self._unary(OperatorType.OP_SIN, x, name)

    def cos(self, x, name=None):
        return self._unary(OperatorType.OP_COS, x, name)

    def rsqrt(self, input, name=None):
        return self._unary(OperatorType.OP_RSQRT, input, name)

    def pow(self, input, exponent, name=None):
        return self._unary(OperatorType.OP_POW, input, name, scalar=float(exponent))

    def relu(self, input, inplace=True, name=None):
        return self._unary(OperatorType.OP_RELU, input, name)

    def gelu(self, input, inplace=True, name=None):
        return self._unary(OperatorType.OP_GELU, input, name)

    def elu(self, input, inplace=True, name=None):
        return self._unary(OperatorType.OP_ELU, input, name)

    def identity(self, input, name=None):
        return self._unary(OperatorType.OP_IDENTITY, input, name)

    def sigmoid(self, input, name=None):
        return self._unary(OperatorType.OP_SIGMOID, input, name)

    def tanh(self, input, name=None):
        return self._unary(OperatorType.OP_TANH, input, name)

    def scalar_multiply(self, input, scalar, inplace=True, name=None):
        return self._unary(OperatorType.OP_SCALAR_MULTIPLY, input, name, scalar=float(scalar))

    def scalar_add(self, input, scalar, inplace=True, name=None):
        return self._unary(OperatorType.OP_SCALAR_ADD, input, name, scalar=float(scalar))

    def scalar_sub(self, input, scalar, inplace=True, name=None):
        return self._unary(OperatorType.OP_SCALAR_SUB, input, name, scalar=float(scalar))

    def scalar_true_divide(self, input, scalar, inplace=True, name=None):
        return self._unary(OperatorType.OP_SCALAR_TRUE_DIV, input, name, scalar=float(scalar))

    scalar_truediv = scalar_true_divide

    def scalar_floor_divide(self, input, scalar, name=None):
        return self._unary(OperatorType.OP_SCALAR_FLOOR_DIV, input, name, scalar=float(scalar))

    def _binary(self, op, x, y, name=None):
        return self._add(op, [x, y], name).outputs[0]

    def add(self, x, y, inplace_a=False, name=None):
        return self._binary(OperatorType.OP_EW_ADD, x, y, name)

    def subtract(self, x, y, inplace_a=False, name=None):
        return self._binary(OperatorType.OP_EW_SUB, x, y, name)

    def multiply(self, x, y, inplace_a=False, name=None):
        return self._binary(OperatorType.OP_EW_MUL, x, y, name)

    def divide(self, x, y, inplace_a=False, name=None):
        return self._binary(OperatorType.OP_EW_DIV, x, y, name)

    def max(self, x, y, inplace_a=False, name=None):
        return self._binary(OperatorType.OP_EW_MAX, x, y, name)

    def min(self, x, y, inplace_a=False, name=None):
        return self._binary(OperatorType.OP_EW_MIN, x, y, name)

    def dropout(self, input, rate, seed=0, name=None):
        return self._unary(OperatorType.OP_DROPOUT, input, name, rate=float(rate), seed=int(seed))

    def cast(self, input, dtype, name=None):
        return self._add(OperatorType.OP_CAST, [input], name, dtype=dtype).outputs[0]

    # ---- reductions
    def reduce_sum(self, input, axes, keepdims=False, name=None):
        return self._add(OperatorType.OP_REDUCE_SUM, [input], name, axes=list(axes), keepdims=keepdims).outputs[0]

    def mean(self, input, dims, keepdims=False, name=None):
        return self._add(OperatorType.OP_MEAN, [input], name, axes=list(dims), keepdims=keepdims).outputs[0]

    # ---- dense / conv / pool / norm
    def dense(self, input, out_dim, activation=ActiMode.AC_MODE_NONE, use_bias=True, datatype=DataType.DT_FLOAT,
              shared_op=None, kernel_initializer=None, bias_initializer=None,
              kernel_regularizer=None, name=None):
        L = self._add(OperatorType.OP_LINEAR, [input], name, out_dim=int(out_dim), activation=activation,
                      use_bias=use_bias, kernel_init=kernel_initializer, bias_init=bias_initializer,
                      regularizer=kernel_regularizer)
        self._share(L, shared_op)
        return L.outputs[0]

    def conv2d(self, input, out_channels, kernel_h, kernel_w, stride_h, stride_w, padding_h, padding_w,
               activation=ActiMode.AC_MODE_NONE, groups=1, use_bias=True, shared_op=None, kernel_initializer=None,
               bias_initializer=None, name=None):
        L = self._add(OperatorType.OP_CONV2D, [input], name, out_channels=int(out_channels), kernel_h=kernel_h,
                      kernel_w=kernel_w, stride_h=stride_h, stride_w=stride_w, padding_h=padding_h,
                      padding_w=padding_w, activation=activation, groups=groups, use_bias=use_bias,
                      kernel_init=kernel_initializer, bias_init=bias_initializer)
        self._share(L, shared_op)
        return L.outputs[0]

    def pool2d(self, input, kernel_h, kernel_w, stride_h, stride_w, padding_h, padding_w,
               pool_type=PoolType.POOL_MAX, activation=ActiMode.AC_MODE_NONE, name=None, count_include_pad=True):
        """count_include_pad (average pooling only): divide by the full window including padding
        (the reference's cuDNN mode, default) or by the valid elements (ONNX's default)."""
        kw = {} if count_include_pad else {"count_include_pad": False}
        return self._add(OperatorType.OP_POOL2D, [input], name, kernel_h=kernel_h, kernel_w=kernel_w,
                         stride_h=stride_h, stride_w=stride_w, padding_h=padding_h, padding_w=padding_w,
                         pool_type=pool_type, activation=activation, **kw).outputs[0]

    def batch_norm(self, input, relu=True, name=None):
        return self._add(OperatorType.OP_BATCHNORM, [input], name, relu=relu).outputs[0]

    def layer_norm(self, input, axes, elementwise_affine=True, eps=1e-5, name=None):
        return self._add(OperatorType.OP_LAYERNORM, [input], name, axes=list(axes),
                         elementwise_affine=elementwise_affine, eps=eps).outputs[0]

    def rms_norm(self, input, eps=1e-6, name=None):
        """y = x * rsqrt(mean(x^2, -1) + eps) * weight (extension; ops/norm.py RMSNorm)."""
        return self._add(OperatorType.OP_RMS_NORM, [input], name, eps=float(eps)).outputs[0]

    def batch_matmul(self, A, B, a_seq_length_dim=None, b_seq_length_dim=None, name=None):
        return self._add(OperatorType.OP_BATCHMATMUL, [A, B], name, a_seq_length_dim=a_seq_length_dim,
                         b_seq_length_dim=b_seq_length_dim).outputs[0]

    def embedding(self, input, num_embeddings, embedding_dim, aggr=AggrMode.AGGR_MODE_NONE, dtype=DataType.DT_FLOAT,
                  shared_op=None, kernel_initializer=None, name=None):
        L = self._add(OperatorType.OP_EMBEDDING, [input], name, num_entries=int(num_embeddings),
                      out_dim=int(embedding_dim), aggr=aggr, data_type=dtype, kernel_init=kernel_initializer)
        self._share(L, shared_op)
        return L.outputs[0]

    def multihead_attention(self, query, key, value, embed_dim, num_heads, kdim=0, vdim=0, dropout=0.0, bias=True,
                            add_bias_kv=False, add_zero_attn=False, kernel_initializer=None, causal=False, name=None):
        return self._add(OperatorType.OP_MULTIHEAD_ATTENTION, [query, key, value], name, embed_dim=int(embed_dim),
                         num_heads=int(num_heads), kdim=int(kdim), vdim=int(vdim), dropout=float(dropout), bias=bias,
                         add_bias_kv=add_bias_kv, add_zero_attn=add_zero_attn, kernel_init=kernel_initializer,
                         causal=causal, self_attn=(query is key and key is value)).outputs[0]

    # ---- shape ops
    def concat(self, tensors, axis, name=None):
        return self._add(OperatorType.OP_CONCAT, list(tensors), name, axis=int(axis)).outputs[0]

    def split(self, input, sizes, axis, name=None):
        return list(self._add(OperatorType.OP_SPLIT, [input], name, sizes=sizes, axis=int(axis)).outputs)

    def flat(self, input, name=None):
        return self._add(OperatorType.OP_FLAT, [input], name).outputs[0]

    def softmax(self, input, axis=-1, name=None):
        return self._add(OperatorType.OP_SOFTMAX, [input], name, dim=int(axis)).outputs[0]

    def reshape(self, input, shape, name=None):
        return self._add(OperatorType.OP_RESHAPE, [input], name, shape=tuple(shape)).outputs[0]

    def gather(self, input, index, dim, name=None):
        return self._add(OperatorType.OP_GATHER, [input, index], name, dim=int(dim)).outputs[0]

    def transpose(self, input, perm, name=None):
        return self._add(OperatorType.OP_TRANSPOSE, [input], name, perm=tuple(perm)).outputs[0]

    def reverse(self, input, axis, name=None):
        return self._add(OperatorType.OP_REVERSE, [input], name, axis=int(axis)).outputs[0]

    # ---- mixture of experts
    def top_k(self, input, k, sorted=False, name=None):
        return list(self._add(OperatorType.OP_TOPK, [input], name, k=int(k), sorted=sorted).outputs)

    def group_by(self, data, assign, n, alpha, name=None):
        return list(self._add(OperatorType.OP_GROUP_BY, [data, assign], name, n=int(n), alpha=float(alpha)).outputs)

    def aggregate(self, inputs, n, lambda_bal, name=None):
        return self._add(OperatorType.OP_AGGREGATE, list(inputs), name, n=int(n),
                         lambda_bal=float(lambda_bal)).outputs[0]

    def aggregate_spec(self, inputs, n, lambda_bal, name=None):
        return self._add(OperatorType.OP_AGG_SPEC, list(inputs), name, n=int(n),
                         lambda_bal=float(lambda_bal)).outputs[0]

    def cache(self, input, num_batches, score_f=None, name=None):
        L = self._add(OperatorType.OP_CACHE, [input], name, num_batches=int(num_batches))
        L.attrs["score_f"] = score_f
        return L.outputs[0]

    def moe(self, input, num_exp, num_select, expert_hidden_size, alpha, lambda_bal):
        """reference FFModel::moe (src/ops/moe.cc): gate -> top_k -> group_by -> experts -> aggregate."""
        gate = self.dense(input, num_exp, ActiMode.AC_MODE_RELU)
        topk_v, topk_i = self.top_k(gate, num_select, False)
        exp_t = self.group_by(input, topk_i, num_exp, alpha)
        agg = [self.softmax(topk_v), topk_i, topk_i, gate]
        for e in exp_t:
            agg.append(self.softmax(self.dense(e, expert_hidden_size, ActiMode.AC_MODE_RELU)))
        return self.aggregate(agg, num_exp, lambda_bal)

    # ---- explicit parallel ops (ops/parallel_ops.py): identity compute, pinned output layout
    def repartition(self, input, dim, degree, name=None):
        return self._add(OperatorType.OP_REPARTITION, [input], name, dim=int(dim), degree=int(degree)).outputs[0]

    def combine(self, input, dim=0, degree=None, name=None):
        return self._add(OperatorType.OP_COMBINE, [input], name, dim=int(dim), degree=degree).outputs[0]

    def replicate(self, input, degree, name=None):
        return self._add(OperatorType.OP_REPLICATE, [input], name, degree=int(degree)).outputs[0]

    def reduction(self, input, dim=0, degree=1, name=None):
        return self._add(OperatorType.OP_REDUCTION, [input], name, dim=int(dim), degree=int(degree)).outputs[0]

    def allreduce(self, input, name=None):
        return self._add(OperatorType.OP_ALLREDUCE, [input], name).outputs[0]

    def fused_parallel(self, input, ops, name=None):
        """ops: [(kind, dim, degree)] with kind in repartition/combine/replicate/allreduce."""
        return self._add(OperatorType.OP_FUSED_PARALLEL, [input], name, ops=[tuple(o) for o in ops]).outputs[0]

    def _share(self, L, shared_op):
        if shared_op is None:
            return
        src = shared_op if isinstance(shared_op, Layer) else getattr(shared_op, "owner_layer", None)
        assert src is not None and len(src.weights) == len(L.weights), "shared_op must have matching weights"
        for i, w in enumerate(src.weights):
            assert w.dims == L.weights[i].dims
        L.weights = list(src.weights)
        L.attrs["shared_with"] = src.name

    # ================================================================== introspection
    def get_layers(self):
        return {i: L for i, L in enumerate(self.layers) if L.op_type != OperatorType.OP_INPUT}

    def _non_input_layers(self):
        return [L for L in self.layers if L.op_type != OperatorType.OP_INPUT]

    def get_layer_by_id(self, layer_id):
        return self._non_input_layers()[layer_id]

    def get_last_layer(self):
        return self._non_input_layers()[-1]

    def get_layer_by_name(self, layer_name):
        for L in self.layers:
            if L.name == layer_name:
                return L
        return None

    def get_tensor_by_id(self, id):
        for L in self.layers:
            for t in L.outputs:
                if t.guid == id:
                    return t
        return None

    def print_layers(self, id=-1):
        for i, L in enumerate(self._non_input_layers()):
            if id in (-1, i):
                cfg = self.strategy.get(L.name) if self.strategy else None
                print(f"layer[{i}] {L} cfg={cfg}")

    def output_tensor(self):
        if self._output is not None:
            return self._output
        for L in reversed(self.layers):
            if L.op_type != OperatorType.OP_INPUT:
                return L.outputs[0]
        return None

    def set_output(self, t):
        self._output = t

    # ================================================================== compile
    def compile(self, optimizer=None, loss_type=None, metrics=None, comp_mode=None):
        cfg = self.config
        if optimizer is not None:
            self.optimizer = optimizer
        if comp_mode is not None:
            self.comp_mode = comp_mode
        self.loss_type = loss_type
        self.metrics = list(metrics or [])
        _ensure_dist(cfg)
        self.subst_report = None
        if os.environ.get("FF_NO_SUBST", "0") != "1":
            try:
                from ..pcg.substitutions import optimize_graph
                self.subst_report = optimize_graph(self)
            except ImportError:  # native core not built: run the graph as written
                self.subst_report = {"skipped": "native core unavailable"}
        out = self.output_tensor()
        if loss_type is not None and out is not None:
            if loss_type == LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY:
                lab_dims = tuple(out.dims[:-1]) + (1,)
                self.label_tensor = Tensor(lab_dims, DataType.DT_INT32, name="label")
            else:
                self.label_tensor = Tensor(out.dims, out.data_type, name="label")
        from ..pcg.search import choose_strategy
        self.strategy, self.search_report = choose_strategy(self)
        from ..runtime.executor import Executor
        training = self.comp_mode == CompMode.TRAINING
        self.executor = Executor(self, self.strategy, loss_type, self.metrics, training=training)
        self.executor.init_weights(cfg.seed)
        if os.environ.get("FF_NO_INPLACE") != "1":
            self.executor._plan_inplace()
            self.executor._plan_binary_relu()
        self.executor._plan_bias_grad_fusion()
        self.executor._plan_dact_fusion()
        if self.optimizer is not None and training:
            self.executor.init_optimizer(self.optimizer)
        for guid, v in self._pending_values.items():
            t = self._find_tensor(guid)
            if t is not None:
                self.executor.feed(t, v)
        if self._pending_weights:
            by_guid = {w.guid: w for L in self.layers for w in L.weights}
            for guid, v in self._pending_weights.items():
                if guid in by_guid:
                    self.executor.set_weight(by_guid[guid], v)
                else:  # a weight a graph rewrite stacked into a larger one
                    tgt = self._resolve_weight_alias(guid)
                    if tgt is not None:
                        self._set_weight_block(tgt, v)
        for L in self.layers:
            for t in L.outputs:
                if t._attached is not None:
                    self.executor.feed(t, t._attached)
        self._compiled = True
        if cfg.export_strategy_file and cfg.rank == 0:
            from ..pcg.strategy import save_strategy
            save_strategy(cfg.export_strategy_file, self.strategy, cfg.num_devices,
                          extra={"search": self.search_report})
        # aux subsystems: per-op profiling / traces, non-finite detection, hang watchdog, dot export
        self.profiler = None
        self.guard = None
        self.watchdog = None
        if cfg.profiling or cfg.trace_dir:
            from ..runtime.profiler import OpProfiler
            self.profiler = OpProfiler(self.executor, cfg.rank)
            self.executor.hooks.append(self.profiler)
        if cfg.check_nan_every or os.environ.get("FF_DEBUG_NAN") == "1":
            from ..runtime.health import NonFiniteGuard
            self.guard = NonFiniteGuard(self.executor, cfg.check_nan_every or 1,
                                        per_op=os.environ.get("FF_DEBUG_NAN") == "1")
            if self.guard.per_op:
                self.executor.hooks.append(self.guard)
        if cfg.watchdog_s > 0:
            from ..runtime.health import Watchdog
            self.watchdog = Watchdog(cfg.watchdog_s)
        if cfg.rank == 0 and (cfg.export_strategy_computation_graph_file or cfg.export_strategy_task_graph_file):
            from ..utils.dot import export_computation_graph, export_task_graph
            if cfg.export_strategy_computation_graph_file:
                export_computation_graph(self, cfg.export_strategy_computation_graph_file,
                                         include_costs=cfg.include_costs_dot_graph)
            if cfg.export_strategy_task_graph_file:
                export_task_graph(self, cfg.export_strategy_task_graph_file)

    def _find_tensor(self, guid):
        for L in self.layers:
            for t in L.outputs:
                if t.guid == guid:
                    return t
        if self.label_tensor is not None and self.label_tensor.guid == guid:
            return self.label_tensor
        return None

    def init_layers(self):
        """Weights are initialised at compile (reference init_operators)."""
        return None

    init_operators = init_layers

    def prefetch(self):
        return None

    # ================================================================== training loop
    def forward(self, seq_length=None):
        if seq_length is not None:
            self.iter_config_seq_length = seq_length
        from ..runtime.trace import traced_call
        traced_call(self, "forward", self._eager_forward)
        self._metrics_pending = True

    def zero_gradients(self):
        from ..runtime.trace import traced_call
        traced_call(self, "zero_gradients", self._eager_zero_gradients)

    def backward(self, seq_length=None):
        from ..runtime.trace import traced_call
        traced_call(self, "backward", self._eager_backward)  # loss gradient + metrics of the last forward
        self._metrics_pending = False

    def _eager_forward(self):
        self.executor.forward()

    def _eager_zero_gradients(self):
        self.executor.zero_gradients()

    def _eager_backward(self):
        self.executor.backward()

    def update(self):
        from ..runtime.trace import note_update
        note_update(self)
        self.executor.update(self.optimizer)

    def compute_metrics(self):
        """Metrics of the last forward (reference FFModel::compute_metrics). During training they
        are produced by backward's fused loss kernel; after a forward-only pass (evaluation) the
        loss/metric kernels run here."""
        if getattr(self, "_metrics_pending", False):
            self.executor.compute_loss_grad()
            self._metrics_pending = False

    def reset_metrics(self):
        self.executor.reset_metrics()

    def get_perf_metrics(self):
        return PerfMetrics(self.executor.metrics_snapshot(), self.metrics)

    def set_optimizer(self, optimizer):
        self.optimizer = optimizer
        if self.executor is not None:
            self.executor.init_optimizer(optimizer)

    def train_step(self):
        """One full iteration (forward, zero_gradients, backward, update) — the unit captured by
        hipGraphs in runtime/graph.py."""
        from ..runtime.graph import run_train_step
        if self.watchdog is not None:
            self.watchdog.arm()
        hi = self._compute_stream()
        if hi is None:
            run_train_step(self)
        else:  # the step's kernels on a high-priority stream, joined both ways with the caller's
            cur = torch.cuda.current_stream()
            hi.wait_stream(cur)
            with torch.cuda.stream(hi):
                run_train_step(self)
            cur.wait_stream(hi)
        if self.watchdog is not None:
            self.watchdog.disarm()
        if self.profiler is not None:
            self.profiler.next_step()
        if self.guard is not None:
            self.guard.after_step(self.executor._metric_acc[0])

    def _compute_stream(self):
        """FF_COMPUTE_PRIO=high: train steps run on a stream of the device's highest priority, so
        that the overlapped optimizer update (a default-priority side stream) yields freed CU slots
        to the backward's kernels. None (the caller's stream) otherwise, or without a GPU."""
        if os.environ.get("FF_COMPUTE_PRIO", "default") != "high" or not torch.cuda.is_available():
            return None
        st = getattr(self, "_hi_stream", None)
        if st is None:
            _, greatest = torch.cuda.Stream.priority_range()
            st = self._hi_stream = torch.cuda.Stream(priority=greatest)
        return st

    # ---- checkpoint / profiling
    def save_checkpoint(self, path):
        from ..runtime.checkpoint import save_checkpoint
        return save_checkpoint(self, path)

    def load_checkpoint(self, path, strict=True):
        from ..runtime.checkpoint import load_checkpoint
        return load_checkpoint(self, path, strict)

    def profile_report(self, top=40):
        """Per-op device time table (--profiling); also writes the Chrome trace to --trace-dir."""
        if self.profiler is None:
            return ""
        if self.config.trace_dir:
            self.profiler.chrome_trace(os.path.join(self.config.trace_dir, f"trace_rank{self.config.rank}.json"))
        return self.profiler.report(top)

    def export_dot(self, path, include_costs=False):
        from ..utils.dot import export_computation_graph
        return export_computation_graph(self, path, include_costs=include_costs)

    def recompile_on_condition(self, r):
        """reference FFModel::recompile_on_condition (model.cc:2422-2426)."""
        self._recompile = r
        if r.trigger():
            r.alter()

    def fit(self, x=None, y=None, batch_size=None, epochs=1):
        """x, y: SingleDataLoader (or lists of them) as in the reference; numpy arrays are wrapped."""
        from .dataloader import SingleDataLoader
        xs = x if isinstance(x, (list, tuple)) else [x]
        if not isinstance(xs[0], SingleDataLoader):
            inputs = [L.outputs[0] for L in self.layers if L.op_type == OperatorType.OP_INPUT]
            xs = [SingleDataLoader(self, t, a) for t, a in zip(inputs, xs)]
        if y is not None and not isinstance(y, SingleDataLoader):
            y = SingleDataLoader(self, self.label_tensor, y)
        bs = batch_size or self.config.batch_size
        num_samples = xs[0].num_samples
        iters = num_samples // bs
        ts = time.perf_counter()
        for ep in range(epochs):
            for d in xs:
                d.reset()
            if y is not None:
                y.reset()
            self.reset_metrics()
            for it in range(iters):
                for d in xs:
                    d.next_batch(self)
                if y is not None:
                    y.next_batch(self)
                self.train_step()
            if self.config.rank == 0 and self.metrics:
                pm = self.get_perf_metrics()
                print(f"epoch {ep}: {pm}", flush=True)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        el = time.perf_counter() - ts
        if self.config.rank == 0:
            print(f"ELAPSED TIME = {el:.4f}s, THROUGHPUT = {num_samples * epochs / max(el, 1e-9):.2f} samples/s",
                  flush=True)

    def eval(self, x=None, y=None, batch_size=None):
        from .dataloader import SingleDataLoader
        xs = x if isinstance(x, (list, tuple)) else [x]
        if not isinstance(xs[0], SingleDataLoader):
            inputs = [L.outputs[0] for L in self.layers if L.op_type == OperatorType.OP_INPUT]
            xs = [SingleDataLoader(self, t, a) for t, a in zip(inputs, xs)]
        if y is not None and not isinstance(y, SingleDataLoader):
            y = SingleDataLoader(self, self.label_tensor, y)
        bs = batch_size or self.config.batch_size
        iters = xs[0].num_samples // bs
        for d in xs:
            d.reset()
        if y is not None:
            y.reset()
        self.reset_metrics()
        for it in range(iters):
            for d in xs:
                d.next_batch(self)
            if y is not None:
                y.next_batch(self)
            self.executor.forward(training=False)
            self.executor.compute_loss_grad()
        pm = self.get_perf_metrics()
        if self.config.rank == 0:
            print(f"eval: {pm}", flush=True)
        return pm

    # ================================================================== data access
    def create_data_loader(self, batch_tensor, full_array):
        from .dataloader import SingleDataLoader
        return SingleDataLoader(self, batch_tensor, full_array)

    def _set_tensor_value(self, t, arr):
        if isinstance(t, Parameter):
            return self._set_weight_value(t, arr)
        if not self._compiled:
            self._pending_values[t.guid] = np.asarray(arr)
            return
        self.executor.feed(t, np.asarray(arr))

    def resolve_tensor(self, t):
        """The live tensor playing `t`'s role after compile-time graph substitutions (a fused
        layer replaces the tensors of the layers it absorbed)."""
        while t.guid in self._tensor_remap:
            t = self._tensor_remap[t.guid]
        return t

    def _get_tensor_value(self, t):
        v = self.executor.get_value(self.resolve_tensor(t))
        return (v.float() if v.is_floating_point() else v).detach().cpu().numpy().copy()

    def _get_tensor_grad(self, t):
        if isinstance(t, Parameter):
            tgt = self._resolve_weight_alias(t.guid)
            if tgt is not None:
                lw, start, rows = tgt
                return self.executor.get_weight_grad(lw).detach().cpu().numpy()[start:start + rows].copy()
            return self.executor.get_weight_grad(t).detach().cpu().numpy().copy()
        raise NotImplementedError("activation gradients are not retained")

    def _resolve_weight_alias(self, guid):
        """(live weight, first row, rows) holding the original weight `guid` after graph rewrites
        that stacked it into a larger weight (pcg/joint.py MergeSiblings), or None."""
        alias = getattr(self, "_weight_alias", None) or {}
        if guid not in alias:
            return None
        w, start, rows = alias[guid]
        while w.guid in alias:  # merged again: offset into the outer stack
            w2, s2, _ = alias[w.guid]
            w, start = w2, s2 + start
        return w, start, rows

    def _set_weight_block(self, tgt, arr):
        w, start, rows = tgt
        full = self.executor.get_weight(w).float().detach().cpu().numpy().copy()
        full[start:start + rows] = np.asarray(arr, dtype=np.float32).reshape(full[start:start + rows].shape)
        self.executor.set_weight(w, full)

    def _set_weight_value(self, w, arr):
        if not self._compiled:
            self._pending_weights[w.guid] = np.asarray(arr)
            return
        tgt = self._resolve_weight_alias(w.guid)
        if tgt is not None:
            return self._set_weight_block(tgt, arr)
        self.executor.set_weight(w, np.asarray(arr))

    def _get_weight_value(self, w):
        tgt = self._resolve_weight_alias(w.guid)
        if tgt is not None:
            lw, start, rows = tgt
            return self.executor.get_weight(lw).float().detach().cpu().numpy()[start:start + rows].copy()
        return self.executor.get_weight(w).float().detach().cpu().numpy().copy()

    @property
    def ffconfig(self):
        return self.config

    def get_output_tensor(self, ffmodel=None, data_type=None):
        return self._get_tensor_value(self.output_tensor())
