"""flexflow_amd.keras.layers — symbolic Keras-style layers lowered onto FFModel at compile time.

Mirrors the reference's python/flexflow/keras/layers (core.py, convolutional.py, pool.py,
merge.py, normalization.py, input_layer.py): tensors are channels-first (NCHW) like every
FlexFlow CNN; Conv2D/Pooling2D take explicit (ph, pw) padding tuples or 'valid'/'same'.

A layer called on KTensors records the call and returns KTensors with inferred shapes; nothing is
built until Model.compile walks the recorded graph and calls `_lower(ff, inputs)` on each layer.
"""
from __future__ import annotations

import itertools
from typing import List, Optional, Sequence

from ...type import ActiMode, AggrMode, DataType, PoolType
from .. import initializers as kinit
from .. import regularizers as kreg

_uid = itertools.count()

_DT = {"float32": DataType.DT_FLOAT, "float": DataType.DT_FLOAT, "int32": DataType.DT_INT32,
       "int64": DataType.DT_INT64, "float16": DataType.DT_HALF, "bfloat16": DataType.DT_BF16}


def _dtype(d):
    if isinstance(d, DataType):
        return d
    return _DT[str(d)]


_ACT = {None: ActiMode.AC_MODE_NONE, "linear": ActiMode.AC_MODE_NONE, "relu": ActiMode.AC_MODE_RELU,
        "sigmoid": ActiMode.AC_MODE_SIGMOID, "tanh": ActiMode.AC_MODE_TANH, "gelu": ActiMode.AC_MODE_GELU}


class KTensor:
    """Symbolic tensor: shape excludes the batch dimension."""

    def __init__(self, shape, dtype=DataType.DT_FLOAT, layer=None, index=0, name=None):
        self.shape = tuple(int(s) for s in shape)
        self.dtype = _dtype(dtype)
        self.layer = layer
        self.index = index
        self.name = name or f"ktensor_{next(_uid)}"

    @property
    def batch_shape(self):
        return (None,) + self.shape

    @property
    def num_dims(self):
        return len(self.shape) + 1

    def __repr__(self):
        return f"KTensor({self.name}, shape={self.batch_shape}, dtype={self.dtype.name})"

    # elementwise arithmetic records merge layers (tf.keras-style `x + y`)
    def __add__(self, other):
        return Add()([self, other])

    def __sub__(self, other):
        return Subtract()([self, other])

    def __mul__(self, other):
        return Multiply()([self, other])

    def __truediv__(self, other):
        return Divide()([self, other])


class Layer:
    """Base layer: __call__ records (inputs -> outputs); _lower builds FFModel ops."""

    def __init__(self, name=None, input_shape=None, dtype=None, **kwargs):
        self.name = name or f"{type(self).__name__.lower()}_{next(_uid)}"
        self.input_shape = tuple(input_shape) if input_shape is not None else None
        self.dtype = _dtype(dtype) if dtype is not None else None
        self.inbound: List[List[KTensor]] = []   # one entry per call
        self.outbound: List[List[KTensor]] = []
        self.ff_layers = []                        # FFModel layers created when lowered
        self.trainable = kwargs.pop("trainable", True)

    # ---- graph recording
    def __call__(self, inputs):
        xs = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
        shapes = self.compute_output_shape([x.shape for x in xs])
        dts = self.output_dtypes([x.dtype for x in xs])
        outs = [KTensor(s, d, self, i, f"{self.name}:{len(self.inbound)}:{i}") for i, (s, d) in
                enumerate(zip(shapes, dts))]
        self.inbound.append(xs)
        self.outbound.append(outs)
        return outs[0] if len(outs) == 1 else outs

    def compute_output_shape(self, in_shapes):
        return [in_shapes[0]]

    def output_dtypes(self, in_dtypes):
        return [in_dtypes[0]]

    # ---- lowering
    def _lower(self, ff, xs):
        raise NotImplementedError

    def _track(self, ff, out):
        self.ff_layers.append(ff.get_last_layer())
        return out

    def _shared(self, ff):
        """The FFModel layer this layer already lowered to in `ff` (a layer called twice shares its
        weights, as in Keras); None on the first call."""
        for L in self.ff_layers:
            if L.model is ff:
                return L
        return None

    # ---- weights (after compile)
    def get_weights(self, ffmodel=None):
        import numpy as np
        if not self.ff_layers:
            return []
        m = ffmodel or self._model.ffmodel
        L = self._shared(m) or self.ff_layers[-1]
        return [np.asarray(w.get_weights(m)) for w in L.weights]

    def set_weights(self, *args, ffmodel=None):
        """set_weights([kernel, bias], ffmodel=None) (Keras) or set_weights(ffmodel, kernel, bias)
        (reference keras/layers/core.py:105)."""
        from ...core.model import FFModel
        if args and isinstance(args[0], FFModel):
            ffmodel, weights = args[0], list(args[1:])
        else:
            weights = list(args[0]) if args else []
            if len(args) > 1:
                ffmodel = args[1]
        m = ffmodel or self._model.ffmodel
        L = self._shared(m) or self.ff_layers[-1]
        for w, v in zip(L.weights, weights):
            w.set_weights(m, v)

    def get_summary(self):
        outs = self.outbound[0] if self.outbound else []
        ins = self.inbound[0] if self.inbound else []
        return (f"{self.name} ({type(self).__name__})\t\t{[o.batch_shape for o in outs]}\t\t"
                f"{[i.batch_shape for i in ins]}\t{[i.layer.name if i.layer else 'input' for i in ins]}\n")

    def __repr__(self):
        return f"<{type(self).__name__} {self.name}>"


class InputLayer(Layer):
    def __init__(self, shape, dtype="float32", name=None):
        super().__init__(name=name, dtype=dtype)
        self.output_tensor = KTensor(shape, self.dtype, self, 0, self.name)
        self.outbound.append([self.output_tensor])

    def _lower(self, ff, xs):
        raise RuntimeError("input layers are created by the model")


def Input(shape=None, batch_size=None, name=None, dtype="float32", **kwargs):
    """reference keras/layers/input_layer.py: returns the symbolic input tensor."""
    return InputLayer(tuple(shape), dtype=dtype, name=name).output_tensor


# ------------------------------------------------------------------ core
class Dense(Layer):
    def __init__(self, units, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", kernel_regularizer=None, input_shape=None, name=None, **kw):
        super().__init__(name=name, input_shape=input_shape, **kw)
        self.units = int(units)
        self.softmax = activation == "softmax"
        if self.softmax:
            self.activation = ActiMode.AC_MODE_NONE
        else:
            self.activation = _ACT[activation] if not isinstance(activation, ActiMode) else activation
        self.use_bias = use_bias
        self.kernel_initializer = kinit.get(kernel_initializer)
        self.bias_initializer = kinit.get(bias_initializer)
        self.kernel_regularizer = kreg.get(kernel_regularizer)

    def compute_output_shape(self, in_shapes):
        return [in_shapes[0][:-1] + (self.units,)]

    def _lower(self, ff, xs):
        t = ff.dense(xs[0], self.units, self.activation, self.use_bias, shared_op=self._shared(ff),
                     kernel_initializer=self.kernel_initializer.ff() if self.kernel_initializer else None,
                     bias_initializer=self.bias_initializer.ff() if self.bias_initializer else None,
                     kernel_regularizer=self.kernel_regularizer, name=self.name)
        self._track(ff, t)
        return [ff.softmax(t)] if self.softmax else [t]


class Flatten(Layer):
    def compute_output_shape(self, in_shapes):
        n = 1
        for s in in_shapes[0]:
            n *= s
        return [(n,)]

    def _lower(self, ff, xs):
        return [self._track(ff, ff.flat(xs[0], name=self.name))]


class Embedding(Layer):
    def __init__(self, input_dim, output_dim, embeddings_initializer="uniform", input_length=None, name=None,
                 **kw):
        super().__init__(name=name, **kw)
        self.input_dim, self.output_dim = int(input_dim), int(output_dim)
        self.initializer = kinit.get(embeddings_initializer)
        self.input_length = input_length

    def compute_output_shape(self, in_shapes):
        return [in_shapes[0] + (self.output_dim,) if in_shapes[0] != (1,) else (self.output_dim,)]

    def output_dtypes(self, in_dtypes):
        return [DataType.DT_FLOAT]

    def _lower(self, ff, xs):
        x = xs[0]
        if tuple(x.dims[1:]) == (1,):
            t = ff.embedding(x, self.input_dim, self.output_dim, AggrMode.AGGR_MODE_SUM,
                             kernel_initializer=self.initializer.ff() if self.initializer else None, name=self.name)
        else:
            t = ff.embedding(x, self.input_dim, self.output_dim, AggrMode.AGGR_MODE_NONE,
                             kernel_initializer=self.initializer.ff() if self.initializer else None, name=self.name)
        return [self._track(ff, t)]


class Activation(Layer):
    def __init__(self, activation, name=None, **kw):
        super().__init__(name=name, **kw)
        self.activation = activation

    def _lower(self, ff, xs):
        a = self.activation
        fn = {"softmax": ff.softmax, "relu": ff.relu, "sigmoid": ff.sigmoid, "tanh": ff.tanh, "elu": ff.elu,
              "gelu": ff.gelu, "linear": ff.identity}[a]
        return [self._track(ff, fn(xs[0], name=self.name))]


class Dropout(Layer):
    def __init__(self, rate, noise_shape=None, seed=None, name=None, **kw):
        super().__init__(name=name, **kw)
        self.rate, self.seed = float(rate), int(seed or 0)

    def _lower(self, ff, xs):
        return [self._track(ff, ff.dropout(xs[0], self.rate, self.seed, name=self.name))]


class Reshape(Layer):
    def __init__(self, target_shape, name=None, **kw):
        super().__init__(name=name, **kw)
        self.target_shape = tuple(int(s) for s in target_shape)

    def compute_output_shape(self, in_shapes):
        n = 1
        for s in in_shapes[0]:
            n *= s
        tgt = list(self.target_shape)
        if -1 in tgt:
            k = 1
            for s in tgt:
                if s != -1:
                    k *= s
            tgt[tgt.index(-1)] = n // k
        return [tuple(tgt)]

    def _lower(self, ff, xs):
        shp = (xs[0].dims[0],) + self.compute_output_shape([tuple(xs[0].dims[1:])])[0]
        return [self._track(ff, ff.reshape(xs[0], shp, name=self.name))]


class Permute(Layer):
    def __init__(self, dims, name=None, **kw):
        super().__init__(name=name, **kw)
        self.dims = tuple(int(d) for d in dims)  # 1-based over non-batch dims (Keras convention)

    def compute_output_shape(self, in_shapes):
        return [tuple(in_shapes[0][d - 1] for d in self.dims)]

    def _lower(self, ff, xs):
        perm = (0,) + self.dims
        return [self._track(ff, ff.transpose(xs[0], perm, name=self.name))]


# ------------------------------------------------------------------ convolution / pooling
def _pair(v):
    return (int(v), int(v)) if isinstance(v, int) else (int(v[0]), int(v[1]))


def _pads(padding, kernel, stride=(1, 1)):
    if padding == "valid" or padding is None:
        return (0, 0)
    if padding == "same":
        return ((kernel[0] - 1) // 2, (kernel[1] - 1) // 2)
    return _pair(padding)


class Conv2D(Layer):
    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", activation=None, groups=1,
                 use_bias=True, kernel_initializer="glorot_uniform", bias_initializer="zeros",
                 kernel_regularizer=None, input_shape=None, name=None, **kw):
        super().__init__(name=name, input_shape=input_shape, **kw)
        self.filters = int(filters)
        self.kernel = _pair(kernel_size)
        self.strides = _pair(strides)
        self.pads = _pads(padding, self.kernel, self.strides)
        self.activation = _ACT[activation]
        self.groups, self.use_bias = int(groups), use_bias
        self.kernel_initializer = kinit.get(kernel_initializer)
        self.bias_initializer = kinit.get(bias_initializer)
        self.kernel_regularizer = kreg.get(kernel_regularizer)

    def compute_output_shape(self, in_shapes):
        c, h, w = in_shapes[0]
        oh = (h + 2 * self.pads[0] - self.kernel[0]) // self.strides[0] + 1
        ow = (w + 2 * self.pads[1] - self.kernel[1]) // self.strides[1] + 1
        return [(self.filters, oh, ow)]

    def _lower(self, ff, xs):
        t = ff.conv2d(xs[0], self.filters, self.kernel[0], self.kernel[1], self.strides[0], self.strides[1],
                      self.pads[0], self.pads[1], self.activation, self.groups, self.use_bias,
                      shared_op=self._shared(ff), kernel_initializer=self.kernel_initializer.ff() if self.kernel_initializer else None,
                      bias_initializer=self.bias_initializer.ff() if self.bias_initializer else None, name=self.name)
        return [self._track(ff, t)]


class Pooling2D(Layer):
    pool_type = PoolType.POOL_MAX

    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", name=None, **kw):
        super().__init__(name=name, **kw)
        self.pool = _pair(pool_size)
        self.strides = _pair(strides) if strides is not None else self.pool
        self.pads = _pads(padding, self.pool, self.strides)

    def compute_output_shape(self, in_shapes):
        c, h, w = in_shapes[0]
        oh = (h + 2 * self.pads[0] - self.pool[0]) // self.strides[0] + 1
        ow = (w + 2 * self.pads[1] - self.pool[1]) // self.strides[1] + 1
        return [(c, oh, ow)]

    def _lower(self, ff, xs):
        t = ff.pool2d(xs[0], self.pool[0], self.pool[1], self.strides[0], self.strides[1], self.pads[0],
                      self.pads[1], self.pool_type, name=self.name)
        return [self._track(ff, t)]


class MaxPooling2D(Pooling2D):
    pool_type = PoolType.POOL_MAX


class AveragePooling2D(Pooling2D):
    pool_type = PoolType.POOL_AVG


class BatchNormalization(Layer):
    def __init__(self, axis=1, momentum=0.99, epsilon=0.001, name=None, **kw):
        super().__init__(name=name, **kw)
        assert axis == 1, "channels-first batch norm (axis=1), as the reference"

    def _lower(self, ff, xs):
        return [self._track(ff, ff.batch_norm(xs[0], relu=False, name=self.name))]


class LayerNormalization(Layer):
    def __init__(self, axis=-1, epsilon=1e-5, name=None, **kw):
        super().__init__(name=name, **kw)
        self.axis = [axis] if isinstance(axis, int) else list(axis)
        self.epsilon = epsilon

    def _lower(self, ff, xs):
        return [self._track(ff, ff.layer_norm(xs[0], self.axis, True, self.epsilon, name=self.name))]


# ------------------------------------------------------------------ merge
class _Merge(Layer):
    def compute_output_shape(self, in_shapes):
        return [in_shapes[0]]


class Concatenate(_Merge):
    def __init__(self, axis=1, name=None, **kw):
        super().__init__(name=name, **kw)
        self.axis = int(axis)

    def compute_output_shape(self, in_shapes):
        ax = self.axis - 1 if self.axis > 0 else len(in_shapes[0]) + self.axis
        out = list(in_shapes[0])
        out[ax] = sum(s[ax] for s in in_shapes)
        return [tuple(out)]

    def _lower(self, ff, xs):
        ax = self.axis if self.axis >= 0 else len(xs[0].dims) + self.axis
        return [self._track(ff, ff.concat(xs, ax, name=self.name))]


class _Binary(_Merge):
    fn = "add"

    def compute_output_shape(self, in_shapes):
        import numpy as np
        return [tuple(np.broadcast_shapes(*[tuple(s) for s in in_shapes]))]

    def _lower(self, ff, xs):
        t = xs[0]
        for y in xs[1:]:
            t = getattr(ff, self.fn)(t, y)
            self.ff_layers.append(ff.get_last_layer())
        return [t]


class Add(_Binary):
    fn = "add"


class Subtract(_Binary):
    fn = "subtract"


class Multiply(_Binary):
    fn = "multiply"


class Divide(_Binary):
    fn = "divide"


class Maximum(_Binary):
    fn = "max"


class Minimum(_Binary):
    fn = "min"


def concatenate(input_tensors, axis=1):
    return Concatenate(axis=axis)(input_tensors)


def add(input_tensors):
    return Add()(input_tensors)


def subtract(input_tensors):
    return Subtract()(input_tensors)


def multiply(input_tensors):
    return Multiply()(input_tensors)


def maximum(input_tensors):
    return Maximum()(input_tensors)


def minimum(input_tensors):
    return Minimum()(input_tensors)


__all__ = ["KTensor", "Layer", "InputLayer", "Input", "Dense", "Flatten", "Embedding", "Activation", "Dropout",
           "Reshape", "Permute", "Conv2D", "Pooling2D", "MaxPooling2D", "AveragePooling2D", "BatchNormalization",
           "LayerNormalization", "Concatenate", "Add", "Subtract", "Multiply", "Maximum", "Minimum", "concatenate",
           "add", "subtract", "multiply", "maximum", "minimum"]
