"""keras_exp Model / Sequential: Keras models compiled through ONNX (reference
python/flexflow/keras_exp/models/model.py: tf.keras model -> keras2onnx -> ONNXModelKeras ->
FFModel). `Model(inputs={key: Input(...)}, outputs=...)` takes the reference's input dict keyed by
an integer (graph inputs are named "input_<key>") or a tensor / list of tensors.

With TensorFlow installed, tf.keras models are accepted and converted by keras2onnx/tf2onnx, as
in the reference. This image has no TensorFlow, so the same graphs are written with
flexflow_amd.keras layers and exported by our keras2onnx-convention exporter (onnx_export.py);
either way the FFModel is built only from the ONNX graph, and compile/fit/evaluate are the Keras
API of flexflow_amd.keras.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from ...core import FFConfig, FFModel
from ...keras import losses as klosses
from ...keras import metrics as kmetrics
from ...keras import optimizers as kopt
from ...keras.models import Model as _KerasModel
from ...onnx.model import ONNXModelKeras
from ...type import CompMode
from ..onnx_export import export_keras_model


def _is_tf(x) -> bool:
    return type(x).__module__.split(".")[0] in ("tensorflow", "keras", "tf_keras")


def _tf_to_onnx(tf_model):  # pragma: no cover - TensorFlow is not in this image
    try:
        import keras2onnx  # type: ignore
        return keras2onnx.convert_keras(tf_model, tf_model.name).SerializeToString()
    except ImportError:
        try:
            import tf2onnx  # type: ignore
            proto, _ = tf2onnx.convert.from_keras(tf_model)
            return proto.SerializeToString()
        except ImportError as e:
            raise ImportError("keras_exp with a tf.keras model needs keras2onnx or tf2onnx") from e


class Model(_KerasModel):
    def __init__(self, inputs=None, outputs=None, name=None, onnx_model=None):
        if isinstance(inputs, dict):
            keys = list(inputs.keys())
            ins = [inputs[k] for k in keys]
        else:
            ins = list(inputs) if isinstance(inputs, (list, tuple)) else ([inputs] if inputs is not None else [])
            keys = list(range(1, len(ins) + 1))
        self._tf_model = None
        if ins and _is_tf(ins[0]):  # pragma: no cover - TensorFlow is not in this image
            import tensorflow as tf  # type: ignore
            self._tf_model = tf.keras.Model(inputs=ins, outputs=outputs)
            onnx_model = _tf_to_onnx(self._tf_model)
            ins, outputs = [], None
        super().__init__(ins, outputs, name=name or "keras_exp_model")
        self._input_keys = keys
        self._onnx_bytes = onnx_model
        self._my_onnx_model = None

    @property
    def onnx_model(self) -> Optional[bytes]:
        return self._onnx_bytes

    def compile(self, optimizer, loss=None, metrics=None, loss_weights=None, weighted_metrics=None,
                run_eagerly=None, comp_mode=CompMode.TRAINING, batch_size=None, ffconfig=None, **kwargs):
        if loss_weights is not None or weighted_metrics is not None or run_eagerly is not None:
            raise NotImplementedError("loss_weights / weighted_metrics / run_eagerly are not supported (as the "
                                      "reference)")
        if loss is None:
            raise ValueError("loss is None")
        self._loss = klosses.get(loss)
        self._metrics = [kmetrics.get(m) for m in (metrics or [])]
        self._ffconfig = ffconfig or FFConfig()
        if batch_size is not None:
            self._ffconfig.batch_size = int(batch_size)
        bs = self._ffconfig.batch_size
        if self._onnx_bytes is None:
            self._onnx_bytes = export_keras_model(self, self._input_keys, bs, seed=self._ffconfig.seed)
        ff = FFModel(self._ffconfig)
        self._my_onnx_model = ONNXModelKeras(self._onnx_bytes, self._ffconfig, ff)
        g = self._my_onnx_model.model.graph
        self._ff_inputs = []
        feed = {}
        for vi in g.input:
            if vi.name in self._my_onnx_model.inits:
                continue
            dims = [bs] + [int(d) for d in list(vi.shape)[1:]]
            t = ff.create_tensor(dims, self._input_dtype(vi), name=vi.name)
            feed[vi.name] = t
            self._ff_inputs.append(t)
        self._ff_output = self._my_onnx_model.apply(ff, feed)
        self._optimizer = kopt.get(optimizer)
        ff.optimizer = self._optimizer.create_ffhandle(ff)
        ff.compile(loss_type=self._loss.type, metrics=[m.type for m in self._metrics], comp_mode=comp_mode)
        self._my_onnx_model.load_initializers(ff)
        self._ffmodel = ff

    @staticmethod
    def _input_dtype(vi):
        from ...type import DataType
        elem = getattr(vi, "elem_type", 1) or 1
        return {1: DataType.DT_FLOAT, 6: DataType.DT_INT32, 7: DataType.DT_INT64}.get(int(elem), DataType.DT_FLOAT)

    def get_weights(self, ffmodel=None):
        m = ffmodel or self._ffmodel
        return [np.asarray(w.get_weights(m)) for L in m.layers for w in L.weights]


class Sequential(Model):
    """keras_exp Sequential: layers stacked on one input, exported and compiled like Model."""

    def __init__(self, layers=None, name=None):
        from ...keras.layers import Input
        self._pending = list(layers or [])
        super().__init__(None, None, name=name or "keras_exp_sequential")
        for L in list(self._pending):
            self.add(L)
        self._pending = []
        self._Input = Input

    def add(self, layer):
        from ...keras.layers import Input
        if not self._inputs:
            if layer.input_shape is None:
                raise ValueError("the first layer of a Sequential model needs input_shape")
            self._inputs = [Input(shape=layer.input_shape)]
            self._input_keys = [1]
            self._outputs = [layer(self._inputs[0])]
        else:
            self._outputs = [layer(self._outputs[0])]
        self._onnx_bytes = None
