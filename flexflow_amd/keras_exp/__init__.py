"""keras_exp: Keras models compiled through ONNX (reference python/flexflow/keras_exp)."""
from . import models  # noqa: F401
from .onnx_export import export_keras_model  # noqa: F401
