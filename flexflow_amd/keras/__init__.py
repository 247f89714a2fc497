"""flexflow_amd.keras — the Keras-style frontend of the reference (python/flexflow/keras), lowered
onto FFModel (and from there onto the searched parallel strategy and the HIP kernels)."""
from . import backend, callbacks, datasets, initializers, layers, losses, metrics, models, optimizers  # noqa: F401
from . import preprocessing, regularizers, utils  # noqa: F401
