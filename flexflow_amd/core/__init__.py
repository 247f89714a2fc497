"""`from flexflow_amd.core import *` — the FlexFlow Python API surface (reference
python/flexflow/core/__init__.py + flexflow_cffi.py)."""
from ..config import FFConfig, FFIterationConfig  # noqa: F401
from ..type import *  # noqa: F401,F403
from .dataloader import SingleDataLoader  # noqa: F401
from .initializers import (ConstantInitializer, GlorotUniformInitializer, Initializer,  # noqa: F401
                           NormInitializer, UniformInitializer, ZeroInitializer)
from .layer import OP_CLASSES, Layer  # noqa: F401
from .layer import op_class as _op_class

for _c in OP_CLASSES.values():  # reference per-op layer classes: Linear, Conv2D, Exp, ...
    globals()[_c.__name__] = _c
Batch_Norm = _op_class(OperatorType.OP_BATCHNORM)
from .model import FFModel, PerfMetrics  # noqa: F401
from .netconfig import DLRMConfig, NetConfig  # noqa: F401
from .optimizers import AdamOptimizer, Optimizer, SGDOptimizer  # noqa: F401
from .tensor import Parameter, RegionNdarray, Tensor  # noqa: F401

Op = Layer
