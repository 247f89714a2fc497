"""`from flexflow_amd.core import *` — the FlexFlow Python API surface (reference
python/flexflow/core/__init__.py + flexflow_cffi.py)."""
from ..config import FFConfig, FFIterationConfig  # noqa: F401
from ..type import *  # noqa: F401,F403
from .dataloader import SingleDataLoader  # noqa: F401
from .initializers import (ConstantInitializer, GlorotUniformInitializer, Initializer,  # noqa: F401
                           NormInitializer, UniformInitializer, ZeroInitializer)
from .layer import Layer  # noqa: F401
from .model import FFModel, PerfMetrics  # noqa: F401
from .netconfig import DLRMConfig, NetConfig  # noqa: F401
from .optimizers import AdamOptimizer, Optimizer, SGDOptimizer  # noqa: F401
from .tensor import Parameter, Tensor  # noqa: F401

Op = Layer
