from .model import Model, Sequential  # noqa: F401
from .tensor import Tensor  # noqa: F401
