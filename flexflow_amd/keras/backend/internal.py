"""reference python/flexflow/keras/backend/internal.py: backend ops used as layers."""
from . import gather, rsqrt, sum  # noqa: F401,A004

__all__ = ["gather", "rsqrt", "sum"]
