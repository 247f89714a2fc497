"""flexflow_amd — an MI355X-native auto-parallelizing training framework with the capabilities of
FlexFlow (Unity): FFModel / Keras / torch.fx / ONNX frontends, PCG + Unity/MCMC search over
data/operator/attribute/parameter parallelism against an MI355X cost model, RCCL collectives over
xGMI, and hand-written gfx950 HIP kernels for the hot ops.
"""
__version__ = "0.1.0"

from .config import FFConfig  # noqa: F401
from .type import *  # noqa: F401,F403
