"""flexflow_amd.torch — torch.fx frontend (reference python/flexflow/torch)."""
from .model import IR_DELIMITER, INOUT_NODE_DELIMITER, IRNode, PyTorchModel  # noqa: F401
