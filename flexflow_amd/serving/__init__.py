"""Inference serving: a Triton-protocol HTTP server over a model repository of ONNX models with
optional partitioning strategies (the reference's `triton/` Legion backend prototype, rebuilt on
our ONNX frontend, executor and a native dynamic batcher). See server.py for the endpoints.

    python -m flexflow_amd.serving --model-repository DIR [--http-port 8000] [FFConfig flags]
"""
from .client import InferenceServerClient, InferInput, InferRequestedOutput, InferResult  # noqa: F401
from .config import ModelConfig, TensorSpec, parse_pbtxt  # noqa: F401
from .engine import DynamicBatcher, InferError, ServedModel  # noqa: F401
from .repository import ModelRepository  # noqa: F401
from .server import InferenceServer  # noqa: F401
